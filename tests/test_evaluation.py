"""Batched evaluation / social metrics (crowdnav_dsrnn_amd/evaluation.py) vs the reference's
pytorchBaselines/evaluation.py evaluate() + metrics.py.

tests/golden/eval_*.npz hold a scripted test-episode stream and what the reference's evaluate() logged and
returned for it, running the episodes one after the other in a single env (oracle/gen_golden.py gen_eval).
Here the same episodes are replayed through EpisodeRecorder as a batched VecEnv would produce them
(E envs in lockstep, env i running global episodes i, i+E, ...; episodes >= test_size run but uncounted),
then _report rebuilds the log. The log must match the reference line for line (the scenario order of the
breakdown follows Python set iteration, so those lines are compared as sets per block), and the returned
per-episode reward / distance lists must match exactly.
"""
import logging as _logging

import numpy as np
import pytest
import torch

from crowdnav_dsrnn_amd import abi
from crowdnav_dsrnn_amd.config import Config, clone_config
from crowdnav_dsrnn_amd.evaluation import EpisodeRecorder, Metrics, _report
from tests.helpers import load


class _Log:
    def __init__(self):
        self.lines = []

    def info(self, msg):
        self.lines.append(str(msg))


class _Envs:
    scenario_names = list(abi.SCENARIOS)

    def close(self):
        pass


def _episodes(z):
    off = np.concatenate([[0], np.cumsum(z["ep_len"])])
    eps = []
    for k in range(len(z["ep_len"])):
        a, b = off[k], off[k + 1]
        eps.append({"first": z["ep_first"][k], "scenario": str(z["ep_scenario"][k]),
                    "steps": {key[3:]: z[key][a:b] for key in z if key.startswith("st_")}})
    return eps


def _config(z):
    c = clone_config(Config())
    c.env.test_size = int(z["test_size"])
    c.env.time_step = float(z["time_step"])
    c.env.time_limit = float(z["time_limit"])
    c.test.social_metrics = bool(z["social_metrics"])
    c.test.side_preference = bool(z["side_preference"])
    c.sim.train_val_sim = [str(x) for x in z["train_val_sim"]]
    c.sim.test_sim = [str(x) for x in z["test_sim"]]
    return c


def _replay(z, E, env_offset=0, nenv=None, device="cpu"):
    """Feed the script to an EpisodeRecorder as E lockstep envs of a VecEnv (auto-reset semantics)."""
    eps = _episodes(z)
    c = _config(z)
    T = int(z["test_size"])
    nenv = E if nenv is None else nenv
    names = list(abi.SCENARIOS)
    side_scen = c.sim.test_sim[0] if c.test.side_preference else None
    rec = EpisodeRecorder(E, T, env_offset, nenv, device, c.env.time_step, 0.99, c.robot.v_pref,
                          c.test.side_preference, side_scen, names, keep_traces=True)
    g = [env_offset + i for i in range(E)]     # global episode index per env
    t = [0] * E

    def first_obs():
        rn = torch.zeros(E, 1, 7)
        te = torch.zeros(E, 1, 2)
        for i in range(E):
            rn[i, 0, :2] = torch.from_numpy(eps[g[i] % T]["first"])
        return {"robot_node": rn.to(device), "temporal_edges": te.to(device)}

    rec.start(first_obs())
    for _ in range(100000):
        rn = torch.zeros(E, 1, 7)
        te = torch.zeros(E, 1, 2)
        rew = torch.zeros(E)
        done = torch.zeros(E, dtype=torch.uint8)
        ev = torch.zeros(E, dtype=torch.int8)
        info = torch.zeros(E, abi.INFO_K)
        for i in range(E):
            e = eps[g[i] % T]
            s = e["steps"]
            j = t[i]
            rew[i] = float(s["reward"][j])
            ev[i] = int(s["event"][j])
            info[i, abi.INFO_AGG_NAV_TIME] = float(s["aggregate_nav_time"][j])
            info[i, abi.INFO_PATH_VIOLATION] = float(s["path_violation"][j])
            info[i, abi.INFO_PERSONAL_VIOLATION] = float(s["personal_violation"][j])
            info[i, abi.INFO_JERK_COST] = float(s["jerk_cost"][j])
            info[i, abi.INFO_DIST_TO_GOAL] = float(s["dist_to_goal"][j])
            info[i, abi.INFO_SPEED_VIOLATION] = float(s["speed_violation"][j])
            info[i, abi.INFO_MIN_DIST] = float(s["min_dist"][j])
            info[i, abi.INFO_SCENARIO] = float(names.index(e["scenario"]))
            info[i, abi.INFO_SIDE_LEFT] = float(s["left"][j])
            info[i, abi.INFO_SIDE_RIGHT] = float(s["right"][j])
            t[i] += 1
            if t[i] == len(s["reward"]):
                done[i] = 1
                t[i] = 0
                g[i] += nenv
                rn[i, 0, :2] = torch.from_numpy(eps[g[i] % T]["first"])
            else:
                rn[i, 0, :2] = torch.from_numpy(s["pos"][j])
                te[i, 0, :] = torch.from_numpy(s["vel"][j])
        obs = {"robot_node": rn.to(device), "temporal_edges": te.to(device)}
        rec.step(obs, rew.to(device), done.to(device), ev.to(device), info.to(device))
        if rec.finished():
            break
    return rec, c


def _blocks(lines):
    """Split the log into comparable units: scenario-breakdown blocks as sets, other lines verbatim."""
    out, cur = [], None
    for ln in lines:
        if ln.endswith(" CASES: "):
            cur = set()
            out.append((ln, cur))
        elif cur is not None and ln and ":" in ln and not ln.endswith("======"):
            cur.add(ln)
        else:
            cur = None
            out.append(ln)
    return out


def _check_against_golden(z, rec, c, traces=None):
    log = _Log()
    raw, disc, d2g = _report(rec.host_records(), rec.episode_traces() if traces is None else traces, c, log, int(z["test_size"]),
                             c.env.time_step, 0.99, c.test.side_preference,
                             c.sim.test_sim[0] if c.test.side_preference else None, _Envs(), verbose=False)
    want = str(z["log"]).split("\n")
    assert _blocks(log.lines) == _blocks(want)
    for tag, d in (("raw", raw), ("disc", disc), ("d2g", d2g)):
        for b, lists in d.items():
            np.testing.assert_array_equal([len(x) for x in lists], z["ret_%s_%s_len" % (tag, b)])
            got = np.array([v for x in lists for v in x], np.float64)
            np.testing.assert_allclose(got, z["ret_%s_%s" % (tag, b)], rtol=1e-12, atol=0, err_msg=tag + b)


@pytest.mark.parametrize("case", ["eval_social", "eval_sidepref"])
@pytest.mark.parametrize("E", [1, 3, 5, 40])
def test_batched_evaluation_matches_reference_log(case, E):
    z = load(case + ".npz")
    rec, c = _replay(z, E)
    _check_against_golden(z, rec, c)


def test_sharded_evaluation_records_sum_to_the_whole():
    """Two shards (env_offset 0 / 4 of nenv 8): summing their records (what host_records does with an
    all_reduce) gives the single-shard log."""
    z = load("eval_social.npz")
    r0, c = _replay(z, 4, env_offset=0, nenv=8)
    r1, _ = _replay(z, 4, env_offset=4, nenv=8)
    traces = {**r0.episode_traces(), **r1.episode_traces()}     # what evaluate() all_gathers
    for k in r0.rec:
        r0.rec[k] += r1.rec[k]
    _check_against_golden(z, r0, c, traces)


def test_metrics_formula():
    """metrics.py:13-25: mean, population std, 90% t-interval around the mean."""
    import scipy.stats

    m = Metrics(_logging.getLogger("t"))
    x = [1.0, 2.5, 4.0, 0.5, 3.0]
    m.add_metric("a", x)
    mean, std, ci = m["a"]
    assert mean == np.mean(x) and std == np.std(x)
    lo, hi = scipy.stats.t.interval(0.9, len(x) - 1, np.mean(x), scipy.stats.sem(x))
    assert ci == [lo, hi]


class _GoalSeeker:
    """Deterministic elementwise controller (holonomic: unit velocity toward the goal), so every env's
    trajectory is independent of how many envs are batched together."""

    def __init__(self, N):
        self.base = type("B", (), {"human_num": N})()

    def act(self, obs, hxs, masks, deterministic=False):
        rn = obs["robot_node"][:, 0, :]
        d = rn[:, 3:5] - rn[:, 0:2]
        n = torch.sqrt((d * d).sum(-1, keepdim=True)).clamp_min(1e-6)
        return None, d / n * 0.9, None, hxs


def _gpu_eval(E, test_size=12):
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.evaluation import evaluate

    c = clone_config(Config())
    c.sim.human_num = 5
    c.action_space.kinematics = "holonomic"
    # one scenario: the reference draws among several with the unseeded `random` module (crowd_sim_dict.py:125)
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.test.social_metrics = True
    c.env.test_size = test_size
    envs = CrowdNavVecEnv(c, E, c.env.seed, "cuda:0", allow_early_resets=True, nenv=E, phase="test")
    log = _Log()
    out = evaluate(_GoalSeeker(5), False, envs, E, "cuda:0", c, log, verbose=False)
    return log.lines, out, evaluate.last


@pytest.mark.gpu
def test_batched_evaluation_on_engine_matches_sequential():
    """evaluate() over the real engine: 1 env running the 12 test episodes one after the other (what
    test.py does) and 4 / 12 envs running them concurrently give the same per-episode records, log and
    returned lists (test seeds offset + g for global episode g, crowd_sim_dict.py:147-164)."""
    l1, o1, s1 = _gpu_eval(1)
    for E in (4, 12):
        lE, oE, sE = _gpu_eval(E)
        assert lE == l1
        for k in ("steps", "event", "scenario", "raw", "disc", "gt", "pv", "pathv", "agg", "jerk", "sv"):
            np.testing.assert_array_equal(sE["records"][k], s1["records"][k], err_msg=k)
        for k in ("path", "chc"):
            np.testing.assert_allclose(sE["records"][k], s1["records"][k], rtol=1e-6, err_msg=k)
        for a, b in zip(oE, o1):
            assert a == b
    assert sum(s1["num_events"][k]["total"] for k in s1["num_events"]) == 12


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["eval_social", "eval_sidepref"])
@pytest.mark.parametrize("E", [1, 7, 40])
def test_device_evaluation_matches_reference_log(case, E):
    """EpisodeRecorder with its running sums on the GPU (the evaluate() path on a cuda VecEnv): the
    reference's evaluate() log and returned lists (tests/golden/eval_*.npz, evaluation.py:96-330,
    metrics.py:5-44) reproduced from device-side records, batched over E envs."""
    z = load(case + ".npz")
    rec, c = _replay(z, E, device="cuda:0")
    assert all(v.device.type == "cuda" for v in rec.rec.values())
    _check_against_golden(z, rec, c)
