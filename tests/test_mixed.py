"""Mixed engine: per-env scenario dispatch with per-env human counts in ONE engine (cn_create_mixed,
SURVEY §8d C5; reference: the per-reset scenario choice crowd_sim_dict.py:110-125 and the side-preference
scenarios' own geometry crowd_sim.py:334-357,642-651).

CPU: the oracle's mixed engine (oracle/cpu_ref.py:RefMixedEngine) is pinned against the plain oracle
engine: splitting the envs of one configuration into two groups by scenario must reproduce the plain
engine bit for bit (seeds and round-robin scenarios follow the global env index, outputs land on the
env's own row). GPU: the HIP mixed engine against the oracle's on the C5 workload (teacher-forced, the
same bar as tests/test_gpu_parity.py), and split == plain on the device."""
import os
import sys

import numpy as np
import pytest

from crowdnav_dsrnn_amd import abi
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config, make_mixed_cn_configs
from tests import helpers as H

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (C5 workload definition)

TRAFFIC = ["parallel_traffic", "perpendicular_traffic"]


def _traffic_cfg(N=5):
    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.action_space.kinematics = "holonomic"
    c.sim.train_val_sim = c.sim.test_sim = list(TRAFFIC)
    return c


def _split_vs_plain(make_plain, make_mixed, E, steps, exact=True):
    """plain engine over `TRAFFIC` vs a mixed engine whose two groups (one per scenario) carry equal
    configurations: identical outputs and per-env states."""
    c = _traffic_cfg()
    plain = make_plain(make_cn_config(c, num_envs=E, env_offset=3, nenv=E + 7, phase="train"))
    c2 = clone_config(c)
    cfgs, eg = make_mixed_cn_configs({TRAFFIC[0]: c, TRAFFIC[1]: c2}, TRAFFIC, E, env_offset=3, nenv=E + 7,
                                     phase="train")
    assert len(cfgs) == 2 and np.array_equal(eg, (3 + np.arange(E)) % 2)
    mixed = make_mixed(cfgs, eg)
    o1, o2 = plain.reset(), mixed.reset()
    for k in o1:
        np.testing.assert_array_equal(o2[k], o1[k], err_msg=k)
    rng = np.random.RandomState(2)
    for t in range(steps):
        a = rng.normal(0, 0.6, (E, 2)).astype(np.float32)
        r1, r2 = plain.step(a), mixed.step(a)
        for k in r1[0]:
            np.testing.assert_array_equal(r2[0][k], r1[0][k], err_msg="%s t=%d" % (k, t))
        for j in range(1, 7):
            np.testing.assert_array_equal(np.asarray(r2[j]), np.asarray(r1[j]), err_msg="out %d t=%d" % (j, t))
    sp = plain.get_state()
    for rows, sv in mixed.get_state():
        for n, _, _ in abi.STATE_FIELDS:
            np.testing.assert_array_equal(getattr(sv, n), getattr(sp, n)[rows], err_msg=n)


def test_oracle_mixed_split_equals_plain(oracle):
    _split_vs_plain(oracle.RefEngine, oracle.RefMixedEngine, 60, 120)


def test_oracle_mixed_c5_shapes(oracle):
    """C5 on the oracle: env r runs scenario (r % 5); side_pref envs carry one human and the four padding
    slots of their spatial_edges hold the never-seen human (15, 15) relative to the robot; the
    side-preference robot starts at (0, -4)."""
    E = 40
    cfgs, eg = bench.c5_mixed(E, 0, E)
    assert [c.human_num for c in cfgs] == [5, 1]
    assert np.array_equal(eg, (np.arange(E) % 5 >= 2).astype(np.int32))
    m = oracle.RefMixedEngine(cfgs, eg)
    obs = m.reset()
    side = np.arange(E) % 5 >= 2
    for rows, sv in m.get_state():
        np.testing.assert_array_equal(sv.scenario, [abi.SCENARIO_ID[bench.C5_SCENARIOS[r % 5]] for r in rows])
    rn = obs["robot_node"][:, 0]
    np.testing.assert_array_equal(rn[side, :2], np.tile([0.0, -4.0], (side.sum(), 1)).astype(np.float32))
    rng = np.random.RandomState(0)
    for t in range(80):
        out = m.step(rng.normal(0, 0.5, (E, 2)).astype(np.float32))
        st = {int(r): (sv.r_px[k], sv.r_py[k]) for rows, sv in m.get_state() for k, r in enumerate(rows)}
        pad = out[0]["spatial_edges"][side, 1:]
        want = np.array([[15.0 - st[r][0], 15.0 - st[r][1]] for r in np.nonzero(side)[0]], np.float64)
        np.testing.assert_array_equal(pad, np.repeat(want.astype(np.float32)[:, None], 4, axis=1))
        assert np.isfinite(out[1]).all()


# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu_mixed():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine, NumpyEngine

    class NumpyMixed(NumpyEngine):
        def __init__(self, cfgs, env_group):
            self.eng = CrowdNavEngine.mixed(cfgs, env_group)
            self.E, self.N = self.eng.E, self.eng.N

    return NumpyEngine, NumpyMixed


@pytest.mark.gpu
def test_gpu_mixed_split_equals_plain(gpu_mixed):
    """Same HIP code, envs split over two group launches: bit-identical to the plain engine (free running,
    auto-resets and spawns drawn ahead included)."""
    plain, mixed = gpu_mixed
    _split_vs_plain(plain, mixed, 300, 150)


@pytest.mark.gpu
def test_gpu_mixed_c5_vs_oracle(gpu_mixed, oracle):
    """C5 mixed engine on the GPU vs the oracle's, teacher-forced over 60 steps at 500 envs: events / done
    exact, rewards / observations (padding included) / states within 1e-5; a reward may differ by exactly
    the norm-zone penalty only where the oracle puts the robot's disc within one heading ulp of a zone
    (the rule of tests/test_gpu_parity.py::_teacher_forced)."""
    _, mixed = gpu_mixed
    E = 500
    cfgs, eg = bench.c5_mixed(E, 0, E)
    ref, g = oracle.RefMixedEngine(cfgs, eg), mixed(cfgs, eg)
    o1 = ref.reset()
    g.set_state(ref.get_state())
    rng = np.random.RandomState(7)
    flips = 0
    for t in range(60):
        a = rng.normal(0, 0.8, (E, 2)).astype(np.float32)
        pre = ref.get_state()
        g.set_state(pre)
        r_out, g_out = ref.step(a), g.step(a)
        np.testing.assert_array_equal(g_out[2], r_out[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(g_out[3], r_out[3], err_msg="event t=%d" % t)
        dr = np.abs(g_out[1].astype(np.float64) - r_out[1])
        flip = np.abs(dr - abs(cfgs[0].norm_zone_penalty)) < 1e-5
        for (rows, sv) in pre:
            for k, r in enumerate(rows):
                if flip[r]:
                    f32 = bool(int(sv.flags[k]) & abi.FLAG_ROBOT_F32)
                    mg = oracle.norm_zone_margin(sv.r_px[k], sv.r_py[k], sv.r_vx[k], sv.r_vy[k], sv.r_radius[k], f32,
                                                 cfgs[0].norm_zone_lhs)
                    assert abs(mg) < (1e-6 if f32 else 1e-12), "t=%d env %d: flip %g m from the zone" % (t, r, mg)
        flips += int(flip.sum())
        keep = ~flip
        np.testing.assert_allclose(g_out[1][keep], r_out[1][keep], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in ("robot_node", "temporal_edges", "spatial_edges"):
            np.testing.assert_allclose(g_out[0][k], r_out[0][k], atol=1e-5, rtol=0, err_msg="%s t=%d" % (k, t))
        for (rows, rs), (_, gs) in zip(ref.get_state(), g.get_state()):
            d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
            d["post_mt_crc"] = H.mt_crc(rs)
            errs = H.compare_state(gs, d, "post_", tol=1e-5, where="t=%d " % t, skip=("ep_return",))
            errs += H.compare_state(gs, {"post_ep_return": d["post_ep_return"]}, "post_", tol=1e-5,
                                    env_mask=keep[rows], where="t=%d " % t)
            assert not errs, errs
        np.testing.assert_array_equal(g_out[4][:, abi.INFO_PATH_VIOLATION], r_out[4][:, abi.INFO_PATH_VIOLATION])
        np.testing.assert_array_equal(g_out[4][:, abi.INFO_SCENARIO], r_out[4][:, abi.INFO_SCENARIO])
    assert flips <= E * 60 * 0.001, flips


@pytest.mark.gpu
def test_gpu_mixed_stream_ordering():
    """The mixed engine forks its group launches off the caller's stream and joins them back: work queued on
    the caller's (non-default) stream right after cn_step sees every group's outputs, with no device-wide
    synchronisation in between (compared with the same engine stepped and synchronised step by step)."""
    import torch

    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    E = 1000
    cfgs, eg = bench.c5_mixed(E, 0, E)
    a, b = CrowdNavEngine.mixed(cfgs, eg), CrowdNavEngine.mixed(cfgs, eg)
    g = torch.Generator(device="cuda").manual_seed(3)
    acts = torch.randn((30, E, 2), generator=g, device="cuda") * 0.5
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a.reset()
        snaps = []
        for t in range(30):
            obs, rew, done = a.step(acts[t])[:3]
            snaps.append((obs["spatial_edges"].clone(), rew.clone(), done.clone()))   # queued on s after the join
    b.reset()
    torch.cuda.synchronize()
    for t in range(30):
        obs, rew, done = b.step(acts[t])[:3]
        torch.cuda.synchronize()
        s.synchronize()
        assert torch.equal(snaps[t][0], obs["spatial_edges"]) and torch.equal(snaps[t][1], rew), t
        assert torch.equal(snaps[t][2], done), t
