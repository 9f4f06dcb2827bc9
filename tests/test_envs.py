"""VecEnv drop-in (crowdnav_dsrnn_amd.envs) against the reference's VecPyTorch / ShmemVecEnv / Monitor
contract (pytorchBaselines/a2c_ppo_acktr/envs.py:106-239, train.py:261-281,
evaluation.py:71-251), and env sharding with world-size-2 gloo on CPU."""
import os

import numpy as np
import pytest
import torch

from crowdnav_dsrnn_amd import abi, envs, info as info_mod, spaces
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config


def _config(N=5, kin="holonomic", policy="orca", scen=("circle_crossing",)):
    c = clone_config(Config())
    c.sim.human_num = N
    c.action_space.kinematics = kin
    c.humans.policy = policy
    c.sim.train_val_sim = list(scen)
    c.sim.test_sim = list(scen)
    return c


# ------------------------------------------------------------------------------------------- CPU
def test_registry_and_spaces():
    assert "CrowdSimDict-v0" in envs.registry()
    with pytest.raises(KeyError):
        envs.make_vec_envs("CrowdSim-v0", 0, 2, 0.99, None, "cpu", False, config=_config())
    obs = spaces.observation_space(7)
    assert list(obs.spaces.keys()) == ["robot_node", "temporal_edges", "spatial_edges"]
    assert [tuple(s.shape) for s in obs.spaces.values()] == [(1, 7), (1, 2), (7, 2)]
    assert all(np.dtype(s.dtype) == np.float32 for s in obs.spaces.values())
    act = spaces.action_space()
    assert act.__class__.__name__ == "Box" and tuple(act.shape) == (2,)


def test_registry_resolves_entry_points():
    """make_vec_envs builds the class the id is registered to (gym.make's "module:attr" loading)."""
    assert envs.resolve("CrowdSimDict-v0") is envs.CrowdNavVecEnv
    seen = {}

    class Probe:
        def __init__(self, config, E, seed, device, **kw):
            seen.update(E=E, seed=seed, kw=kw)

    envs.register("ProbeEnv-v0", Probe)
    try:
        envs.make_vec_envs("ProbeEnv-v0", 3, 4, 0.99, None, "cpu", False, config=_config(), shard=(1, 2))
        assert seen["E"] == 2 and seen["seed"] == 3 and seen["kw"]["env_offset"] == 2 and seen["kw"]["nenv"] == 4
    finally:
        envs._REGISTRY.pop("ProbeEnv-v0")


def test_rejects_out_of_scope_options():
    with pytest.raises(NotImplementedError):
        envs.make_vec_envs("CrowdSimDict-v0", 0, 1, 0.99, None, "cpu", False, config=_config(), ax=object())
    with pytest.raises(ValueError):
        envs.make_vec_envs("CrowdSimDict-v0", 0, 3, 0.99, None, "cpu", False, config=_config(), shard=(0, 2))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_no_gpu_fails_loudly():
    with pytest.raises(RuntimeError, match="GPU"):
        envs.make_vec_envs("CrowdSimDict-v0", 0, 4, 0.99, None, "cpu", False, config=_config())


class _FakeVenv:
    scenario_names = list(abi.SCENARIOS)

    def __init__(self, side_preference=False):
        self.side_preference = side_preference


def test_lazy_infos_match_reference_structure():
    """{'info': step_info} with calc_reward's key order (crowd_sim.py:973-1035), events as info.py
    instances, Monitor's episode {r (6 d.p.), l, t} only at episode end."""
    E = 5
    ev = np.array([abi.EV_NOTHING, abi.EV_DANGER, abi.EV_COLLISION, abi.EV_REACHGOAL, abi.EV_TIMEOUT], np.int8)
    done = np.array([0, 0, 1, 1, 1], bool)
    info = np.zeros((E, abi.INFO_K), np.float32)
    info[:, abi.INFO_AGG_NAV_TIME] = [6, 5, 4, 3, 2]
    info[:, abi.INFO_PATH_VIOLATION] = [0, 1, 2, 0, 0]
    info[:, abi.INFO_PERSONAL_VIOLATION] = [0, 1, 1, 0, 0]
    info[:, abi.INFO_JERK_COST] = [0.5, 0.25, 0, 0, 1]
    info[:, abi.INFO_DIST_TO_GOAL] = [3, 2, 1, 0.1, 4]
    info[:, abi.INFO_MIN_DIST] = [np.inf, 0.125, 0, 1, 1]
    info[:, abi.INFO_SCENARIO] = [0, 1, 2, 3, 0]
    epr = np.array([0, 0, -20.1234567, 9.87654321, 1.5])
    epl = np.array([0, 0, 12, 40, 200], np.int32)
    infos = envs._LazyInfos(_FakeVenv(), ev, done, info, epr, epl, 1.25)
    assert len(infos) == E
    keys = ["aggregate_nav_time", "path_violation", "personal_violation", "jerk_cost", "dist_to_goal",
            "speed_violation", "scenario", "event"]
    for i, d in enumerate(infos):
        assert list(d["info"].keys()) == keys
        assert d["info"]["scenario"] == abi.SCENARIOS[int(info[i, abi.INFO_SCENARIO])]
        assert ("episode" in d) == bool(done[i])
        assert "bad_transition" not in d
    cls = [info_mod.Nothing, info_mod.Danger, info_mod.Collision, info_mod.ReachGoal, info_mod.Timeout]
    for i, c in enumerate(cls):
        assert isinstance(infos[i]["info"]["event"], c)
    assert infos[1]["info"]["event"].min_dist == 0.125
    assert str(infos[4]["info"]["event"]) == "Timeout"
    assert infos[2]["episode"] == {"r": -20.123457, "l": 12, "t": 1.25}
    assert infos[3]["episode"]["r"] == 9.876543
    assert infos[0]["info"]["aggregate_nav_time"] == 6 and isinstance(infos[0]["info"]["aggregate_nav_time"], int)
    side = envs._LazyInfos(_FakeVenv(True), ev, done, info, epr, epl, 0.0)
    assert list(side[0]["info"].keys())[:4] == ["aggregate_nav_time", "path_violation", "circle_crossing", "separation"]
    assert infos[-1] is infos[4] and len(infos[1:3]) == 2


def _shard_worker(rank, world, port, E, steps, out):
    import torch.distributed as dist

    from oracle import cpu_ref

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = make_cn_config(_config(N=5), num_envs=E // world, env_offset=rank * (E // world), nenv=E)
        eng = cpu_ref.RefEngine(cfg)
        obs = eng.reset()
        rng = np.random.RandomState(0)
        acts = rng.normal(0, 0.5, (steps, E, 2)).astype(np.float32)
        trace = [obs["spatial_edges"].copy()]
        rews = []
        lo, hi = rank * (E // world), (rank + 1) * (E // world)
        for s in range(steps):
            o, r, d, ev, *_ = eng.step(acts[s, lo:hi])
            trace.append(o["spatial_edges"].copy())
            rews.append(r.copy())
        local = torch.from_numpy(np.concatenate([np.stack(trace).reshape(-1), np.stack(rews).reshape(-1)]))
        gathered = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        if rank == 0:
            np.save(out, torch.stack(gathered).numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_envs_equal_unsharded_gloo(tmp_path, oracle):
    """world_size 2: each rank steps its contiguous env block with global seeds (thisSeed = seed + global
    index, nenv = total); gathered results equal one unsharded run of all envs."""
    import socket

    import torch.multiprocessing as mp

    E, steps, world = 8, 30, 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "g.npy")
    mp.start_processes(_shard_worker, args=(world, port, E, steps, out), nprocs=world, join=True,
                       start_method="spawn")
    g = np.load(out)
    full = oracle.RefEngine(make_cn_config(_config(N=5), num_envs=E, nenv=E))
    obs = full.reset()
    acts = np.random.RandomState(0).normal(0, 0.5, (steps, E, 2)).astype(np.float32)
    trace, rews = [obs["spatial_edges"]], []
    for s_ in range(steps):
        o, r, *_ = full.step(acts[s_])
        trace.append(o["spatial_edges"])
        rews.append(r)
    trace, rews = np.stack(trace), np.stack(rews)
    h = E // world
    n_obs = (steps + 1) * h * 5 * 2
    for rk in range(world):
        got_obs = g[rk, :n_obs].reshape(steps + 1, h, 5, 2)
        got_rew = g[rk, n_obs:].reshape(steps, h)
        np.testing.assert_array_equal(got_obs, trace[:, rk * h:(rk + 1) * h])
        np.testing.assert_array_equal(got_rew, rews[:, rk * h:(rk + 1) * h])


# ------------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("kin", ["holonomic", "unicycle"])
def test_vecenv_matches_oracle(oracle, kin):
    E, N = 16, 5
    c = _config(N=N, kin=kin)
    venv = envs.make_vec_envs("CrowdSimDict-v0", c.env.seed, E, 0.99, None, "cuda:0", False, config=c)
    ref = oracle.RefEngine(make_cn_config(c, num_envs=E, nenv=E))
    o_g, o_r = venv.reset(), ref.reset()
    for k in o_r:
        assert o_g[k].device.type == "cuda" and o_g[k].dtype == torch.float32
        np.testing.assert_allclose(o_g[k].cpu().numpy(), o_r[k], atol=1e-5, rtol=0)
    rng = np.random.RandomState(3)
    scale = 0.1 if kin == "unicycle" else 0.8
    n_done = 0
    for s in range(120):
        a = rng.uniform(-scale, scale, (E, 2)).astype(np.float32)
        obs, rew, done, infos = venv.step(torch.from_numpy(a).to("cuda:0"))
        r_obs, r_rew, r_done, r_ev, r_info, r_epr, r_epl = ref.step(a)
        assert rew.shape == (E, 1) and rew.dtype == torch.float32 and rew.device.type == "cpu"
        assert isinstance(done, np.ndarray) and done.dtype == bool
        np.testing.assert_array_equal(done, r_done)
        np.testing.assert_allclose(rew.numpy()[:, 0], r_rew, atol=1e-5, rtol=0)
        for k in r_obs:
            np.testing.assert_allclose(obs[k].cpu().numpy(), r_obs[k], atol=1e-5, rtol=0)
        for i, inf in enumerate(infos):
            want = info_mod.make_event(int(r_ev[i]), r_info[i, abi.INFO_MIN_DIST])
            assert type(inf["info"]["event"]) is type(want)
            if done[i]:
                n_done += 1
                assert inf["episode"]["l"] == int(r_epl[i])
                assert abs(inf["episode"]["r"] - round(float(r_epr[i]), 6)) < 1e-5
    assert n_done > 0
    venv.close()


@pytest.mark.gpu
def test_single_env_eval_attributes():
    """1-env eval path: phase 'test', venv.envs[0].env.{global_time,time_step,time_limit,robot.*}."""
    c = _config(N=5)
    venv = envs.make_vec_envs("CrowdSimDict-v0", c.env.seed, 1, None, None, "cuda:0", True, config=c)
    base_env = venv.venv.envs[0].env
    assert base_env.phase == "test" and base_env.nenv == 1 and base_env.thisSeed == c.env.seed
    venv.reset()
    assert base_env.global_time == 0.0
    assert base_env.time_step == c.env.time_step and base_env.time_limit == c.env.time_limit
    assert base_env.robot.v_pref == c.robot.v_pref and base_env.robot.time_step == c.env.time_step
    for s in range(3):
        _, _, done, _ = venv.step(torch.zeros((1, 2)))
        if not done[0]:
            assert abs(base_env.global_time - (s + 1) * c.env.time_step) < 1e-12
    venv.reset()  # allow_early_resets=True
    venv.close()


@pytest.mark.gpu
def test_sharded_gpu_equals_unsharded():
    E, N = 32, 5
    c = _config(N=N)
    full = envs.make_vec_envs("CrowdSimDict-v0", 0, E, 0.99, None, "cuda:0", False, config=c)
    shards = [envs.make_vec_envs("CrowdSimDict-v0", 0, E, 0.99, None, "cuda:0", False, config=c, shard=(r, 2))
              for r in range(2)]
    o_f = full.reset()
    o_s = [s.reset() for s in shards]
    for k in o_f:
        assert torch.equal(o_f[k], torch.cat([o[k] for o in o_s]))
    rng = np.random.RandomState(5)
    for _ in range(60):
        a = torch.from_numpy(rng.normal(0, 0.5, (E, 2)).astype(np.float32))
        of, rf, df, _ = full.step(a)
        outs = [s.step(a[r * 16:(r + 1) * 16]) for r, s in enumerate(shards)]
        for k in of:
            assert torch.equal(of[k], torch.cat([o[0][k] for o in outs]))
        assert torch.equal(rf, torch.cat([o[1] for o in outs]))
        assert np.array_equal(df, np.concatenate([o[2] for o in outs]))


@pytest.mark.gpu
def test_step_seq_equals_single_steps():
    """cn_step_seq (T launches issued from native code over a [T][E][2] action tensor) == T cn_step calls:
    same state blob, same outputs of the last step, bit for bit (C2-like config incl. auto-resets and goal
    changes: 64 envs x 10 humans, unicycle, 60 steps), for a plain and a mixed engine."""
    from crowdnav_dsrnn_amd.config import make_mixed_cn_configs
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    T, E = 60, 64
    c = _config(10, "unicycle")
    g = torch.Generator(device="cuda:0").manual_seed(7)
    acts = (torch.rand((T, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    c5 = {s: _config(5, "holonomic", scen=(s,)) for s in ("parallel_traffic", "perpendicular_traffic")}
    makers = [lambda: CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0"),
              lambda: CrowdNavEngine.mixed(*make_mixed_cn_configs(c5, list(c5), E, nenv=E, phase="train"),
                                           device="cuda:0")]
    for make in makers:
        outs = []
        for seq in (False, True):
            eng = make()
            eng.reset()
            if seq:
                o = eng.step_seq(acts)
            else:
                for t in range(T):
                    o = eng.step(acts[t])
            torch.cuda.synchronize()
            st = eng.get_state()
            blob = np.concatenate([v.blob.view(np.uint8).ravel() for _, v in st]) if isinstance(st, list) \
                else np.asarray(st.blob).view(np.uint8)
            outs.append([x.cpu().numpy().copy() for x in (o[0]["robot_node"], o[0]["spatial_edges"])] +
                        [x.cpu().numpy().copy() for x in o[1:]] + [blob.copy()])
            eng.close()
        for a, b in zip(*outs):
            np.testing.assert_array_equal(a, b)


def _c3_engine(E, shape="c3"):
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    c = clone_config(Config())
    c.humans.policy = "orca"
    if shape == "c3":
        c.sim.human_num = 25
        c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
    else:   # C2 (quad path)
        c.sim.human_num = 10
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.action_space.kinematics = "unicycle"
    return CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["c3", "c2"])
def test_c3_first_launches_find_their_spawns_and_runs_repeat(shape):
    """After cn_reset (C3 shape, 1024 envs x 25 humans, the kd-tree path; C2 shape, 4096 x 10, the quad path,
    whose spawning waves park too since round 6; 60 launches): the reset kernel draws every env's next two
    spawns, so no reset of the first launches draws a spawn inline; and runs from the same reset and actions
    end in the same state bit for bit, at the default spawn budget (spawns parked and resumed at run-dependent
    points) and with the spawn waves parking after every human (20 k cycles)."""
    E, T = (1024, 60) if shape == "c3" else (4096, 60)
    g = torch.Generator(device="cuda:0").manual_seed(11)
    acts = (torch.randn((T, E, 2), generator=g, device="cuda:0") * 0.5).contiguous() if shape == "c3" else \
        (torch.rand((T, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    blobs = []
    for budget in (None, None, 20000):
        eng = _c3_engine(E, shape)
        if budget is not None:
            eng.set_spawn_budget(budget)
        eng.reset()
        st0 = eng.spawn_stats()
        resets = 0
        for t in range(T):
            eng.step(acts[t])
            resets += int(eng.done.sum().item())
        st = eng.spawn_stats()
        assert resets > 0
        if budget is None:
            assert st["inline_resets"] - st0["inline_resets"] == 0, st
        blobs.append(np.asarray(eng.get_state().blob).copy())
        eng.close()
    np.testing.assert_array_equal(blobs[0], blobs[1])
    np.testing.assert_array_equal(blobs[0], blobs[2])


@pytest.mark.gpu
@pytest.mark.parametrize("shape,budget", [("c3", 300000), ("c2", 20000)])
def test_full_size_runs_repeat_bit_for_bit(shape, budget):
    """Run-to-run determinism of the spawn machinery at full size (4096 envs; C3: kd-tree path, C2: quad path),
    12 runs of 300 launches from the same reset and actions with a spawn budget that parks spawns in every
    launch: the final state (every stream, every pending-spawn-dependent episode) equal bit for bit. The pending
    slots are written and consumed by different workgroups of one launch (spawn waves, resumes, resets), so a
    handshake race shows as a departing run (round 5: 5 of 149 C3 runs before the keyed spawn lists; round 6:
    1 of 60 with an ok word that did not carry its key; tools/probe_c3_diverge2.py for the per-launch catcher)."""
    E, T, R = 4096, 300, 12
    g = torch.Generator(device="cuda:0").manual_seed(5)
    acts = (torch.randn((T, E, 2), generator=g, device="cuda:0") * 0.5).contiguous() if shape == "c3" else \
        (torch.rand((T, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    ref = None
    for r in range(R):
        eng = _c3_engine(E, shape)
        eng.set_spawn_budget(budget)
        eng.reset()
        eng.step_seq(acts)
        blob = np.asarray(eng.get_state().blob).copy()
        st = eng.spawn_stats()
        eng.close()
        assert st["parked_midway"] > 0 and st["completed_on_resume"] > 0, st
        if ref is None:
            ref = blob
        else:
            np.testing.assert_array_equal(blob, ref, err_msg="run %d departs from run 0" % r)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["c2", "c3"])
def test_graph_mode_replays_equal_eager_with_spawns_drawn_ahead(shape):
    """Graph mode (cn_set_graph_mode: the step sequence, spawn-list indices and launch ids live on the device):
    a HIP graph of 16 cn_step launches replayed 12 times equals 192 eager launches bit for bit, AND the spawns
    stay drawn ahead -- no more resets drawn inline than the eager run. The replayed launches' kernel arguments
    are those of the captured launches; a kernel reading the spawn-list pointers, the launch id or the draw-both
    flag from its arguments instead of the device-derived copy would queue the spawns into a stale list (every
    reset then drawn inline, results still equal) or accept a pending entry completed by its own launch."""
    E = 1024 if shape == "c3" else 4096
    T, R = 16, 12
    g = torch.Generator(device="cuda:0").manual_seed(3)
    acts = (torch.randn((T * R + 1, E, 2), generator=g, device="cuda:0") * 0.5).contiguous() if shape == "c3" else \
        (torch.rand((T * R + 1, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    out = []
    for graph in (False, True):
        eng = _c3_engine(E, shape)
        eng.reset()
        eng.step(acts[0])   # (one eager launch before the capture, as RolloutTrainer's warm-up does)
        st0 = eng.spawn_stats()
        if graph:
            buf = acts[1:1 + T].clone()
            eng.set_graph_mode(True)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for t in range(T):
                    eng.step(buf[t])
            eng.set_graph_mode(False)   # (recorded, not run: the device sequence is unchanged)
            eng.set_graph_mode(True)
            for r in range(R):
                buf.copy_(acts[1 + r * T:1 + (r + 1) * T])
                gr.replay()
            torch.cuda.synchronize()
            eng.set_graph_mode(False)
        else:
            for t in range(T * R):
                eng.step(acts[1 + t])
        st = eng.spawn_stats()
        out.append((np.asarray(eng.get_state().blob).copy(), st["inline_resets"] - st0["inline_resets"]))
        eng.close()
    assert out[1][1] <= out[0][1] + 2, (out[0][1], out[1][1])
    np.testing.assert_array_equal(out[0][0], out[1][0])
