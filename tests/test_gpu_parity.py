"""HIP engine parity (MI355X). The GPU path is called through the C ABI (crowdnav_dsrnn_amd.engine)
and checked against (a) golden vectors recorded from the reference and (b) the CPU oracle.
Tolerances: bit-exact on events / done / flags / indices / RNG stream, 1e-5 on positions, rewards
and observations (BASELINE.json north star)."""
import glob
import os

import numpy as np
import pytest

from crowdnav_dsrnn_amd import abi
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config
from tests import helpers as H

pytestmark = pytest.mark.gpu

SPAWN = sorted(os.path.basename(p) for p in glob.glob(os.path.join(H.GOLDEN, "spawn_*.npz")))
ROLL = sorted(os.path.basename(p) for p in glob.glob(os.path.join(H.GOLDEN, "roll_*.npz")))


@pytest.fixture(scope="module")
def gpu():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    from crowdnav_dsrnn_amd.engine import NumpyEngine

    return NumpyEngine


@pytest.mark.parametrize("name", SPAWN)
def test_gpu_spawn_vs_reference(gpu, name):
    d = H.load(name)
    cfg = H.cn_config_from_meta(d)
    eng = gpu(cfg)
    for k in range(int(d["resets"])):
        eng.set_state(H.state_from(d, "k%d_pre_" % k, cfg))
        obs = eng.reset()
        errs = H.compare_state(eng.get_state(), d, "k%d_post_" % k, tol=1e-9)
        assert not errs, errs
        for key, ok in (("robot_node", "robot_node"), ("temporal", "temporal_edges"), ("spatial", "spatial_edges")):
            np.testing.assert_allclose(obs[ok].reshape(d["k%d_%s" % (k, key)].shape), d["k%d_%s" % (k, key)],
                                       atol=1e-6, rtol=0)


@pytest.mark.parametrize("name", ROLL)
def test_gpu_rollout_vs_reference(gpu, name):
    d = H.load(name)
    cfg = H.cn_config_from_meta(d)
    errs = H.run_teacher_forced(gpu(cfg), d, cfg, tol=H.POS_TOL)
    assert not errs, "\n".join(errs[:20])


def _cfg(N=10, kin="unicycle", scen="circle_crossing", policy="orca", E=256, fov=2.0, **over):
    c = clone_config(Config())
    c.sim.human_num = N
    c.action_space.kinematics = kin
    c.sim.train_val_sim = list(scen) if isinstance(scen, (list, tuple)) else [scen]
    c.sim.test_sim = c.sim.train_val_sim
    c.humans.policy = policy
    c.robot.FOV = fov
    c.humans.FOV = fov
    for k, v in over.items():   # "section__field": value
        sec, fld = k.split("__")
        setattr(getattr(c, sec), fld, v)
    if c.test.side_preference:
        c.humans.random_goal_changing = False
        c.humans.end_goal_changing = False
    return make_cn_config(c, num_envs=E)


def _teacher_forced(gpu, oracle, cfg, kin, steps=60, seed=5):
    """Norm zones: the zones are built around the robot itself, so its disc sits within
    ~1e-8 m of a zone corner in a few % of states and the -0.5 penalty then depends on the last ulp of
    the heading: the GPU's atan2f / cos (ocml), the oracle's (glibc) and the reference's (numpy's SIMD
    float32 atan2, which differs from glibc's in ~40 % of inputs) are all different roundings. An
    env-step whose reward differs by exactly the penalty is accepted ONLY if the oracle's geometric
    margin of that state (oracle/cpu_ref.c:cnref_norm_zone_margin: separating-axis gap between the
    64-gon and the nearer zone) is within what one float32-ulp heading change can move a zone corner
    (2.4e-7 rad x <= 2.4 m lever: 1e-6 m; 1e-12 m for float64 headings); every other difference fails.
    path_violation must match exactly."""
    ref = oracle.RefEngine(cfg)
    g = gpu(cfg)
    ref.reset()
    rng = np.random.RandomState(seed)
    mism = flips = 0
    for t in range(steps):
        a = (rng.uniform(-0.15, 0.15, (cfg.num_envs, 2)) if kin == "unicycle"
             else rng.normal(0, 0.8, (cfg.num_envs, 2))).astype(np.float32)
        pre = ref.get_state()
        g.set_state(pre)
        r_out = ref.step(a)
        g_out = g.step(a)
        rs, gs = ref.get_state(), g.get_state()
        np.testing.assert_array_equal(g_out[2], r_out[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(g_out[3], r_out[3], err_msg="event t=%d" % t)
        keep = np.ones(cfg.num_envs, bool)
        if cfg.norm_zones:
            dr = np.abs(g_out[1].astype(np.float64) - r_out[1])
            flip = np.abs(dr - abs(cfg.norm_zone_penalty)) < 1e-5
            for e in np.nonzero(flip)[0]:
                f32 = bool(int(pre.flags[e]) & abi.FLAG_ROBOT_F32)
                m = oracle.norm_zone_margin(pre.r_px[e], pre.r_py[e], pre.r_vx[e], pre.r_vy[e], pre.r_radius[e], f32,
                                            cfg.norm_zone_lhs)
                assert abs(m) < (1e-6 if f32 else 1e-12), "t=%d env %d: norm-zone flip %g m from the boundary" % (
                    t, e, m)
            flips += int(flip.sum())
            keep = ~flip
        np.testing.assert_allclose(g_out[1][keep], r_out[1][keep], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in ("robot_node", "temporal_edges", "spatial_edges"):
            np.testing.assert_allclose(g_out[0][k], r_out[0][k], atol=1e-5, rtol=0, err_msg="%s t=%d" % (k, t))
        d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
        d["post_mt_crc"] = H.mt_crc(rs)
        errs = H.compare_state(gs, d, "post_", tol=1e-5, where="t=%d " % t, skip=("ep_return",))
        errs += H.compare_state(gs, {"post_ep_return": d["post_ep_return"]}, "post_", tol=1e-5, env_mask=keep,
                                where="t=%d " % t)
        assert not errs, errs
        mism += int((g_out[4][:, abi.INFO_PATH_VIOLATION] != r_out[4][:, abi.INFO_PATH_VIOLATION]).sum())
    assert mism == 0, mism
    assert flips <= cfg.num_envs * steps * 0.001, flips


@pytest.mark.parametrize("name,kin,N,policy,scen,over", [
    ("c5_traffic_normzones", "holonomic", 5, "orca", ("parallel_traffic", "perpendicular_traffic"),
     {"reward__norm_zones": True}),
    ("c5_side_pref", "holonomic", 1, "orca", ("side_pref_passing", "side_pref_overtaking", "side_pref_crossing"),
     {"test__side_preference": True, "sim__circle_radius": 4}),
    ("social_metrics_sequential", "holonomic", 5, "orca",
     ("parallel_traffic", "perpendicular_traffic", "circle_crossing", "square_crossing"),
     {"test__social_metrics": True, "sim__circle_radius": 4}),
    ("robot_visible_quad", "unicycle", 9, "orca", "circle_crossing", {"robot__visible": True}),
    ("random_radii_vpref", "holonomic", 6, "orca", "circle_crossing",
     {"humans__random_radii": True, "humans__random_v_pref": True}),
    ("unicycle_sf_perp", "unicycle", 5, "social_force", "perpendicular_traffic", {}),
    ("single_human", "holonomic", 1, "orca", "circle_crossing", {}),
    ("two_humans_time_factor", "unicycle", 2, "orca", "circle_crossing", {"reward__time_factor": True}),
    ("kd_tree_max_agents", "holonomic", 31, "orca", "square_crossing",
     {"robot__visible": True, "robot__FOV": 1.0, "humans__FOV": 1.0}),
    ("kd_tree_11_agents", "unicycle", 11, "orca", "circle_crossing", {"humans__FOV": 0.5}),
    # CN_RNG_PHILOX fast mode: same draw order on both sides, so the same parity bar
    ("philox_c2", "unicycle", 10, "orca", "circle_crossing", {"env__rng": "philox"}),
    ("philox_kd_square_fov", "holonomic", 25, "orca", "square_crossing",
     {"env__rng": "philox", "robot__FOV": 1.0, "humans__FOV": 1.0}),
    ("philox_radii_vpref", "holonomic", 6, "orca", "circle_crossing",
     {"env__rng": "philox", "humans__random_radii": True, "humans__random_v_pref": True}),
    ("philox_social_metrics", "holonomic", 5, "orca",
     ("parallel_traffic", "perpendicular_traffic", "circle_crossing", "square_crossing"),
     {"env__rng": "philox", "test__social_metrics": True, "sim__circle_radius": 4}),
])
def test_gpu_vs_oracle_configs(gpu, oracle, name, kin, N, policy, scen, over):
    """Teacher-forced GPU vs oracle over the option space the reference exposes (SURVEY §8d C5 shapes,
    norm zones, side preference, social-metrics scenario order, visible robot, radius/v_pref jitter)."""
    _teacher_forced(gpu, oracle, _cfg(N, kin, scen, policy, 256, 2.0, **over), kin)


@pytest.mark.parametrize("kin,N,policy,scen,fov", [
    ("unicycle", 10, "orca", "circle_crossing", 2.0),      # C2 shape (BASELINE config 2)
    ("holonomic", 5, "orca", "circle_crossing", 2.0),      # C1 shape
    ("holonomic", 25, "orca", "square_crossing", 1.0),     # C3 shape (FOV pi, kd-tree)
    ("holonomic", 10, "social_force", "parallel_traffic", 2.0),
])
def test_gpu_vs_oracle_teacher_forced(gpu, oracle, kin, N, policy, scen, fov):
    """Same seeded inputs on both sides, 60 teacher-forced steps over 256 envs (the oracle's state is
    loaded into the GPU engine before every step; auto-resets included)."""
    cfg = _cfg(N, kin, scen, policy, 256, fov)
    ref = oracle.RefEngine(cfg)
    g = gpu(cfg)
    o_ref = ref.reset()
    g.set_state(ref.get_state())
    rng = np.random.RandomState(5)
    mism = 0
    for t in range(60):
        a = (rng.uniform(-0.15, 0.15, (cfg.num_envs, 2)) if kin == "unicycle"
             else rng.normal(0, 0.8, (cfg.num_envs, 2))).astype(np.float32)
        st = ref.get_state()
        g.set_state(st)
        r_out = ref.step(a)
        g_out = g.step(a)
        rs, gs = ref.get_state(), g.get_state()
        np.testing.assert_array_equal(g_out[2], r_out[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(g_out[3], r_out[3], err_msg="event t=%d" % t)
        np.testing.assert_allclose(g_out[1], r_out[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in ("robot_node", "temporal_edges", "spatial_edges"):
            np.testing.assert_allclose(g_out[0][k], r_out[0][k], atol=1e-5, rtol=0, err_msg="%s t=%d" % (k, t))
        d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
        d["post_mt_crc"] = H.mt_crc(rs)
        errs = H.compare_state(gs, d, "post_", tol=1e-5, where="t=%d " % t)
        assert not errs, errs
        mism += int((g_out[4][:, abi.INFO_PATH_VIOLATION] != r_out[4][:, abi.INFO_PATH_VIOLATION]).sum())
    assert mism == 0, mism


@pytest.mark.parametrize("rng,shape", [("mt19937", "c2"), ("philox", "c2"), ("mt19937", "c3")])
def test_gpu_free_running_matches_oracle_short_horizon(gpu, oracle, rng, shape):
    """Free-running (no teacher forcing) rollout: identical for the first 40 steps, auto-resets from the
    spawns the spare workgroups draw ahead included. c3 (25 humans, square_crossing, FOV pi, kd-tree path)
    also runs the spawns' binned disc test and the workgroup-cooperative crowded rejection of the spare
    workgroups (a few resets per step; teacher-forced tests redraw every spawn after set_state instead)."""
    if shape == "c3":
        cfg = _cfg(25, "holonomic", "square_crossing", E=512, fov=1.0, env__rng=rng)
    else:
        cfg = _cfg(10, "unicycle", E=512, env__rng=rng)
    ref, g = oracle.RefEngine(cfg), gpu(cfg)
    o1, o2 = ref.reset(), g.reset()
    for k in o1:
        np.testing.assert_allclose(o2[k], o1[k], atol=1e-6, rtol=0)
    rng = np.random.RandomState(11)
    for t in range(40):
        a = (rng.uniform(-0.1, 0.1, (cfg.num_envs, 2)) if shape == "c2"
             else rng.normal(0, 0.5, (cfg.num_envs, 2))).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        np.testing.assert_array_equal(r2[2], r1[2])
        np.testing.assert_array_equal(r2[3], r1[3])
        np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0)
    if shape == "c3":   # every stream (spawn draws included) at the same position, states within 1e-5
        rs, gs = ref.get_state(), g.get_state()
        d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
        d["post_mt_crc"] = H.mt_crc(rs)
        errs = H.compare_state(gs, d, "post_", tol=1e-5)
        assert not errs, errs


def _free_run_exact(ref, g, cfg, steps, kind, seed):
    """Free-running GPU vs oracle with identical actions: done / event exact, rewards 1e-5 every step."""
    rng = np.random.RandomState(seed)
    for t in range(steps):
        a = (rng.uniform(-0.1, 0.1, (cfg.num_envs, 2)) if kind == "unicycle"
             else rng.normal(0, 0.5, (cfg.num_envs, 2))).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        np.testing.assert_array_equal(r2[2], r1[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(r2[3], r1[3], err_msg="event t=%d" % t)
        np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)


def test_gpu_forced_spawn_parking_matches_oracle(gpu, oracle):
    """Resumable spawns (the kd-tree path's and, since round 6, the quad path's) under a 1-cycle budget: every
    spawning wave parks its spawn after each human (at least one human per launch), so every upcoming episode
    is drawn over ~10-25 launches through
    the park / resume machinery (stored MT block and stream position, the robot and the humans so far,
    overflow count, scenario, Philox key), and resets that find their spawn unfinished draw inline. The
    rollout must equal the oracle exactly (done / event every step, state and every stream at the end), and
    the counters must show spawns parked mid-way, resumed and completed by a resume."""
    for rngmode, shape in (("mt19937", "c3"), ("philox", "c3"), ("mt19937", "c2")):
        # 96 envs: fewer pending items than the spawning waves, so every parked spawn is resumed by the
        # next launch and completes ~25 (C3) / ~10 (C2, the quad path's parking, round 6) launches after it started
        cfg = (_cfg(25, "holonomic", "square_crossing", E=96, fov=1.0, env__rng=rngmode) if shape == "c3" else
               _cfg(10, "unicycle", E=96, env__rng=rngmode))
        ref, g = oracle.RefEngine(cfg), gpu(cfg)
        g.eng.set_spawn_budget(1)
        ref.reset()
        g.reset()
        _free_run_exact(ref, g, cfg, 200, "holonomic" if shape == "c3" else "unicycle", 17)
        rs, gs = ref.get_state(), g.get_state()
        d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
        d["post_mt_crc"] = H.mt_crc(rs)
        errs = H.compare_state(gs, d, "post_", tol=1e-5)
        assert not errs, errs
        st = g.eng.spawn_stats()
        # (cn_reset draws every env's next two spawns itself, so the spawn waves' work starts at the third: 200
        # launches instead of round 4's 100 keep the resume path's coverage floor at 50 completions)
        assert st["parked_midway"] > 1000 and st["resumed"] > 1000 and st["completed_on_resume"] > 50, (rngmode, shape, st)


@pytest.mark.parametrize("shape,budget,start,tl", [
    ("c3", None, "reset", 1), ("c3", None, "set_state", 1), ("c3", None, "set_state", 2),
    ("c3", 1, "set_state", 1), ("c3", 1, "set_state", 2),
    ("c2", None, "reset", 1), ("c2", None, "set_state", 1), ("c2", None, "set_state", 2), ("c2", 1, "set_state", 2),
])
def test_gpu_every_env_resets_every_launch(gpu, oracle, shape, budget, start, tl):
    """Spawn-key races. time_limit = 1 makes every env time out at its first step
    (crowd_sim.py:1032-1035: global_time >= time_limit - 1), so every env auto-resets in every launch
    (shmem_vec_env.py:164-168) and draws its next episode from the seed schedule (crowd_sim_dict.py:147-164);
    time_limit = 2 ends episodes after at most 4 steps, so a pending spawn waits a few launches before a reset
    consumes it. Both races key a spawn item from counters that a reset of the SAME launch rewrites: round 5's
    list path (an env resetting twice before its spawn is keyed) and the draw-both launch after cn_set_state /
    the quad path's cn_reset (PEND_BOTH: the step workgroups' inline resets advance reset_count / case_counter
    while the spawn waves key both pending slots; now keyed from cn_keysnap_kernel's snapshot). The state is
    re-loaded every 8 launches (from the oracle's), so a run holds eight draw-both launches. kd-tree path (C3
    shape; E = 1000, so an env's two items of a draw-both launch go to different spawning waves) at the default
    spawn budget and at a 1-cycle budget (E = 192, so parked spawns are resumed), quad path (C2 shape, 4096 envs;
    192 at a 1-cycle budget); 64 launches each: done / event exact and rewards 1e-5 every launch, the whole state
    and every MT19937 stream at the end."""
    E = 192 if budget == 1 else (4096 if shape == "c2" else 1000)
    if shape == "c3":
        cfg = _cfg(25, "holonomic", "square_crossing", E=E, fov=1.0, env__time_limit=tl)
    else:
        cfg = _cfg(10, "unicycle", E=E, env__time_limit=tl)
    oracle.lib().cnref_set_threads(min(16, os.cpu_count() or 1))
    ref, g = oracle.RefEngine(cfg), gpu(cfg)
    if budget is not None:
        g.eng.set_spawn_budget(budget)
    ref.reset()
    if start == "reset":
        g.reset()
    kind = "holonomic" if shape == "c3" else "unicycle"
    rng = np.random.RandomState(23)
    resets = 0
    for t in range(64):
        if start == "set_state" and t % 8 == 0:
            g.set_state(ref.get_state())
        a = (rng.uniform(-0.1, 0.1, (E, 2)) if kind == "unicycle" else rng.normal(0, 0.5, (E, 2))).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        if tl == 1:
            assert r1[2].all(), "time_limit = 1: every env ends its episode at every step (t=%d)" % t
        resets += int(r1[2].sum())
        np.testing.assert_array_equal(r2[2], r1[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(r2[3], r1[3], err_msg="event t=%d" % t)
        np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
    assert resets >= 64 * E // 6, resets   # episodes of at most 5 steps
    rs, gs = ref.get_state(), g.get_state()
    d = {"post_" + n: np.asarray(getattr(rs, n)) for n, _, _ in abi.STATE_FIELDS if n != "mt"}
    d["post_mt_crc"] = H.mt_crc(rs)
    errs = H.compare_state(gs, d, "post_", tol=1e-5)
    assert not errs, errs[:20]
    if budget == 1:
        st = g.eng.spawn_stats()
        assert st["parked_midway"] > 0, st
        if tl == 2:   # at time_limit = 1 every wave's first item is a new spawn, so parked ones are never resumed
            assert st["resumed"] > 0, st


def test_gpu_full_size_c3_free_running(gpu, oracle):
    """BASELINE config 3 at its full size (4096 envs x 25 humans, square_crossing, robot / human FOV pi,
    holonomic: the kd-tree path, the bench's --workload c3) for 400 free-running steps: the first 40 steps
    identical to the oracle, then finite outputs, done exactly where the event is terminal, Monitor lengths
    within the time limit, each env's reset count = 1 + its episodes ended, episode counts / mean return
    within 2 % of the oracle's over the 400 steps, and the spawn counters show spawns parked and resumed at
    the default 600 k-cycle budget (the crowded spawns of this workload outlast it)."""
    E = 4096
    cfg = _cfg(25, "holonomic", "square_crossing", E=E, fov=1.0)
    oracle.lib().cnref_set_threads(min(16, os.cpu_count() or 1))
    ref, g = oracle.RefEngine(cfg), gpu(cfg)
    g.eng.set_spawn_budget(600000)
    ref.reset()
    g.reset()
    rc0 = np.asarray(g.get_state().reset_count).copy()
    rng = np.random.RandomState(5)
    term = np.isin(np.arange(5), [abi.EV_COLLISION, abi.EV_REACHGOAL, abi.EV_TIMEOUT])
    n_ep, ret = [0, 0], [0.0, 0.0]
    ended = np.zeros(E, np.int64)
    tmax = int(round(cfg.time_limit / cfg.time_step)) + 1
    for t in range(400):
        a = rng.normal(0, 0.5, (E, 2)).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        if t < 40:
            np.testing.assert_array_equal(r2[2], r1[2], err_msg="done t=%d" % t)
            np.testing.assert_array_equal(r2[3], r1[3], err_msg="event t=%d" % t)
            np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in r2[0]:
            assert np.isfinite(r2[0][k]).all(), (k, t)
        assert np.isfinite(r2[1]).all()
        d = r2[2].astype(bool)
        np.testing.assert_array_equal(d, term[r2[3]], err_msg="done vs event t=%d" % t)
        assert (r2[6][d] >= 1).all() and (r2[6][d] <= tmax).all(), t
        ended += d
        for k, r in enumerate((r1, r2)):
            dd = r[2].astype(bool)
            n_ep[k] += int(dd.sum())
            ret[k] += float(r[5][dd].sum())
    np.testing.assert_array_equal(np.asarray(g.get_state().reset_count) - rc0, ended)
    assert n_ep[1] > 1000, n_ep
    assert abs(n_ep[1] - n_ep[0]) <= 0.02 * n_ep[0], n_ep
    assert abs(ret[1] / n_ep[1] - ret[0] / n_ep[0]) <= 0.02 * abs(ret[0] / n_ep[0]) + 0.05, (ret, n_ep)
    st = g.eng.spawn_stats()
    assert st["parked_midway"] > 0 and st["resumed"] > 0 and st["completed_on_resume"] > 0, st


def test_gpu_full_size_c2_free_running(gpu, oracle):
    """BASELINE config 2 at its full size (4096 envs x 10 humans, the bench workload) for 400 free-running
    steps: the first 50 steps identical to the oracle (done / event exact, rewards 1e-5; the oracle on all
    host threads), then size-independent properties over the whole run: finite outputs, done exactly
    where the event is terminal, Monitor lengths within the time limit, and episode counts / mean return
    within 2 % of the oracle's over the same 400 steps (spawn lists, pending-spawn slots and their
    counters are exercised for hundreds of launches)."""
    cfg = _cfg(10, "unicycle", E=4096)
    oracle.lib().cnref_set_threads(min(16, os.cpu_count() or 1))
    ref, g = oracle.RefEngine(cfg), gpu(cfg)
    ref.reset()
    g.reset()
    rng = np.random.RandomState(3)
    term = np.isin(np.arange(5), [abi.EV_COLLISION, abi.EV_REACHGOAL, abi.EV_TIMEOUT])
    n_ep = [0, 0]
    ret = [0.0, 0.0]
    tmax = int(round(cfg.time_limit / cfg.time_step)) + 1
    for t in range(400):
        a = rng.uniform(-0.1, 0.1, (4096, 2)).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        if t < 50:
            np.testing.assert_array_equal(r2[2], r1[2], err_msg="done t=%d" % t)
            np.testing.assert_array_equal(r2[3], r1[3], err_msg="event t=%d" % t)
            np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in r2[0]:
            assert np.isfinite(r2[0][k]).all(), (k, t)
        assert np.isfinite(r2[1]).all()
        d = r2[2].astype(bool)
        np.testing.assert_array_equal(d, term[r2[3]], err_msg="done vs event t=%d" % t)
        assert (r2[6][d] >= 1).all() and (r2[6][d] <= tmax).all(), t
        for k, r in enumerate((r1, r2)):
            dd = r[2].astype(bool)
            n_ep[k] += int(dd.sum())
            ret[k] += float(r[5][dd].sum())
    assert n_ep[1] > 1000, n_ep
    assert abs(n_ep[1] - n_ep[0]) <= 0.02 * n_ep[0], n_ep
    assert abs(ret[1] / n_ep[1] - ret[0] / n_ep[0]) <= 0.02 * abs(ret[0] / n_ep[0]) + 0.05, (ret, n_ep)


@pytest.mark.parametrize("E,N,kin,scen,fov", [
    (4099, 10, "unicycle", "circle_crossing", 2.0),    # ragged: E not a multiple of the 6 envs per workgroup
    (1, 10, "unicycle", "circle_crossing", 2.0),       # a single env (one partly filled workgroup)
    (203, 25, "holonomic", "square_crossing", 1.0),    # ragged on the kd-tree path (2 envs per workgroup)
])
def test_gpu_ragged_sizes_match_oracle(gpu, oracle, E, N, kin, scen, fov):
    """Free-running GPU == oracle for 30 steps at batch sizes that leave the last workgroup partly empty."""
    cfg = _cfg(N, kin, scen, E=E, fov=fov)
    ref, g = oracle.RefEngine(cfg), gpu(cfg)
    o1, o2 = ref.reset(), g.reset()
    for k in o1:
        np.testing.assert_allclose(o2[k], o1[k], atol=1e-6, rtol=0)
    rng = np.random.RandomState(13)
    for t in range(30):
        a = (rng.uniform(-0.1, 0.1, (E, 2)) if kin == "unicycle" else rng.normal(0, 0.5, (E, 2))).astype(np.float32)
        r1, r2 = ref.step(a), g.step(a)
        np.testing.assert_array_equal(r2[2], r1[2], err_msg="done t=%d" % t)
        np.testing.assert_array_equal(r2[3], r1[3], err_msg="event t=%d" % t)
        np.testing.assert_allclose(r2[1], r1[1], atol=1e-5, rtol=0, err_msg="reward t=%d" % t)
        for k in r1[0]:
            np.testing.assert_allclose(r2[0][k], r1[0][k], atol=1e-5, rtol=0, err_msg="%s t=%d" % (k, t))


def test_gpu_large_batch_properties(gpu):
    """A large batch (131,072 envs x 10 humans, 32x the bench's: 21,846 workgroups, spawn lists of
    thousands of entries) for 40 steps: finite outputs, done exactly on terminal events, Monitor lengths
    positive where done, every env's stream position advanced consistently with its resets."""
    E = 131072
    cfg = _cfg(10, "unicycle", E=E)
    g = gpu(cfg)
    g.reset()
    rng = np.random.RandomState(1)
    term = np.isin(np.arange(5), [abi.EV_COLLISION, abi.EV_REACHGOAL, abi.EV_TIMEOUT])
    resets = np.zeros(E, np.int64)
    for t in range(40):
        r = g.step(rng.uniform(-0.1, 0.1, (E, 2)).astype(np.float32))
        assert np.isfinite(r[1]).all() and all(np.isfinite(v).all() for v in r[0].values()), t
        d = r[2].astype(bool)
        np.testing.assert_array_equal(d, term[r[3]], err_msg="t=%d" % t)
        assert (r[6][d] >= 1).all()
        resets += d
    st = g.get_state()
    np.testing.assert_array_equal(st.reset_count.astype(np.int64), 1 + resets)   # cn_reset + auto-resets
