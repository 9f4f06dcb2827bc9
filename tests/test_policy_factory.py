"""Agent policy plugin surface: policy_factory[name](config).predict(JointState) -> ActionXY,
crowd_nav/policy/policy_factory.py:1-17, orca.py:64-139, social_force.py:11-66, srnn.py:18-48.

CPU: the factory's names, SRNN.clip_action (in-place, like the reference), ORCA's frozen-simulator
bookkeeping (orca.py:85-115). GPU: ORCA.predict against the oracle's RVO2 restatement
(oracle/cpu_ref.c:cnref_rvo2_agent0, itself pinned by the Appendix A.4 known answers in
tests/test_orca_known_answers.py) -- exact float32; SOCIAL_FORCE.predict against the reference formula
evaluated in numpy float64 (1e-12: ocml vs glibc exp); predict_batch == one predict per agent."""
import os
import sys

import numpy as np
import pytest

from crowdnav_dsrnn_amd.config import Config, UnsupportedConfig, clone_config
from crowdnav_dsrnn_amd.policy_factory import (ActionRot, ActionXY, FullState, JointState, ObservableState,
                                               policy_factory, predict_batch)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg():
    return clone_config(Config())


def _random_state(rng, M, far=False):
    s = FullState(*rng.uniform(-4, 4, 2), *rng.uniform(-1, 1, 2), rng.uniform(0.3, 0.5), *rng.uniform(-5, 5, 2),
                  rng.uniform(0.5, 1.5), rng.uniform(0, 6.28))
    hs = [ObservableState(*(rng.uniform(-4, 4, 2) + (20 if far else 0)), *rng.uniform(-1, 1, 2),
                          rng.uniform(0.3, 0.5)) for _ in range(M)]
    return JointState(s, hs)


def test_factory_names_match_reference():
    assert set(policy_factory) == {"orca", "none", "social_force", "srnn", "convgru"}
    assert policy_factory["none"]() is None
    c = _cfg()
    assert policy_factory["orca"](c).name == "ORCA"
    assert policy_factory["social_force"](c).name == "social_force"


def test_srnn_clip_action_in_place():
    c = _cfg()
    p = policy_factory["srnn"](c)
    a = np.array([3.0, 4.0], np.float32)
    act = p.clip_action(a, 1.0)
    assert isinstance(act, ActionXY)
    np.testing.assert_allclose(a, [0.6, 0.8], rtol=1e-6)   # mutated like srnn.py:35-37
    c.action_space.kinematics = "unicycle"
    a = np.array([0.5, -0.3], np.float32)
    act = policy_factory["srnn"](c).clip_action(a, 1.0)
    assert isinstance(act, ActionRot) and np.allclose(a, [0.1, -0.1])


def test_orca_frozen_simulator_parameters():
    """orca.py:85-115: radius / max speed fixed when the simulator is created, re-created only when the
    agent count changes."""
    c = _cfg()
    p = policy_factory["orca"](c)
    rng = np.random.RandomState(0)
    st = _random_state(rng, 4)
    ag, sf = p._frame(st)
    r0 = ag[:, 4].copy()
    np.testing.assert_allclose(r0[0], np.float32(st.self_state.radius + 0.01 + c.orca.safety_space))
    assert sf[0] == np.float32(st.self_state.v_pref)
    st.self_state.radius += 1.0
    st.self_state.v_pref += 1.0
    for h in st.human_states:
        h.radius += 1.0
    ag2, sf2 = p._frame(st)
    np.testing.assert_array_equal(ag2[:, 4], r0)        # frozen
    assert sf2[0] == sf[0]
    ag3, _ = p._frame(JointState(st.self_state, st.human_states[:3]))   # agent count changed: new simulator
    np.testing.assert_allclose(ag3[0, 4], np.float32(st.self_state.radius + 0.01 + c.orca.safety_space))
    ag4, _ = p._frame(_random_state(rng, 31))            # 32 agents: the KdTree path (cn_orca_predict_kd)
    assert ag4.shape == (32, 5) and list(p.sim[3]) == list(range(32))   # a new simulator: identity agents_ order
    with pytest.raises(UnsupportedConfig):
        p._frame(_random_state(rng, 64))                 # 65 agents: beyond the predict's limit


def _sf_reference(st, c):
    """social_force.py:11-66 verbatim arithmetic (numpy float64)."""
    s = st.self_state
    dx, dy = s.gx - s.px, s.gy - s.py
    d = np.sqrt(dx ** 2 + dy ** 2)
    cvx = c.sf.KI * ((dx / d) * s.v_pref - s.vx)
    cvy = c.sf.KI * ((dy / d) * s.v_pref - s.vy)
    ix = iy = 0
    for o in st.human_states:
        ddx, ddy = s.px - o.px, s.py - o.py
        dd = np.sqrt(ddx ** 2 + ddy ** 2)
        ix += c.sf.A * np.exp((s.radius + o.radius - dd) / c.sf.B) * (ddx / dd)
        iy += c.sf.A * np.exp((s.radius + o.radius - dd) / c.sf.B) * (ddy / dd)
    nvx = s.vx + (cvx + ix) * c.env.time_step
    nvy = s.vy + (cvy + iy) * c.env.time_step
    n = np.linalg.norm([nvx, nvy])
    return (nvx / n * s.v_pref, nvy / n * s.v_pref) if n > s.v_pref else (nvx, nvy)


@pytest.mark.gpu
def test_gpu_orca_predict_equals_oracle(oracle):
    c = _cfg()
    rng = np.random.RandomState(3)
    for t in range(200):
        M = 1 + t % 9
        st = _random_state(rng, M, far=(t % 17 == 0))
        p = policy_factory["orca"](c)
        got = p.predict(st)
        ag, sf = p._frame(st)
        want = oracle.rvo2_agent0(ag[:, 0], ag[:, 1], ag[:, 2], ag[:, 3], ag[:, 4], float(sf[0]), sf[1:],
                                  c.orca.neighbor_dist, c.orca.time_horizon, c.env.time_step)
        assert (np.float32(got.vx), np.float32(got.vy)) == (want[0], want[1]), (t, got, want)


def _shim_predict(sim, st, c, ts):
    """orca.py:64-139 against oracle/shims/rvo2.py's PyRVOSimulator (the RVO2 restatement that recorded the
    ORCA fixtures; its KdTree keeps agents_ across doStep). Returns (sim, (vx, vy))."""
    sys.path.insert(0, os.path.join(REPO, "oracle", "shims"))
    import rvo2
    s, hs = st.self_state, st.human_states
    params = (c.orca.neighbor_dist, len(hs), c.orca.time_horizon, c.orca.time_horizon_obst)
    if sim is not None and sim.getNumAgents() != len(hs) + 1:
        sim = None
    if sim is None:
        sim = rvo2.PyRVOSimulator(ts, *params, s.radius, 1)
        sim.addAgent((s.px, s.py), *params, s.radius + 0.01 + c.orca.safety_space, s.v_pref, (s.vx, s.vy))
        for h in hs:
            sim.addAgent((h.px, h.py), *params, h.radius + 0.01 + c.orca.safety_space, 1, (h.vx, h.vy))
    else:
        sim.setAgentPosition(0, (s.px, s.py))
        sim.setAgentVelocity(0, (s.vx, s.vy))
        for i, h in enumerate(hs):
            sim.setAgentPosition(i + 1, (h.px, h.py))
            sim.setAgentVelocity(i + 1, (h.vx, h.vy))
    v = np.array((s.gx - s.px, s.gy - s.py))
    speed = np.linalg.norm(v)
    pref = v / speed if speed > 1 else v
    sim.setAgentPrefVelocity(0, tuple(pref))
    for i in range(len(hs)):
        sim.setAgentPrefVelocity(i + 1, (0, 0))
    sim.doStep()
    return sim, sim.getAgentVelocity(0)


def _crowded_state(rng, M):
    """A crowded simulator with ties: some humans share a position (equal distances, so the KdTree's
    visiting order decides the neighbour order) and some sit at the reference's dummy spot (7, 7)."""
    st = _random_state(rng, M)
    for k, h in enumerate(st.human_states):
        if k % 7 == 3:
            src = st.human_states[rng.randint(0, M)]
            h.px, h.py = src.px, src.py
        elif k % 11 == 5:
            h.px, h.py, h.vx, h.vy = 7.0, 7.0, 0.0, 0.0
    return st


def _kd_sequences(oracle, gpu):
    """Simulators of A = 11..32 (+ 40, 48, 64) agents, two per size, each stepped through 4 predicts on ONE
    ORCA object / shim simulator / oracle perm (the crowd moves a little between predicts, the agent count
    stays, so the simulator and its KdTree agent order persist). Per predict: oracle == shim (velocity and
    agents_ order) and, with `gpu`, the GPU plugin == both."""
    c = _cfg()
    rng = np.random.RandomState(11)
    n_sims = 0
    for A in list(range(11, 33)) + [40, 48, 64]:
        for rep in range(2):
            p = policy_factory["orca"](c)
            sim = None
            perm = np.arange(A, dtype=np.uint8)
            st = _crowded_state(rng, A - 1)
            for step in range(4):
                if gpu:
                    got = p.predict(st)
                ag, sf = p._frame(st)
                perm = perm.copy()   # cnref_rvo2_agent0 re-permutes it in place
                want = oracle.rvo2_agent0(ag[:, 0], ag[:, 1], ag[:, 2], ag[:, 3], ag[:, 4], float(sf[0]), sf[1:],
                                          c.orca.neighbor_dist, c.orca.time_horizon, c.env.time_step, perm=perm)
                sim, sv = _shim_predict(sim, st, c, c.env.time_step)
                assert (np.float32(sv[0]), np.float32(sv[1])) == (want[0], want[1]), (A, rep, step, sv, want)
                np.testing.assert_array_equal(np.array(sim.kd_agents, np.uint8), perm)
                if gpu:
                    assert (np.float32(got.vx), np.float32(got.vy)) == (want[0], want[1]), (A, rep, step, got, want)
                    np.testing.assert_array_equal(p.sim[3], perm)
                for h in st.human_states:
                    h.px += rng.uniform(-0.3, 0.3)
                    h.py += rng.uniform(-0.3, 0.3)
                st.self_state.px += 0.1
            n_sims += 1
    assert n_sims == 2 * 25


def test_orca_kdtree_oracle_equals_shim(oracle):
    """The oracle's KdTree ORCA (cpu_ref.c:kd_build / kd_query) equals the rvo2 shim over persisted-order
    predict sequences, A = 11..64 (CPU)."""
    _kd_sequences(oracle, gpu=False)


@pytest.mark.gpu
def test_gpu_orca_predict_kdtree_equals_oracle_and_shim(oracle):
    """ORCA.predict for simulators of more than 10 agents (crowd_sim.py:1121-1161 passes N-1 humans + the
    robot when visible): the GPU KdTree path (cn_orca_predict_kd) == oracle/cpu_ref.c:cnref_rvo2_agent0 ==
    the rvo2 shim, bit for bit in float32, over a sequence of predicts on ONE ORCA object per simulator (the
    KdTree agent order persists across doStep and is carried by the host object), incl. the order itself."""
    _kd_sequences(oracle, gpu=True)


@pytest.mark.gpu
def test_gpu_social_force_predict_equals_reference_formula():
    c = _cfg()
    rng = np.random.RandomState(4)
    for t in range(100):
        st = _random_state(rng, t % 12)
        got = policy_factory["social_force"](c).predict(st)
        want = _sf_reference(st, c)
        np.testing.assert_allclose([got.vx, got.vy], want, rtol=0, atol=1e-12)


@pytest.mark.gpu
def test_gpu_predict_batch_equals_single():
    c = _cfg()
    rng = np.random.RandomState(5)
    pols, states = [], []
    for k in range(64):
        pols.append(policy_factory["orca" if k % 2 else "social_force"](c))
        states.append(_random_state(rng, 1 + k % 8))
    batch = predict_batch(pols, states)
    for p, s, b in zip(pols, states, batch):
        assert p.predict(s) == b
