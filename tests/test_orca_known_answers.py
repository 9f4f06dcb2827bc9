"""ORCA / RVO2 v2.0 known-answer tests.

RVO2 (Python-RVO2, git master, unpinned; setup/full_setup.sh:40-44) is third-party and absent here, so
ORCA's arithmetic is pinned by hand-derived answers rather than by the reference. Each case below is a
one-simulator configuration as crowd_nav/policy/orca.py:92-136 builds it (agent 0 = the human being
moved, agents 1.. = its observed neighbours, pref velocity set on agent 0 only, doStep, then
getAgentVelocity(0)), and its answer is derived in closed form from Appendix A (the derivation is in
each case's comment). Three restatements are checked against the same answers:

  * the HIP step kernel's own quad-path functions (orca_lines_quad, lp2_q, lp3_q) through
    cn_debug_orca (GPU),
  * oracle/cpu_ref.c:cnref_rvo2_agent0 (CPU),
  * oracle/shims/rvo2.py's PyRVOSimulator (CPU; it generated the roll_*_orca fixtures).

Tolerance: 2e-6 absolute on velocities of magnitude <= 2 (RVO2 computes in float32: a handful of ulps
of 1.2e-7 relative; the inputs themselves are float32 roundings of the decimal positions). The line
index linearProgram2 failed at (which selects linearProgram3) must match exactly. Branches covered:
no neighbours / out of range, cut-off circle, left leg, right leg, overlapping pair (invTimeStep, with
dt = 0.25 and 0.1), linearProgram1's |den| <= eps branch both ways (parallel: num >= 0 continues,
antiparallel: num < 0 fails), linearProgram3 with an infeasible single line, with the antiparallel
midpoint projection, with the same-direction skip, and the boxed-in agent.
"""
import ctypes
import math
import sys
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 2e-6
S15 = math.sqrt(15.0)


def _one_line(point, d, pref, vmax):
    """linearProgram2 over ONE line (Appendix A.3): pref clamped to vmax; if it violates the line,
    linearProgram1 projects it onto the line inside the speed circle."""
    px, py = pref
    if px * px + py * py > vmax * vmax:
        n = math.hypot(px, py)
        px, py = px / n * vmax, py / n * vmax
    if d[0] * (point[1] - py) - d[1] * (point[0] - px) <= 0:
        return (px, py)
    dot = point[0] * d[0] + point[1] * d[1]
    disc = dot * dot + vmax * vmax - (point[0] ** 2 + point[1] ** 2)
    tl, tr = -dot - math.sqrt(disc), -dot + math.sqrt(disc)
    t = d[0] * (pref[0] - point[0]) + d[1] * (pref[1] - point[1])
    t = min(max(t, tl), tr)
    return (point[0] + t * d[0], point[1] + t * d[1])


def _left_leg_case():
    # self (0,0) v (1,0) r .5; other (4,0) v (-1,-0.1) r .5: R = 1, relPos (4,0), relVel (2, 0.1),
    # w = relVel - relPos/5 = (1.2, 0.1), w.relPos = 4.8 > 0 -> legs; det(relPos, w) = 0.4 > 0 -> left
    # leg: dir = (4 sqrt15, 4) / 16, u = (relVel.dir) dir - relVel, point = v + u/2
    d = (S15 / 4, 0.25)
    rv = (2.0, 0.1)
    k = rv[0] * d[0] + rv[1] * d[1]
    u = (k * d[0] - rv[0], k * d[1] - rv[1])
    point = (1 + 0.5 * u[0], 0.5 * u[1])
    return _one_line(point, d, (1.0, 0.0), 1.0)


# (name, agents [(px, py, vx, vy, radius)], vmax, pref, time_step, expected (vx, vy), expected fail_at)
CASES = [
    # A.4-1 no neighbours: pref (0.6, 0.8) inside the speed circle is returned as is
    ("no_neighbours", [(0, 0, 0, 0, 0.3)], 1.5, (0.6, 0.8), 0.25, (0.6, 0.8), 0),
    # pref (3, 4) beyond maxSpeed 1: normalize(pref) * maxSpeed
    ("pref_clamped", [(0, 0, 0, 0, 0.3)], 1.0, (3.0, 4.0), 0.25, (0.6, 0.8), 0),
    # neighbour 12 m away, beyond neighborDist 10: no line, pref returned
    ("out_of_range", [(0, 0, 1, 0, 0.3), (12, 0, 0, 0, 0.3)], 1.0, (1.0, 0.0), 0.25, (1.0, 0.0), 0),
    # A.4-2 static neighbour off the path at (0, 5): w = (1,0) - (0,5)/5 = (1,-1), w.relPos = -5 < 0 and
    # 25 > R^2 |w|^2 = 0.72 -> cut-off circle; pref (1, 0) satisfies the line (det = -0.65 < 0)
    ("cutoff_circle_far", [(0, 0, 1, 0, 0.3), (0, 5, 0, 0, 0.3)], 1.0, (1.0, 0.0), 0.25, (1.0, 0.0), 1),
    # A.4-3 head-on pair: det(relPos, w) = 0 -> right leg, dir = (-sqrt15/4, 1/4), point =
    # (15/16, -sqrt15/16); pref projects onto the line at t = 0 -> deflected to the right (y < 0)
    ("head_on_right_leg", [(0, 0, 1, 0, 0.5), (4, 0, -1, 0, 0.5)], 1.0, (1.0, 0.0), 0.25,
     (15 / 16, -S15 / 16), 1),
    ("left_leg", [(0, 0, 1, 0, 0.5), (4, 0, -1, -0.1, 0.5)], 1.0, (1.0, 0.0), 0.25, _left_leg_case(), 1),
    # A.4-4 overlapping pair, invTS = 1/dt = 4: w = -4 (0.5, 0), u = (4 - 2)(-1, 0), point (-1, 0),
    # dir (0, 1); linearProgram1 with disc = 0 -> exactly the point
    ("overlap_invTS4", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5)], 1.0, (0.0, 0.0), 0.25, (-1.0, 0.0), 1),
    # dt = 0.1: point (-2.5, 0) is beyond maxSpeed 1 (disc < 0) -> linearProgram2 fails at line 0,
    # linearProgram3 with no earlier lines: the direction-optimal (-dir.y, dir.x) * maxSpeed = (-1, 0)
    ("overlap_invTS10_lp3", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5)], 1.0, (0.0, 0.0), 0.1, (-1.0, 0.0), 0),
    # parallel lines (dir (0,1) both): line 0 x <= -1, line 1 x <= -1.6 (R = 1.4); linearProgram1 on line 1
    # meets |den| <= eps with num = 0.6 >= 0 and continues -> (-1.6, 0)
    ("parallel_continue", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5), (0.6, 0, 0, 0, 0.9)], 2.0, (0.0, 0.0), 0.25,
     (-1.6, 0.0), 2),
    # antiparallel: x <= -1 and x >= 0.8 -> |den| <= eps with num = -1.8 < 0, linearProgram2 fails at 1;
    # linearProgram3: the projected line is the midpoint (-0.1, 0) with dir (0, 1), direction-optimal
    # along (1, 0) picks tLeft -> (-0.1, -sqrt(3.99))
    ("antiparallel_lp3_midpoint", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5), (-0.6, 0, 0, 0, 0.5)], 2.0, (0.0, 0.0),
     0.25, (-0.1, -math.sqrt(3.99)), 1),
    # + a third line x >= 1 (same direction as line 1): linearProgram3 at line 2 skips line 1
    # (|det| <= eps, dir.dir > 0), projects line 0 to the midpoint (0, 0) -> (0, -2)
    ("lp3_same_direction_skip", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5), (-0.6, 0, 0, 0, 0.5),
                                 (-0.75, 0, 0, 0, 0.75)], 2.0, (0.0, 0.0), 0.25, (0.0, -2.0), 1),
    # A.4-5 boxed in by four overlapping neighbours (x <= -1, x >= 1, y <= -1, y >= 1; equal distSq, so
    # slot order): linearProgram3 minimises the largest violation, uniquely at the origin
    ("boxed_in_lp3", [(0, 0, 0, 0, 0.5), (0.5, 0, 0, 0, 0.5), (-0.5, 0, 0, 0, 0.5), (0, 0.5, 0, 0, 0.5),
                      (0, -0.5, 0, 0, 0.5)], 1.0, (0.0, 0.0), 0.25, (0.0, 0.0), 1),
]
IDS = [c[0] for c in CASES]


def _shim():
    sys.path.insert(0, os.path.join(REPO, "oracle", "shims"))
    try:
        import rvo2
    finally:
        sys.path.pop(0)
    return rvo2


def _shim_solve(agents, vmax, pref, dt):
    """orca.py:92-136's call sequence on the shim (neighborDist 10, timeHorizon 5, maxNeighbors A - 1)."""
    rvo2 = _shim()
    A = len(agents)
    sim = rvo2.PyRVOSimulator(dt, 10.0, max(A - 1, 1), 5.0, 5.0, 0.3, 1.0)
    for k, (x, y, vx, vy, r) in enumerate(agents):
        sim.addAgent((x, y), 10.0, max(A - 1, 1), 5.0, 5.0, r, vmax if k == 0 else 1.0, (vx, vy))
    sim.setAgentPrefVelocity(0, pref)
    for k in range(1, A):
        sim.setAgentPrefVelocity(k, (0, 0))
    sim.doStep()
    return sim.getAgentVelocity(0)


def _oracle_solve(agents, vmax, pref, dt):
    from oracle import cpu_ref

    a = np.asarray(agents, np.float64)
    return cpu_ref.rvo2_agent0(a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], vmax, pref, 10.0, 5.0, dt)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_known_answer(case):
    _, agents, vmax, pref, dt, want, _ = case
    got = _oracle_solve(agents, vmax, pref, dt)
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0)


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_shim_known_answer(case):
    _, agents, vmax, pref, dt, want, _ = case
    got = _shim_solve(agents, vmax, pref, dt)
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0)


def _random_sims(n, seed):
    """Random simulators of 2..10 agents packed in clusters (many overlapping / infeasible ones)."""
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        A = rng.randint(2, 11)
        spread = rng.choice([0.6, 1.5, 4.0])
        ag = np.zeros((A, 5), np.float32)
        ag[:, 0:2] = rng.uniform(-spread, spread, (A, 2))
        ag[:, 2:4] = rng.uniform(-1, 1, (A, 2))
        ag[:, 4] = rng.uniform(0.3, 0.6, A)
        if rng.rand() < 0.2:   # dummies of unseen humans: coincident at (7, 7), still
            k = rng.randint(1, A)
            ag[k:, 0:2] = 7.0
            ag[k:, 2:4] = 0.0
        vmax = np.float32(rng.uniform(0.5, 1.5))
        pref = rng.uniform(-1.2, 1.2, 2).astype(np.float32)
        dt = float(rng.choice([0.25, 0.1]))
        out.append((ag, vmax, pref, dt))
    return out


def test_shim_equals_oracle_on_random_simulators():
    """The two CPU restatements agree bit for bit (both float32, RVO2's operation order)."""
    for ag, vmax, pref, dt in _random_sims(300, 1):
        a = _oracle_solve(ag.astype(np.float64), float(vmax), pref, dt)
        b = _shim_solve([tuple(map(float, r)) for r in ag], float(vmax), tuple(map(float, pref)), dt)
        assert np.float32(a[0]) == np.float32(b[0]) and np.float32(a[1]) == np.float32(b[1]), (ag, vmax, pref, dt)


def _gpu_solve(sims, A):
    import torch

    from crowdnav_dsrnn_amd import _lib

    dev = torch.device("cuda:0")
    ag = torch.from_numpy(np.stack([s[0] for s in sims]).astype(np.float32)).to(dev)
    se = torch.from_numpy(np.array([[s[1], s[2][0], s[2][1]] for s in sims], np.float32)).to(dev)
    out = torch.zeros((len(sims), 4), dtype=torch.float32, device=dev)
    dts = {s[3] for s in sims}
    assert len(dts) == 1
    L = _lib.lib()
    _lib.check(L.cn_debug_orca(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), len(sims), A,
                               ag.data_ptr(), se.data_ptr(), 10.0, 5.0, float(dts.pop()), out.data_ptr()))
    torch.cuda.synchronize(dev)
    return out.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_gpu_known_answer(case):
    _, agents, vmax, pref, dt, want, fail_at = case
    sims = [(np.asarray(agents, np.float32), np.float32(vmax), np.asarray(pref, np.float32), dt)] * 3
    got = _gpu_solve(sims, len(agents))
    np.testing.assert_allclose(got[:, :2], np.tile(want, (3, 1)), atol=TOL, rtol=0)
    assert int(got[0, 2]) == fail_at


@pytest.mark.gpu
def test_gpu_equals_oracle_on_random_simulators():
    """The kernel's quad-path LP equals the C oracle bit for bit on random dense simulators (incl. the
    linearProgram3 fallback), per agent count."""
    sims = _random_sims(4000, 2)
    n_lp3 = 0
    for A in range(2, 11):
        for dt in (0.25, 0.1):
            grp = [s for s in sims if len(s[0]) == A and s[3] == dt]
            if not grp:
                continue
            got = _gpu_solve(grp, A)
            for s, g in zip(grp, got):
                want = _oracle_solve(s[0].astype(np.float64), float(s[1]), s[2], dt)
                assert np.float32(want[0]) == g[0] and np.float32(want[1]) == g[1], (s, g, want)
                n_lp3 += int(g[2] < g[3])
    assert n_lp3 > 100   # the linearProgram3 fallback is well exercised
