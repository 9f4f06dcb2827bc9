"""Norm-zone predicate: the robot disc as GEOS's 64-gon (Point.buffer(r)) intersecting a zone quad
(crowd_sim.py norm-zone penalty; shapely semantics restated per SURVEY §9-6/9-7, parity vs GEOS unpinned).

The oracle (oracle/cpu_ref.c:disc_quad_intersect) runs the separating-axis test over all 68 edge normals
with all 64 vertices per axis. The step kernel classifies by centre distance away from the polygon's
boundary band and runs a windowed separating-axis test inside it; both must give the oracle's boolean on
every case, including centres placed within 1e-3 r of the band and rectangles at every angle."""
import ctypes

import numpy as np
import pytest

from oracle import cpu_ref


def _oracle(px, py, r, qx, qy):
    L = cpu_ref.lib()
    L.cnref_disc_quad.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 6
    out = np.zeros(len(px), np.int32)
    args = [np.ascontiguousarray(a, np.float64) for a in (px, py, r, qx, qy)]
    L.cnref_disc_quad(len(px), *[a.ctypes.data_as(ctypes.c_void_p) for a in args], out.ctypes.data_as(ctypes.c_void_p))
    return out


def _rects(rng, n):
    """Rotated rectangles shaped like the zones (width 2 r 1.5, length 1.8) at random centres / angles."""
    w = rng.uniform(0.5, 1.6, n)
    ln = np.full(n, 1.8)
    th = rng.uniform(-np.pi, np.pi, n)
    cx, cy = rng.uniform(-5, 5, n), rng.uniform(-5, 5, n)
    bx = np.stack([w / 2, w / 2, -w / 2, -w / 2], 1)
    by = np.stack([-ln / 2, ln / 2, ln / 2, -ln / 2], 1)
    c, s = np.cos(th)[:, None], np.sin(th)[:, None]
    return c * bx - s * by + cx[:, None], s * bx + c * by + cy[:, None]


def _cases(n=60000, seed=0):
    """Half uniform around the quad, half with the centre at distance ~r (the 64-gon's boundary band) from
    a random boundary point, along that edge's outward normal or towards a corner."""
    rng = np.random.RandomState(seed)
    qx, qy = _rects(rng, n)
    r = rng.uniform(0.2, 0.5, n)
    cx, cy = qx.mean(1), qy.mean(1)
    px = cx + rng.uniform(-2.5, 2.5, n)
    py = cy + rng.uniform(-2.5, 2.5, n)
    h = n // 2
    k = rng.randint(0, 4, h)
    t = rng.uniform(-0.1, 1.1, h)
    i = np.arange(h)
    x0, y0 = qx[i, k], qy[i, k]
    x1, y1 = qx[i, (k + 1) % 4], qy[i, (k + 1) % 4]
    bx, by = x0 + np.clip(t, 0, 1) * (x1 - x0), y0 + np.clip(t, 0, 1) * (y1 - y0)
    ox, oy = bx - cx[:h], by - cy[:h]
    on = np.hypot(ox, oy)
    d = r[:h] * rng.uniform(np.cos(np.pi / 64) - 1e-3, 1 + 1e-3, h)
    px[:h] = bx + ox / on * d
    py[:h] = by + oy / on * d
    return px, py, r, qx, qy


def _zone_cases(n=40000, seed=1):
    """The norm zones' own geometry (crowd_sim.py norm-zone penalty; cn_engine.hip:norm_zone): a rectangle
    whose corner sits ON the robot's circle at the heading (perturbed radially by up to +-1e-3 r, and
    exactly on it for a quarter of the cases), extending sideways (either side, width 3 r) and forwards
    (1.8 m) -- the configuration where the 64-gon's vertices decide the answer."""
    rng = np.random.RandomState(seed)
    r = rng.uniform(0.2, 0.5, n)
    px, py = rng.uniform(-5, 5, n), rng.uniform(-5, 5, n)
    h = rng.uniform(-np.pi, np.pi, n)
    eps = rng.uniform(-1e-3, 1e-3, n) * r
    eps[: n // 4] = 0.0
    cx, cy = px + (r + eps) * np.cos(h), py + (r + eps) * np.sin(h)
    side = np.where(rng.rand(n) < 0.5, 1.0, -1.0)
    tx, ty = -np.sin(h) * side, np.cos(h) * side        # tangent (either side)
    fx, fy = np.cos(h), np.sin(h)                       # forward
    w, ln = 3 * r, 1.8
    qx = np.stack([cx, cx + w * tx, cx + w * tx + ln * fx, cx + ln * fx], 1)
    qy = np.stack([cy, cy + w * ty, cy + w * ty + ln * fy, cy + ln * fy], 1)
    return px, py, r, qx, qy


def test_oracle_known_answers():
    sq_x = np.array([[1.0, 1.0, -1.0, -1.0]])
    sq_y = np.array([[-1.0, 1.0, 1.0, -1.0]])
    one = lambda x, y, r: int(_oracle(np.array([x]), np.array([y]), np.array([r]), sq_x, sq_y)[0])  # noqa: E731
    assert one(0, 0, 0.3) == 1              # centre inside
    assert one(1.5, 0, 0.3) == 0            # 0.5 from the edge
    assert one(1.29, 0, 0.3) == 1           # vertex 0 (angle 0) reaches x = 1.29 + 0.3
    assert one(1.3001, 0, 0.3) == 0
    d = 0.3 * np.cos(np.pi / 64)            # the 64-gon reaches only r cos(pi/64) towards a vertex gap...
    assert one(0, 1 + d - 1e-7, 0.3) == 1   # ...but has a vertex straight down (angle -pi/2 = vertex 16)
    assert one(1 + 0.3 / np.sqrt(2) - 1e-7, 1 + 0.3 / np.sqrt(2) - 1e-7, 0.3) == 1   # vertex 56 towards the corner
    assert one(1 + 0.3 / np.sqrt(2) + 1e-7, 1 + 0.3 / np.sqrt(2) + 1e-7, 0.3) == 0


@pytest.mark.gpu
def test_gpu_predicate_equals_oracle():
    import torch

    from crowdnav_dsrnn_amd import _lib

    a, b = _cases(), _zone_cases()
    px, py, r, qx, qy = (np.concatenate([u, v]) for u, v in zip(a, b))
    want = _oracle(px, py, r, qx, qy)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev) for a in (px, py, r, qx, qy)]
    L = _lib.lib()
    for mode in (0, 1):
        out = torch.zeros(len(px), dtype=torch.int32, device=dev)
        _lib.check(L.cn_debug_disc_quad(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), len(px), mode,
                                        *[a.data_ptr() for a in t], out.data_ptr()))
        got = out.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (mode, len(bad), bad[:5])
    assert 0.2 < want.mean() < 0.8   # both outcomes well represented
    zw = _oracle(*_zone_cases())
    assert 0.05 < zw.mean() < 0.95, zw.mean()   # the corner-on-circle cases split both ways too


@pytest.mark.gpu
def test_gpu_norm_zone_penalty_predicate_equals_oracle():
    """The step kernel's whole norm-zone predicate (cn_debug_disc_quad mode 2: both zones built around the robot,
    crowd_sim.py:918-926, the heading's trigonometry shared by the two zones and the quad edges' extreme 64-gon
    vertices taken from the heading) against the oracle's (oracle/cpu_ref.c:cnref_norm_zone_violation) on 200 k
    robot states, float32 and float64 headings, both side preferences. The zones' corner lies on the robot's
    circle by construction, so the heading's last ulp can decide: a disagreement is accepted only
    where the oracle's separating-axis margin is within what one heading ulp moves a zone corner (1e-6 m f32,
    1e-12 m f64), as in the teacher-forced C5 test."""
    import torch

    from crowdnav_dsrnn_amd import _lib

    L = cpu_ref.lib()
    L.cnref_norm_zone_violation.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 6 + [ctypes.c_int32, ctypes.c_void_p]
    L.cnref_norm_zone_margin.argtypes = [ctypes.c_double] * 5 + [ctypes.c_int, ctypes.c_int]
    L.cnref_norm_zone_margin.restype = ctypes.c_double
    rng = np.random.RandomState(7)
    n = 100000
    dev = torch.device("cuda:0")
    flips = 0
    for lhs in (0, 1):
        px, py = rng.uniform(-6, 6, n), rng.uniform(-6, 6, n)
        sp = rng.uniform(0, 1.2, n)
        sp[: n // 50] = 0.0                      # standing robots: heading atan2(0, 0)
        h = rng.uniform(-np.pi, np.pi, n)
        h[n // 50: n // 10] = np.round(h[n // 50: n // 10] / (np.pi / 32)) * (np.pi / 32)   # on 64-gon axes
        vx, vy = sp * np.cos(h), sp * np.sin(h)
        r = rng.uniform(0.2, 0.5, n)
        f32 = (rng.rand(n) < 0.5).astype(np.int32)
        want = np.zeros(n, np.int32)
        args = [np.ascontiguousarray(a, np.float64) for a in (px, py, vx, vy, r)]
        L.cnref_norm_zone_violation(n, *[a.ctypes.data_as(ctypes.c_void_p) for a in args],
                                    f32.ctypes.data_as(ctypes.c_void_p), lhs, want.ctypes.data_as(ctypes.c_void_p))
        qx = np.zeros((n, 4)); qy = np.zeros((n, 4))
        qx[:, 0], qy[:, 0], qx[:, 1], qy[:, 1] = vx, vy, f32, lhs
        t = [torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(dev) for a in (px, py, r, qx, qy)]
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        _lib.check(_lib.lib().cn_debug_disc_quad(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), n, 2,
                                                 *[a.data_ptr() for a in t], out.data_ptr()))
        got = out.cpu().numpy()
        for i in np.nonzero(got != want)[0]:
            m = L.cnref_norm_zone_margin(px[i], py[i], vx[i], vy[i], r[i], int(f32[i]), lhs)
            assert abs(m) < (1e-6 if f32[i] else 1e-12), (lhs, i, m, got[i], want[i])
            flips += 1
        assert want.sum() > 100 and (want == 0).sum() > 100, want.mean()   # (true mostly on the 64-gon's axes)
    assert flips <= 2 * n * 0.02, flips   # the on-axis headings (8 %) sit on the boundary by construction
