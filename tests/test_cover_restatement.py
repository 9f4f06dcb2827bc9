"""CPU check of the candidate-box cover's arithmetic (GoalCover in csrc/cn_engine.hip: goal_cover_build /
goal_cover_hit), restated in numpy float32 exactly as the kernel computes it, on crowded square_crossing states
of the oracle: a cell marked covered must never hold a try the exact test (norm < min_dist) accepts, and
arow[iy] & acol[ix] must hold every agent whose disc holds the try. The kernel's results are pinned by the GPU
parity suite; this pins the margins argument the cover relies on."""
import numpy as np
import pytest

from oracle.cpu_ref import RefEngine

f = np.float32
GC = 32


def build(tx, ty, tgx, tgy, tmd, NA, hb):
    sd = 2 * hb / GC
    m, x0, inv = f(1e-4), f(-hb), f(GC / (2 * hb))
    cov = np.zeros(GC, np.uint64)
    arow = np.zeros(GC, np.uint64)
    acol = np.zeros(GC, np.uint64)
    for r in range(GC):
        s0, s1 = f(f(-hb + r * sd) - m), f(f(-hb + (r + 1) * sd) + m)
        for a in range(NA):
            d = f(tmd[a]); dl = f(d + m); ds = f(d - m)
            for cxd, cyd in ((tx[a], ty[a]), (tgx[a], tgy[a])):
                cx, cy = f(cxd), f(cyd)
                if f(cy + dl) >= s0 and f(cy - dl) <= s1:
                    arow[r] |= np.uint64(1 << a)
                if f(cx + dl) >= s0 and f(cx - dl) <= s1:
                    acol[r] |= np.uint64(1 << a)
                dy = max(abs(f(s0 - cy)), abs(f(s1 - cy)))
                if ds > dy:
                    w = np.sqrt(f(f(ds * ds) - f(dy * dy)))
                    lo = max(int(np.floor(f(f(f(cx - w) - x0) + m) * inv)) + 1, 0)
                    hi = min(int(np.floor(f(f(f(cx + w) - x0) - m) * inv)) - 1, GC - 1)
                    for i in range(lo, hi + 1):
                        cov[r] |= np.uint64(1 << i)
    return cov, arow, acol


def test_cover_never_rejects_an_accepted_try():
    from bench import make_config
    E, N = 6, 25
    eng = RefEngine(make_config(E, N, 0, E, workload="c3"))
    eng.reset()
    rng = np.random.default_rng(3)
    ntries = ncov = 0
    for t in range(40):
        eng.step(rng.uniform(-1, 1, (E, 2)).astype(np.float32))
        if t < 25 or t % 5:
            continue
        s = eng.get_state()
        for e in range(E):
            h = int(rng.integers(N))
            o = [j for j in range(N) if j != h]
            r = s.h_r[e]
            tx = np.concatenate([[s.r_px[e]], s.h_px[e][o]]); ty = np.concatenate([[s.r_py[e]], s.h_py[e][o]])
            tgx = np.concatenate([[s.r_gx[e]], s.h_gx[e][o]]); tgy = np.concatenate([[s.r_gy[e]], s.h_gy[e][o]])
            tmd = np.concatenate([[r[h] + s.r_radius[e] + 0.25], r[h] + r[o] + 0.25])
            hb = 0.1 * 20 + 0.5 + 1e-3
            cov, arow, acol = build(tx, ty, tgx, tgy, tmd, N, hb)
            u = rng.random((3000, 4))   # the goal candidates, plus points seeded just inside every disc's rim
            gx = (u[:, 2] - 0.5) * 10 * 0.4 + (u[:, 0] - 0.5); gy = (u[:, 3] - 0.5) * 10 * 0.4 + (u[:, 1] - 0.5)
            ang = rng.random(2000) * 2 * np.pi; a = rng.integers(N, size=2000); g = rng.integers(2, size=2000)
            rad = tmd[a] * (1 - rng.random(2000) * 1e-3)
            gx = np.concatenate([gx, np.where(g, tgx[a], tx[a]) + rad * np.cos(ang)])
            gy = np.concatenate([gy, np.where(g, tgy[a], ty[a]) + rad * np.sin(ang)])
            inside = np.zeros((len(gx), N), bool)
            for k in range(N):
                inside[:, k] = ((np.sqrt((gx - tx[k]) ** 2 + (gy - ty[k]) ** 2) < tmd[k])
                                | (np.sqrt((gx - tgx[k]) ** 2 + (gy - tgy[k]) ** 2) < tmd[k]))
            fx, fy = (gx + hb) * (GC / (2 * hb)), (gy + hb) * (GC / (2 * hb))
            inb = (fx >= 0) & (fx < GC) & (fy >= 0) & (fy < GC)
            ix, iy = np.clip(fx.astype(int), 0, GC - 1), np.clip(fy.astype(int), 0, GC - 1)
            covered = inb & (((cov[iy] >> ix.astype(np.uint64)) & np.uint64(1)) == 1)
            assert not (covered & ~inside.any(1)).any()
            msk = arow[iy] & acol[ix]
            for k in range(N):
                assert not (inb & inside[:, k] & (((msk >> np.uint64(k)) & np.uint64(1)) == 0)).any()
            ntries += len(gx)
            ncov += int(covered.sum())
    assert ncov > 0.5 * ntries   # the cover decides most tries without an exact test
