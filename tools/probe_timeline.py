"""Diagnostic: per launch, which workgroups end last -- the step workgroups or the spare workgroups drawing the
upcoming episodes' spawns -- on the device-wide 100 MHz clock of the -DCN_STAMPS build (cn_debug_stamps_r).

    CN_LIB_PATH=tools/bin/libcn_stamps.so python tools/probe_timeline.py [steps] [c2|c3]

Per launch: kernel time (HIP events, cn_profile), the last step workgroup's end, the last spawn workgroup's
end (ns from the grid's first start), envs done by the previous launch (the spawns this launch draws).
The first 30 launches after cn_reset are printed one by one (bench.py --steps 20 --warmup 5 times launches
6-25), then a summary of the rest.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(steps=400, wl="c2", E=4096):
    c = clone_config(Config())
    c.humans.policy = "orca"
    if wl == "c3":
        N = 25
        c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
    else:
        N = 10
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.action_space.kinematics = "unicycle"
    c.sim.human_num = N
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), "cuda:0")
    eng.reset()
    L = _lib.lib()
    L.cn_debug_stamps_r.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    sp = np.zeros(8192 * 16, np.uint64)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    if wl == "c2":
        acts = torch.rand((steps, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1
    else:
        acts = torch.randn((steps, E, 2), generator=g, device="cuda:0") * 0.5
    epb = min(64 // N, 16)
    blocks = (E + epb - 1) // epb
    r = np.zeros(8192 * 2, np.uint64)
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    rows = []
    prev_done = E   # cn_reset: every env's first spawn was drawn by the reset kernel, the next ones ahead
    st_prev = eng.spawn_stats()
    for s in range(steps):
        r[:] = 0
        _lib.check(L.cn_profile(eng._h, 1, 1))
        eng.step(acts[s])
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
        L.cn_debug_stamps_r(r.ctypes.data_as(ctypes.c_void_p), sp.ctypes.data_as(ctypes.c_void_p))
        R = r.reshape(-1, 2).astype(np.int64)
        live = np.nonzero(R[:, 1] > 0)[0]
        R = R[:live.max() + 1]
        # this launch's workgroups: stamps within 10 ms (100 MHz ticks) of its last end (entries of other
        # launches or never written are older or zero)
        fresh = R[:, 0] > R[:, 1].max() - 1000000
        t0 = R[fresh, 0].min()
        en = (R[:, 1] - t0) * 10
        step_sel = np.zeros(len(R), bool)
        if wl == "c3":
            step_sel[len(R) - blocks:] = True
        else:
            step_sel[:blocks] = True
        d = int(eng.done.sum().item())
        st = eng.spawn_stats()
        rows.append((ta.value * 1e3, en[step_sel].max(), en[~step_sel].max() if (~step_sel).any() else 0,
                     np.percentile(en[step_sel], 50), prev_done, st["inline_resets"] - st_prev["inline_resets"],
                     st["parked_unstarted"] - st_prev["parked_unstarted"] + st["parked_midway"] - st_prev["parked_midway"]))
        st_prev = st
        prev_done = d
    _lib.check(L.cn_profile(eng._h, 0, 0))
    # spawn_env segments (the latest spawn of each env: seeding, robot, humans 0..N-1), cycles
    Sg = sp.reshape(-1, 16).astype(np.int64)[:E]
    ok = Sg[:, min(3 + N - 1, 15)] > Sg[:, 0]
    if ok.any() and 3 + N <= 16:   # segments of up to 13 humans are stamped
        Sg = Sg[ok]
        seg = np.diff(Sg[:, :3 + N], axis=1)
        print("[%s] spawn_env segments over %d envs' latest spawn (cycles, median / p90): seed %d / %d, robot %d / %d, "
              "humans %s; total %d / %d" % (
                  wl, ok.sum(), np.median(seg[:, 0]), np.percentile(seg[:, 0], 90), np.median(seg[:, 1]),
                  np.percentile(seg[:, 1], 90),
                  " ".join("%d" % v for v in np.median(seg[:, 2:], 0)), np.median(Sg[:, 2 + N] - Sg[:, 0]),
                  np.percentile(Sg[:, 2 + N] - Sg[:, 0], 90)))
    a = np.asarray(rows)
    print("[%s] launch | kernel us | last step-WG end us | last spawn-WG end us | median step-WG end | "
          "resets drawn ahead (prev done) | resets drawn inline | spawns parked" % wl)
    for s in range(min(30, steps)):
        print("  %4d  %7.1f  %7.1f  %7.1f  %7.1f  %5d  %5d  %5d" % (s, a[s, 0], a[s, 1] / 1e3, a[s, 2] / 1e3, a[s, 3] / 1e3,
                                                           a[s, 4], a[s, 5], a[s, 6]))
    rest = a[30:]
    if len(rest):
        spawn_last = (rest[:, 2] > rest[:, 1]).mean()
        print("  launches 30..%d: kernel mean %.1f us; last step-WG end mean %.1f us; last spawn-WG end mean %.1f us; "
              "spawn WGs end last in %.0f%% of launches; corr(kernel, prev done) %.2f" % (
                  steps - 1, rest[:, 0].mean(), rest[:, 1].mean() / 1e3, rest[:, 2].mean() / 1e3, 100 * spawn_last,
                  np.corrcoef(rest[:, 0], rest[:, 4])[0, 1]))
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400, sys.argv[2] if len(sys.argv) > 2 else "c2")
