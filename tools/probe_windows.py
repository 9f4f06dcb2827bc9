"""Diagnostic: kernel A / B average times per window of steps over a long C2 run (production library).

    python tools/probe_windows.py [steps] [window] [variant]
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(steps=600, window=50, variant="c2", E=4096, N=10):
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    if variant in ("nogoal", "norand"):
        c.humans.random_goal_changing = False
    if variant in ("noend", "norand"):
        c.humans.end_goal_changing = False
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), "cuda:0")
    eng.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = torch.rand((steps, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1
    L = _lib.lib()
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    for w0 in range(0, steps, window):
        _lib.check(L.cn_profile(eng._h, 1, window))
        dn = 0
        for s in range(w0, min(steps, w0 + window)):
            eng.step(acts[s])
            dn += int(eng.done.sum().item()) if s % 10 == 0 else 0
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
        print("[%s] steps %4d-%4d  A %.1f us  B %.1f us  (done@every10th sum %d)" % (
            variant, w0, w0 + n.value, ta.value * 1e3 / n.value, tb.value * 1e3 / n.value, dn), flush=True)
    _lib.check(L.cn_profile(eng._h, 0, 0))
    eng.close()


def per_step(steps=300, show=60, E=4096, N=10):
    """Kernel time of each individual step (profile window of 1), to see the goal-change bursts."""
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), "cuda:0")
    eng.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = torch.rand((steps, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1
    L = _lib.lib()
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    ts = []
    for s in range(steps):
        _lib.check(L.cn_profile(eng._h, 1, 1))
        eng.step(acts[s])
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
        ts.append(ta.value * 1e3)
    import numpy as np
    t = np.array(ts[steps - show:])
    print("per-step kernel us (last %d): %s" % (show, " ".join("%.0f" % x for x in t)))
    print("median %.1f mean %.1f max %.1f" % (np.median(t), t.mean(), t.max()))
    eng.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "per_step":
        per_step()
        sys.exit(0)
    main(int(a[0]) if a else 600, int(a[1]) if len(a) > 1 else 50, a[2] if len(a) > 2 else "c2")
