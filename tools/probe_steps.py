"""Diagnostic: step-kernel duration per launch over a long C2 run, and (with the -DCN_STAMPS build)
what the slowest workgroup of each launch spent its time on.

    python tools/probe_steps.py [steps]
    CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so python tools/probe_steps.py [steps] stamps
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

NAMES = ["load", "visibility", "policy+terms", "ladder", "kin+obs", "rng"]


def main(steps=400, stamps=False, E=4096, N=10):
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), "cuda:0")
    eng.reset()
    L = _lib.lib()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = torch.rand((steps + 100, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1
    for s in range(100):
        eng.step(acts[s])
    torch.cuda.synchronize()
    if stamps:
        L.cn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        a = np.zeros(4096 * 16, np.uint64)
        b = np.zeros(8192 * 16, np.uint64)
    blocks = (E + (64 // N) - 1) // (64 // N)
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    times, dones, spans, slow_ph, med, meds = [], [], [], [], [], []
    for s in range(steps):
        _lib.check(L.cn_profile(eng._h, 1, 1))
        eng.step(acts[100 + s])
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
        times.append(ta.value * 1e3)
        dones.append(int(eng.done.sum().item()))
        if stamps:
            L.cn_debug_stamps(a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p))
            A = a.reshape(-1, 16)[:blocks].astype(np.int64)
            tot = A[:, 6] - A[:, 0]
            spans.append(A[:, 6].max() - A[:, 0].min())
            k = int(np.argmax(tot))
            slow_ph.append(np.diff(A[k, :7]))
            med.append(np.median(tot))
            meds.append(np.median(np.diff(A[:, :7], axis=1), 0))
    _lib.check(L.cn_profile(eng._h, 0, 0))
    t = np.asarray(times)
    d = np.asarray(dones)
    print("step kernel us: mean %.1f  p10 %.1f  p50 %.1f  p90 %.1f  p99 %.1f  max %.1f" % (
        t.mean(), *np.percentile(t, [10, 50, 90, 99]), t.max()))
    print("dones/step: mean %.1f  corr(time, dones) %.2f" % (d.mean(), np.corrcoef(t, d)[0, 1]))
    order = np.argsort(t)
    for q in (0.1, 0.5, 0.9, 0.99):
        i = order[int(q * (len(t) - 1))]
        print("  q%.2f step %d: %.1f us, %d done" % (q, i, t[i], d[i]))
    if stamps:
        sp = np.asarray(spans)
        sph = np.asarray(slow_ph)
        print("span cycles: mean %d p50 %d p90 %d  (median workgroup %d)" % (sp.mean(), np.median(sp), np.percentile(sp, 90),
                                                                             np.median(med)))
        print("slowest workgroup per launch, mean cycles per phase: " + ", ".join(
            "%s %d" % (nm, v) for nm, v in zip(NAMES, sph.mean(0))))
        print("slowest workgroup per launch, median cycles per phase: " + ", ".join(
            "%s %d" % (nm, v) for nm, v in zip(NAMES, np.median(sph, 0))))
        print("median workgroup, median cycles per phase: " + ", ".join(
            "%s %d" % (nm, v) for nm, v in zip(NAMES, np.median(np.asarray(meds), 0))))
        print("us per kcycle (span vs event time): %.4f" % (np.median(t) / np.median(sp) * 1e3))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400, "stamps" in sys.argv[2:],
         E=int(os.environ.get("CN_PROBE_ENVS", "4096")))
