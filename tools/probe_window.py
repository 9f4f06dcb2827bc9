"""Where a short timed window's wall time goes (C2 engine, the driver's --steps 20 --warmup 5 shape):
for K in a few sizes, repeated windows of K step launches, each bracketed like bench.py (synchronize,
t0, launches, synchronize): wall time vs the GPU span of the K step kernels (HIP events recorded on the
stream right before the first and after the last launch) vs the host's issue time. A fit of
wall = fixed + K * per_step separates the per-window fixed cost from the per-step cost.

    python tools/probe_window.py [reps]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
eng = CrowdNavEngine(bench.make_config(4096, 10, 0, 4096, "c2"), dev)
g = torch.Generator(device=dev).manual_seed(0)
acts = (torch.rand((3000, 4096, 2), generator=g, device=dev) * 0.2 - 0.1).contiguous()
eng.reset()
pos = 0
eng.step_seq(acts[pos:pos + 5])
pos += 5
torch.cuda.synchronize()
rows = []
for mode in ("seq", "host"):
    for K in (1, 5, 20, 100):
        for r in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            idle = 0.0005 if r % 2 else 0.0   # odd reps: the GPU idles 0.5 ms before the window
            torch.cuda.synchronize()
            if idle:
                time.sleep(idle)
            t0 = time.perf_counter()
            e0.record()
            if mode == "seq":
                eng.step_seq(acts[pos:pos + K])
            else:
                for s in range(K):
                    eng.step(acts[pos + s])
            e1.record()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            pos += K
            if pos > 2800:
                pos = 5
            rows.append((mode, K, r % 2, (t2 - t0) * 1e6, (t1 - t0) * 1e6, e0.elapsed_time(e1) * 1e3))
# bench.py's own bracket: reset count read, cn_profile armed (its two HIP events recorded by cn_step), barrier
import ctypes  # noqa: E402

from crowdnav_dsrnn_amd import _lib  # noqa: E402

L = _lib.lib()
for variant in ("bench", "bench_noprof", "bench_noreset"):
    res = []
    for r in range(reps):
        K = 20
        if variant != "bench_noreset":
            bench.reset_total_dev(eng)
        if variant != "bench_noprof":
            _lib.check(L.cn_profile(eng._h, 1, K))
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step_seq(acts[pos:pos + K])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        span = float("nan")
        if variant != "bench_noprof":
            a_ms, b_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
            _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a_ms), ctypes.byref(b_ms), ctypes.byref(n)))
            _lib.check(L.cn_profile(eng._h, 0, 0))
            span = a_ms.value * 1e3
        pos += K
        if pos > 2800:
            pos = 5
        res.append(((t2 - t0) * 1e6, (t1 - t0) * 1e6, span))
    print("%-14s K=20: wall %s us, issue %s us, cn_profile span %s us" % (
        variant, [round(x[0], 1) for x in res], [round(x[1], 1) for x in res], [round(x[2], 1) for x in res]),
        flush=True)
for mode in ("seq", "host"):
    for idle in (0, 1):
        sel = [x for x in rows if x[0] == mode and x[2] == idle]
        Ks = np.array([x[1] for x in sel], float)
        wall = np.array([x[3] for x in sel])
        span = np.array([x[5] for x in sel])
        A = np.stack([np.ones_like(Ks), Ks], 1)
        fw = np.linalg.lstsq(A, wall, rcond=None)[0]
        fs = np.linalg.lstsq(A, span, rcond=None)[0]
        print("%s idle=%d: wall = %.1f us + K x %.2f us; event span = %.1f us + K x %.2f us" %
              (mode, idle, fw[0], fw[1], fs[0], fs[1]), flush=True)
        for K in (1, 5, 20, 100):
            ss = [x for x in sel if x[1] == K]
            print("   K=%3d wall %8.1f us  issue %8.1f us  span %8.1f us" %
                  (K, np.median([x[3] for x in ss]), np.median([x[4] for x in ss]), np.median([x[5] for x in ss])),
                  flush=True)
eng.close()
