"""Diagnostic: where the fixed cost of a short timed window goes (bench.py's --steps 20 --warmup 5).

    python tools/probe_launch_latency.py [reps]

For R repetitions of a fresh engine: W = 5 warm-up launches, then K = 20 launches timed like bench.py
(synchronize, t0, K step() calls, synchronize). Prints per repetition: wall, the host time to submit the K
launches, the cn_profile event span (GPU, first launch start -> last launch end) and the difference
(launch latency at the start + synchronize wake-up at the end). Variants: plain step() calls, pre-sliced
action views, and the K launches captured in one HIP graph (graph mode) and replayed.
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def window(variant, E=4096, N=10, W=5, K=20):
    dev = torch.device("cuda", 0)
    eng = CrowdNavEngine(bench.make_config(E, N, 0, E, "c2"), dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    a = (torch.rand((K + W, E, 2), generator=g, device=dev) * 0.2 - 0.1).contiguous()
    L = _lib.lib()
    eng.reset()
    graph = None
    if variant == "graph":
        eng.set_graph_mode(True)
    for s in range(W):
        eng.step(a[s])
    views = [a[W + s] for s in range(K)]
    if variant == "graph":
        torch.cuda.synchronize()
        s_ = torch.cuda.Stream()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s_):
            with torch.cuda.graph(graph, stream=s_):
                for s in range(K):
                    eng.step(views[s])
    if variant == "readback":   # bench.py's reset count before the window: the whole state to host memory
        bench.reset_total(eng)
    if variant == "fieldread":
        bench.reset_total_dev(eng)
    _lib.check(L.cn_profile(eng._h, 1, K if variant != "graph" else 1))
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if variant == "graph":
        graph.replay()
    else:
        for s in range(K):
            eng.step(views[s] if variant == "views" else a[W + s])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    if variant != "graph":
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
    _lib.check(L.cn_profile(eng._h, 0, 0))
    eng.close()
    wall = (t2 - t0) * 1e6
    span = ta.value * 1e3
    print("%-6s wall %7.1f us  submit %7.1f us  event span %7.1f us  (%.2f us/launch)  wall - span %6.1f us  "
          "-> %.1f M env-steps/s" % (variant, wall, (t1 - t0) * 1e6, span, span / K, wall - span, E * K / wall),
          flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for _ in range(reps):
        for v in ("plain", "readback", "fieldread"):
            window(v)
