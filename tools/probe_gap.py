"""Diagnostic: where the wall time per C2 step goes beyond the step kernel itself.

    python tools/probe_gap.py [steps]

Times K steps (a) as bench.py does (cn_profile events on), (b) without events, (c) host-only cost of
the Python step call (no GPU wait), (d) replayed from a HIP graph captured over 30-step chunks.
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(K=2000, E=4096, N=10):
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    dev = torch.device("cuda:0")
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), dev)
    eng.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = (torch.rand((K + 100, E, 2), generator=g, device=dev) * 0.2 - 0.1).contiguous()
    L = _lib.lib()
    for s in range(100):
        eng.step(acts[s])
    torch.cuda.synchronize()

    def timed(prof):
        if prof:
            _lib.check(L.cn_profile(eng._h, 1, K))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(K):
            eng.step(acts[100 + s])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ker = None
        if prof:
            a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
            _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
            _lib.check(L.cn_profile(eng._h, 0, 0))
            ker = a.value / max(n.value, 1) * 1e3
        return (t2 - t0) / K * 1e6, (t1 - t0) / K * 1e6, ker

    for prof in (True, False, True, False):
        wall, host, ker = timed(prof)
        print("events=%d  wall %.2f us/step  host submit %.2f us/step  kernel %s us" % (
            prof, wall, host, "%.2f" % ker if ker else "-"), flush=True)

    # HIP graph over chunks of 30 steps (a multiple of the 3-way spawn-list rotation)
    CH = 30
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream())
    graphs = []
    nch = K // CH
    with torch.cuda.stream(s):
        for k in range(nch):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for j in range(CH):
                    eng.step(acts[100 + k * CH + j])
            graphs.append(gr)
    torch.cuda.synchronize()
    for rep in range(2):
        t0 = time.perf_counter()
        for gr in graphs:
            gr.replay()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print("graph x%d: wall %.2f us/step" % (CH, (t1 - t0) / (nch * CH) * 1e6), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2000)
