"""Diagnostic: the spawn budget (cn_debug_set_spawn_budget) against step-launch time, C3 (kd-tree path) or C2
(quad path): per budget, 100 warm-up + 200 timed launches after cn_reset (bench.py's side-window shape), alternating.

    python tools/probe_budget.py [c3|c2] [rounds] [budget ...]
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def run(wl, budget, W=100, K=200, E=4096):
    N = 25 if wl == "c3" else 10
    eng = CrowdNavEngine(bench.make_config(E, N, 0, E, workload=wl), "cuda:0")
    eng.set_spawn_budget(budget)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = (torch.randn((W + K, E, 2), generator=g, device="cuda:0") * 0.5 if wl == "c3" else
            torch.rand((W + K, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    eng.reset()
    eng.step_seq(acts[:W])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step_seq(acts[W:])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.spawn_stats()
    eng.close()
    return E * K / dt, st


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    budgets = [int(x) for x in sys.argv[3:]] or [300000, 450000, 600000, 900000]
    for r in range(R):
        for b in budgets:
            v, st = run(wl, b)
            print("%s budget %7d: %.3f M env-steps/s  inline %d parked %d" % (wl, b, v / 1e6, st["inline_resets"],
                                                                          st["parked_midway"]), flush=True)


if __name__ == "__main__":
    main()
