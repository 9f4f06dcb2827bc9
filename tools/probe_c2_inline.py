"""Diagnostic: C2 steady-state spawn counters per launch (auto-resets drawn inline by the step kernel because
no pending spawn was ready) over bench.py's steady window shape (100 + 2,000 launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(E=4096, N=10, W=125, K=2000):
    eng = CrowdNavEngine(bench.make_config(E, N, 0, E, workload="c2"), "cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    eng.reset()
    for s in range(W):
        eng.step(torch.rand((E, 2), generator=g, device="cuda:0") * 0.2 - 0.1)
    st0 = eng.spawn_stats()
    for s in range(K):
        eng.step(torch.rand((E, 2), generator=g, device="cuda:0") * 0.2 - 0.1)
    st1 = eng.spawn_stats()
    print("c2 per launch over %d launches: %s" % (K, {k: round((st1[k] - st0[k]) / K, 3) for k in st1}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
