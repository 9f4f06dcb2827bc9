"""Diagnostic: C3 determinism. Runs the C3 workload R times from the same reset and records a per-env digest
of the state every S launches; prints the first launch / envs / fields where any run departs from run 0.

    python tools/probe_c3_diverge.py OUT.npz [R] [K] [S] [budget]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import abi  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402

FIELDS = [n for n, _, _ in abi.STATE_FIELDS]


def digests(sv, E):
    out = {}
    for n in FIELDS:
        a = np.ascontiguousarray(np.asarray(getattr(sv, n))).reshape(E, -1).view(np.uint8)
        out[n] = np.frombuffer(np.ascontiguousarray(a), np.uint8).reshape(E, -1).astype(np.uint64).sum(1) * 1315423911 \
            + (a.reshape(E, -1)[:, ::7].astype(np.uint64).sum(1))
    return out


def run_once(K, S, budget, E=4096, N=25):
    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
    c.action_space.kinematics = "holonomic"
    c.robot.FOV = c.humans.FOV = 1.0
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0")
    if budget is not None:
        eng.set_spawn_budget(budget)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    eng.reset()
    recs = []
    for s in range(K):
        eng.step(torch.randn((E, 2), generator=g, device="cuda:0") * 0.5)
        if (s + 1) % S == 0:
            recs.append(digests(eng.get_state(), E))
    st = eng.spawn_stats()
    eng.close()
    return recs, st


def main(out, R=4, K=400, S=10, budget=None):
    runs = []
    for r in range(R):
        recs, st = run_once(K, S, budget)
        runs.append(recs)
        print("run %d: %s" % (r, st), flush=True)
    for r in range(1, R):
        for k, (a, b) in enumerate(zip(runs[0], runs[r])):
            bad = {n: np.nonzero(a[n] != b[n])[0] for n in FIELDS if (a[n] != b[n]).any()}
            if bad:
                envs = sorted(set(int(x) for v in bad.values() for x in v))
                print("run %d departs from run 0 by launch %d: envs %s; fields %s" % (
                    r, (k + 1) * S, envs[:12], {n: len(v) for n, v in bad.items()}), flush=True)
                break
        else:
            print("run %d == run 0 through launch %d" % (r, K), flush=True)
    np.savez(out, **{"r%d_%d_%s" % (r, k, n): v for r, recs in enumerate(runs) for k, d in enumerate(recs)
                     for n, v in d.items() if k % 5 == 4})


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(int(x) for x in a[1:4]), *( [int(a[4])] if len(a) > 4 else []))
