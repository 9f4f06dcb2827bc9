"""Diagnostic: catch a C3 run that departs from the first one. Run 0 keeps its full state every S launches;
every later run compares at the same launches and, at the first difference, prints the launch, the envs and
the differing fields with both runs' values for the first envs.

    python tools/probe_c3_diverge2.py [R] [K] [S] [spawn budget] [c3|c2]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import abi  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


WL = "c3"


def make(E=4096, N=25):
    c = clone_config(Config())
    c.humans.policy = "orca"
    if WL == "c2":   # the quad path (its spawns park too since round 6)
        N = 10
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.action_space.kinematics = "unicycle"
    else:
        c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
    c.sim.human_num = N
    return CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0"), E, N


def main(R=12, K=400, S=10, budget=None):
    ref = []
    for r in range(R):
        eng, E, N = make()
        if budget is not None:
            eng.set_spawn_budget(budget)
        g = torch.Generator(device="cuda:0")
        g.manual_seed(0)
        eng.reset()
        found = False
        for s in range(K):
            eng.step(torch.randn((E, 2), generator=g, device="cuda:0") * 0.5 if WL == "c3" else
                     torch.rand((E, 2), generator=g, device="cuda:0") * 0.2 - 0.1)
            if (s + 1) % S:
                continue
            sv = eng.get_state()
            if r == 0:
                ref.append(np.array(sv.blob, copy=True))
                continue
            b0 = ref[(s + 1) // S - 1]
            if np.array_equal(b0, np.asarray(sv.blob)):
                continue
            s0 = abi.StateView(b0, E, N, 0)   # (robot not visible in either workload)
            diff = {}
            for n, _, _ in abi.STATE_FIELDS:
                a0 = np.asarray(getattr(s0, n)).reshape(E, -1)
                a1 = np.asarray(getattr(sv, n)).reshape(E, -1)
                bad = np.nonzero((a0 != a1).any(1))[0]
                if len(bad):
                    diff[n] = bad
            envs = sorted(set(int(x) for v in diff.values() for x in v))
            print("run %d departs at launch %d: %d envs %s; fields %s" % (r, s + 1, len(envs), envs[:10],
                                                                        {n: len(v) for n, v in diff.items()}), flush=True)
            for e in envs[:3]:
                for n in diff:
                    a0 = np.asarray(getattr(s0, n)).reshape(E, -1)[e]
                    a1 = np.asarray(getattr(sv, n)).reshape(E, -1)[e]
                    if (a0 != a1).any():
                        k = np.nonzero(a0 != a1)[0]
                        print("   env %d %s idx %s: %s vs %s" % (e, n, k[:6], a0[k[:6]], a1[k[:6]]), flush=True)
            found = True
            break
        print("run %d: %s%s" % (r, eng.spawn_stats(), "" if found or r == 0 else " == run 0"), flush=True)
        eng.close()


if __name__ == "__main__":
    if len(sys.argv) > 5:
        WL = sys.argv[5]
    main(*(int(x) for x in sys.argv[1:5]))
