"""Diagnostic: C3 step-kernel time per launch with parts of the RNG work switched off (which part of the
launch the goal changes cost). Same workload as bench.py --workload c3 otherwise.

    python tools/probe_c3_variants.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def run(name, end_goal=True, rand_goal=True, E=4096, N=25, W=125, K=400):
    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
    c.action_space.kinematics = "holonomic"
    c.robot.FOV = c.humans.FOV = 1.0
    c.humans.end_goal_changing = end_goal
    c.humans.random_goal_changing = rand_goal
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0")
    if os.environ.get("CN_SPAWN_BUDGET"):
        eng.set_spawn_budget(int(os.environ["CN_SPAWN_BUDGET"]))
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    a = torch.randn((W + K, E, 2), generator=g, device="cuda:0") * 0.5
    eng.reset()
    for s in range(W):
        eng.step(a[s])
    L = _lib.lib()
    st0 = eng.spawn_stats()
    _lib.check(L.cn_profile(eng._h, 1, K))
    for s in range(K):
        eng.step(a[W + s])
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    _lib.check(L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n)))
    us = ta.value * 1e3 / n.value
    st1 = eng.spawn_stats()
    print("%-28s %8.1f us per launch  -> %.2f M env-steps/s; per launch: %s" % (
        name, us, E / us, ", ".join("%s %.1f" % (k, (st1[k] - st0[k]) / K) for k in st1)), flush=True)
    eng.close()


if __name__ == "__main__":
    if sys.argv[1:] == ["default"]:
        run("c3 (default) " + os.environ.get("CN_LIB_PATH", "").split("/")[-1])
        sys.exit(0)
    run("c3 (default)")
    run("c3 no end-goal changes", end_goal=False)
    run("c3 no random goal changes", rand_goal=False)
    run("c3 no goal changes", end_goal=False, rand_goal=False)
