"""Diagnostic: C3 (or C2) step time with parts of the RNG work switched off, to size the goal-change work.

    python tools/c3_variants.py [steps] [c3|c2]

Variants: the C3 workload as benched; without end-goal changing; without random goal changing; without
either. Each: 30 warmup steps, then `steps` timed launches (HIP events on the engine's stream).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def run(end_goal, rand_goal, steps, E=4096, wl="c3"):
    c = clone_config(Config())
    c.humans.policy = "orca"
    if wl == "c3":
        c.sim.human_num = 25
        c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
    else:   # bench.py's C2 workload
        c.sim.human_num = 10
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.action_space.kinematics = "unicycle"
    c.humans.end_goal_changing = end_goal
    c.humans.random_goal_changing = rand_goal
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E, phase="train"), "cuda:0")
    eng.reset()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = torch.rand((steps + 30, E, 2), generator=g, device="cuda:0") * 2 - 1
    for s in range(30):
        eng.step(acts[s])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in range(steps):
        eng.step(acts[30 + s])
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    print("end_goal=%d random_goal=%d: %.3f ms per step, %.2f M env-steps/s" % (end_goal, rand_goal, ms,
                                                                             E / ms / 1e3), flush=True)
    eng.close()


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    wl = sys.argv[2] if len(sys.argv) > 2 else "c3"
    for eg, rg in ((True, True), (False, True), (True, False), (False, False)):
        run(eg, rg, steps, wl=wl)
