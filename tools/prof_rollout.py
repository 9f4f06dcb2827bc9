"""Diagnostic: one rollout step of C4 (DSRNN act -> env step_device -> storage insert) at 4096 envs:
wall time per step vs summed GPU kernel time (is the step launch-bound?), and the top kernels."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd.config import Config, clone_config  # noqa: E402
from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv  # noqa: E402
from crowdnav_dsrnn_amd.learner import PPO  # noqa: E402
from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer  # noqa: E402
from crowdnav_dsrnn_amd.policy import Policy  # noqa: E402


def main(E=4096, N=10):
    dev = torch.device("cuda:0")
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.action_space.kinematics = "holonomic"
    c.training.num_processes = E
    c.ppo.num_steps = 128
    torch.manual_seed(0)
    envs = CrowdNavVecEnv(c, E, c.env.seed, dev, env_offset=0, nenv=E)
    pol = Policy(envs.observation_space.spaces, envs.action_space, base="srnn", base_kwargs=c).to(dev)
    agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, c.ppo.num_mini_batch, c.ppo.value_loss_coef,
                c.ppo.entropy_coef, lr=c.training.lr, eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
    tr = RolloutTrainer(c, envs, pol, agent)
    tr.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.collect()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 128
    print("rollout step wall %.3f ms" % (wall * 1e3))
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.collect()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    gpu = sum(e.self_device_time_total for e in ka if e.device_type.name == "CUDA") / 128
    n = sum(e.count for e in ka if e.device_type.name == "CUDA") / 128
    print("GPU kernel time per step %.3f ms, %.0f kernels per step" % (gpu / 1e3, n))
    print(ka.table(sort_by="self_cuda_time_total", row_limit=30, max_name_column_width=60))


if __name__ == "__main__":
    main()
