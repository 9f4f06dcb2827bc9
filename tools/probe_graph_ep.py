"""Diagnostic: episode bookkeeping of the HIP-graph rollout at C4's shape over several updates (the values
the graph writes into ep_sum / ep_cnt vs the same quantities recomputed eagerly from the storage)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd.config import Config, clone_config  # noqa: E402
from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv  # noqa: E402
from crowdnav_dsrnn_amd.learner import PPO  # noqa: E402
from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer  # noqa: E402
from crowdnav_dsrnn_amd.policy import Policy  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
c = clone_config(Config())
c.sim.human_num = 10
c.humans.policy = "orca"
c.action_space.kinematics = "holonomic"
c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
c.training.num_processes = E
c.ppo.num_steps = 128
c.ppo.epoch = 5
c.ppo.num_mini_batch = 2
torch.manual_seed(11)
envs = CrowdNavVecEnv(c, E, c.env.seed, "cuda:0", nenv=E, phase="train")
pol = Policy(envs.observation_space.spaces, envs.action_space, base="srnn", base_kwargs=c).to("cuda:0")
agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, 2, c.ppo.value_loss_coef, c.ppo.entropy_coef, lr=4e-5, eps=1e-5,
            max_grad_norm=0.5)
tr = RolloutTrainer(c, envs, pol, agent, deterministic=True, graphs=True)
for u in range(5):
    st = tr.update()
    r = tr.rollouts
    dones = int((r.masks[1:] == 0).sum())
    eps = float(tr._ep_ret.sum().item())
    print("update %d graph=%s episodes %d (storage %d) ep_sum %.3f (storage %.3f) mean %.3f" %
          (u, tr._graph is not None, st["episodes"], dones, st["mean_episode_return"] * max(st["episodes"], 1), eps,
           st["mean_episode_return"]), flush=True)
