"""Diagnostic: op-level profile of one PPO minibatch of the DSRNN (evaluate_actions forward + backward
+ Adam step) at C4 size (T = 128 steps x 2048 envs, N = 10)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd.config import Config, clone_config  # noqa: E402
from crowdnav_dsrnn_amd.policy import Policy  # noqa: E402
from crowdnav_dsrnn_amd.spaces import action_space, observation_space  # noqa: E402


def main(T=128, B=2048, N=10):
    dev = "cuda:0"
    c = clone_config(Config())
    c.sim.human_num = N
    c.training.num_processes = 2 * B
    c.ppo.num_steps = T
    c.ppo.num_mini_batch = 2
    pol = Policy(observation_space(N).spaces, action_space(), base="srnn", base_kwargs=c).to(dev)
    opt = torch.optim.Adam(pol.parameters(), lr=4e-5, eps=1e-5)
    g = torch.Generator(device=dev).manual_seed(0)
    obs = {"robot_node": torch.randn(T * B, 1, 7, device=dev, generator=g),
           "temporal_edges": torch.randn(T * B, 1, 2, device=dev, generator=g),
           "spatial_edges": torch.randn(T * B, N, 2, device=dev, generator=g)}
    hxs = {"human_node_rnn": torch.zeros(B, 1, 128, device=dev), "human_human_edge_rnn": torch.zeros(B, N + 1, 256, device=dev)}
    masks = (torch.rand(T * B, 1, device=dev, generator=g) > 0.02).float()
    act = torch.randn(T * B, 2, device=dev, generator=g)

    def mb():
        v, lp, ent, _ = pol.evaluate_actions(obs, dict(hxs), masks, act)
        loss = v.pow(2).mean() - lp.mean() - 0.01 * ent
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(pol.parameters(), 0.5)
        opt.step()

    for _ in range(2):
        mb()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(3):
        mb()
    ev[1].record()
    torch.cuda.synchronize()
    print("minibatch (T=%d, %d envs): %.1f ms" % (T, B, ev[0].elapsed_time(ev[1]) / 3))
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        mb()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=70))


if __name__ == "__main__":
    main()
