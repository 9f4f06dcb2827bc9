"""Diagnostic: op-level profile of the DSRNN training forward/backward at C4 minibatch size
(T = 128 steps x 2048 envs, N = 10) — which GEMMs / kernels dominate one PPO minibatch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import ops  # noqa: E402


def main(T=128, B=2048, N=10):
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    H, F = 256, 64
    x = torch.randn(T, B * N, F, device=dev, generator=g, requires_grad=True)
    h0 = torch.randn(B * N, H, device=dev, generator=g)
    m = (torch.rand(T, B * N, device=dev, generator=g) > 0.02).float()
    gru = torch.nn.GRU(F, H).to(dev)
    w = [gru.weight_ih_l0, gru.weight_hh_l0, gru.bias_ih_l0, gru.bias_hh_l0]
    for _ in range(2):
        out, hT = ops.masked_gru(x, h0, m, *w)
        (out.sum() + hT.sum()).backward()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile, record_function

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        with record_function("gru_fwd"):
            out, hT = ops.masked_gru(x, h0, m, *w)
        torch.cuda.synchronize()
        with record_function("gru_bwd"):
            (out.sum() + hT.sum()).backward()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=60))
    ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev[0].record()
    out, hT = ops.masked_gru(x, h0, m, *w)
    ev[1].record()
    torch.cuda.synchronize()
    f_ms = ev[0].elapsed_time(ev[1])
    ev[0].record()
    (out.sum() + hT.sum()).backward()
    ev[1].record()
    torch.cuda.synchronize()
    print("spatial GRU T=%d rows=%d: forward %.2f ms, backward %.2f ms" % (T, B * N, f_ms, ev[0].elapsed_time(ev[1])))


if __name__ == "__main__":
    main()
