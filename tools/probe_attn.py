"""Diagnostic: per-launch time of the fused spatial attention kernels (cn_spatial_attn_fwd / _bwd) at C4's
PPO minibatch shape (R = 128 x 2,048 rows, N = 10 edges, H = 256), HIP events, and the HBM rate they imply."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402


def main(R=128 * 2048, N=10, H=256, reps=5):
    L = _lib.lib()
    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    hs = torch.randn((R, N, H), generator=g, device=dev)
    u = torch.randn((R, H), generator=g, device=dev) * 0.05
    c = torch.randn((R,), generator=g, device=dev) * 0.05
    out = torch.empty((R, H), device=dev)
    attn = torch.empty((R, N), device=dev)
    dout = torch.randn((R, H), generator=g, device=dev)
    dattn = torch.randn((R, N), generator=g, device=dev)
    dhs = torch.empty_like(hs)
    due = torch.empty((R, H + 4), device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def fwd():
        _lib.check(L.cn_spatial_attn_fwd(st, R, N, H, 1.25, hs.data_ptr(), u.data_ptr(), c.data_ptr(), out.data_ptr(),
                                         attn.data_ptr()))

    def bwd():
        _lib.check(L.cn_spatial_attn_bwd(st, R, N, H, 1.25, hs.data_ptr(), u.data_ptr(), attn.data_ptr(),
                                         dout.data_ptr(), dattn.data_ptr(), dhs.data_ptr(), due.data_ptr(), H + 4,
                                         due.data_ptr() + 4 * H, H + 4))

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    tf, tb = timed(fwd), timed(bwd)
    bf = R * N * H * 4 + R * H * 4 * 2 + R * N * 4
    bb = 2 * R * N * H * 4 + R * H * 4 * 3 + R * N * 8
    print("attn fwd %.1f us (%.2f TB/s), bwd %.1f us (%.2f TB/s)" % (tf, bf / tf / 1e6, tb, bb / tb / 1e6), flush=True)


if __name__ == "__main__":
    main()
