"""Diagnostic: per-launch time of the sequence GRU kernels (cn_gru_fwd_seq / cn_gru_bwd_seq) at C4's PPO
minibatch shapes, timed with HIP events on the launching stream.

    python tools/probe_gru_seq.py            # edge pair (20,480 + 2,048 rows, H = 256) and node GRU (2,048, 128)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402


def case(name, Bs, H, T=16, reps=3, F=0):
    L = _lib.lib()
    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    fs = (_lib.GruSeqFwd * len(Bs))()
    bs = (_lib.GruSeqBwd * len(Bs))()
    keep = []
    for i, B in enumerate(Bs):
        gi = torch.randn((T, B, 3 * H), generator=g, device=dev) if not F else None
        x = torch.randn((T, B, F), generator=g, device=dev) if F else None
        wih = torch.randn((3 * H, F), generator=g, device=dev) / max(F, 1) ** 0.5 if F else None
        bih = torch.randn((3 * H,), generator=g, device=dev) * 0.1 if F else None
        w = torch.randn((3 * H, H), generator=g, device=dev) / H ** 0.5
        b = torch.randn((3 * H,), generator=g, device=dev) * 0.1
        m = (torch.rand((T, B), generator=g, device=dev) > 0.05).float()
        out = torch.empty((T, B, H), device=dev)
        hm = torch.randn((T, B, H), generator=g, device=dev) * 0.5
        save = torch.empty((T, B, 4 * H), device=dev)
        wt = w.t().contiguous()
        dout = torch.randn((T, B, H), generator=g, device=dev)
        acc = torch.zeros((B, H), device=dev)
        gg = torch.empty((T, B, 4 * H), device=dev)
        db = torch.empty((2, 3 * H), device=dev)
        fs[i] = _lib.GruSeqFwd(B, gi.data_ptr() if gi is not None else None, w.data_ptr(), b.data_ptr(), m.data_ptr(),
                               out.data_ptr(), hm.data_ptr(), save.data_ptr(), T,
                               x.data_ptr() if F else None, wih.data_ptr() if F else None,
                               bih.data_ptr() if F else None, F)
        bs[i] = _lib.GruSeqBwd(B, wt.data_ptr(), m.data_ptr(), dout.data_ptr(), save.data_ptr(), hm.data_ptr(),
                               acc.data_ptr(), gg.data_ptr(), db[0].data_ptr(), db[1].data_ptr())
        keep += [gi, x, wih, bih, w, b, m, out, hm, save, wt, dout, acc, gg, db]
    work = torch.empty((L.cn_gru_bwd_seq_work_elems(T, H, len(Bs), bs),), device=dev)

    def timed(fn, launches):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps / launches

    tf = timed(lambda: _lib.check(L.cn_gru_fwd_seq(st, T, H, len(Bs), fs)), T)
    tb = timed(lambda: _lib.check(L.cn_gru_bwd_seq(st, T, H, len(Bs), bs, work.data_ptr(), work.numel())), T + 1)
    rows = sum(Bs)
    fl = 2.0 * rows * H * 3 * H
    flf = 2.0 * rows * (H + F) * 3 * H
    print("%-10s rows %6d H %3d: fwd %7.1f us/launch (%.0f TFLOP/s), bwd %7.1f us/launch (%.0f TFLOP/s)"
          % (name, rows, H, tf, flf / tf / 1e6, tb, fl * T / (T + 1) / tb / 1e6), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "pair":   # the edge-pair case alone (counter passes)
        case("pair, x-mode", (20480, 2048), 256, F=64)
        sys.exit(0)
    case("edge pair", (20480, 2048), 256)
    case("pair, x-mode", (20480, 2048), 256, F=64)
    case("spatial", (20480,), 256)
    case("node", (2048,), 128)
    case("node x-mode", (2048,), 128, F=128)
