"""Micro-benchmark: the masked GRU backward's recurrent GEMM acc += dgh W_hh (B x 3H @ 3H x H) as one
addmm_ vs per-gate batched GEMMs (3 x B x H outputs, 3x the output tiles) + a sum."""
import torch

dev = torch.device("cuda:0")
B, H = 20480, 256
g = torch.Generator(device=dev).manual_seed(0)
dgh = torch.randn(B, 3 * H, device=dev, generator=g)
w = torch.randn(3 * H, H, device=dev, generator=g) * 0.05
acc = torch.randn(B, H, device=dev, generator=g)
w3 = w.view(3, H, H)
out3 = torch.empty(3, B, H, device=dev)


def a():
    acc.addmm_(dgh, w)


def b():
    torch.bmm(dgh.view(B, 3, H).transpose(0, 1), w3, out=out3)
    acc.add_(out3[0]).add_(out3[1]).add_(out3[2])


def c():
    torch.bmm(dgh.view(B, 3, H).transpose(0, 1), w3, out=out3)
    torch.sum(out3, 0, out=tmp)
    acc.add_(tmp)


tmp = torch.empty(B, H, device=dev)
for name, f in (("addmm_", a), ("bmm+3add", b), ("bmm+sum+add", c)):
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    e1.synchronize()
    print("%-12s %.1f us" % (name, e0.elapsed_time(e1) * 1e3 / 50))
