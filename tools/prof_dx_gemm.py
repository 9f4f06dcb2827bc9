"""Micro-benchmark: the masked GRU backward's input gradient dx = dgi (T*B x 3H) @ W_ih (3H x F) at the C4
spatial-edge shape (T*B = 128 x 20480 rows, 3H = 768, F = 64) in a few formulations."""
import torch

dev = torch.device("cuda:0")
R, K, F = 128 * 20480, 768, 64
g = torch.Generator(device=dev).manual_seed(0)
dgi = torch.randn(R, K, device=dev, generator=g)
w = torch.randn(K, F, device=dev, generator=g) * 0.05


def a():
    return dgi @ w


def b():
    return (w.t() @ dgi.t()).t().contiguous()


def c():
    return torch.cat([x @ w for x in dgi.chunk(8)], 0)


def d():
    out = torch.empty(R, F, device=dev)
    for x, o in zip(dgi.chunk(16), out.chunk(16)):
        torch.mm(x, w, out=o)
    return out


ref = a()
for name, f in (("dgi @ w", a), ("(w^T dgi^T)^T", b), ("8 chunks", c), ("16 chunks", d)):
    for _ in range(2):
        y = f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        y = f()
    e1.record()
    e1.synchronize()
    print("%-16s %.3f ms  max|diff| %.2e" % (name, e0.elapsed_time(e1) / 5, (y - ref).abs().max().item()))
