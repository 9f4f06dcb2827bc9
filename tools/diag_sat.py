"""Diagnostic: cn_debug_disc_quad modes 0 / 1 on the predicate test's cases, saved for a CPU-side diff."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from tests.test_norm_zone import _cases, _zone_cases  # noqa: E402

a, b = _cases(), _zone_cases()
px, py, r, qx, qy = (np.concatenate([u, v]) for u, v in zip(a, b))
dev = torch.device("cuda:0")
t = [torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(dev) for x in (px, py, r, qx, qy)]
L = _lib.lib()
res = {}
for mode in (0, 1):
    out = torch.zeros(len(px), dtype=torch.int32, device=dev)
    _lib.check(L.cn_debug_disc_quad(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), len(px), mode,
                                    *[x.data_ptr() for x in t], out.data_ptr()))
    res["m%d" % mode] = out.cpu().numpy()
np.savez("gpurun_out/sat_modes.npz", **res)
print({k: int(v.sum()) for k, v in res.items()})
