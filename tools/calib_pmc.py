"""FETCH_SIZE / WRITE_SIZE calibration on the step kernel's own access shape (run under rocprofv3 --pmc on
the GPU box; profiles/run_profile.sh does). cn_debug_copy64 moves a known number of bytes: 8 M doubles
(64 MiB each way, inside the 256 MiB Infinity Cache like the engine state) with one 8-B load + store per
lane, as full 64-lane segments (seg64) and as 6-lane (48-B) segments (seg6, a per-env field of one
workgroup). profiles/summarize.py divides the counters by the known bytes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from crowdnav_dsrnn_amd import _lib  # noqa: E402

N = 8 << 20
L = _lib.lib()
dev = torch.device("cuda:0")
src = torch.randn(N, dtype=torch.float64, device=dev)
dst = torch.empty_like(src)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
for seg in (64, 6):
    for _ in range(10):
        _lib.check(L.cn_debug_copy64(st, N, seg, src.data_ptr(), dst.data_ptr()))
    torch.cuda.synchronize(dev)
    assert torch.equal(dst, src)
print("calib ok: %d doubles per launch (%d bytes each way), seg 64 then seg 6, 10 launches each" % (N, N * 8))
