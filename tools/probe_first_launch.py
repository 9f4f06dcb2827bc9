"""Diagnostic: the first kernel launches of the HIP library in a fresh process (round-3 NoDevice probe)."""
import ctypes
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np  # noqa: E402

from oracle import cpu_ref  # noqa: E402

cpu_ref.lib()
print("oracle loaded", flush=True)
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config  # noqa: E402
from crowdnav_dsrnn_amd.policy_factory import FullState, JointState, ObservableState, policy_factory  # noqa: E402

L = _lib.lib()
print("version", L.cn_version().decode(), flush=True)
c = clone_config(Config())
p = policy_factory["orca"](c)
st = JointState(FullState(0, 0, 0, 0, 0.3, 3, 3, 1.0, 0), [ObservableState(1, 1, 0, 0, 0.3)])
try:
    print("predict", p.predict(st), flush=True)
except Exception as e:
    print("predict failed:", e, flush=True)
import torch  # noqa: E402
src = torch.arange(64, dtype=torch.float64, device="cuda")
dst = torch.zeros_like(src)
st_ = torch.cuda.current_stream().cuda_stream
print("copy64 rc", L.cn_debug_copy64(ctypes.c_void_p(st_), 64, 64, src.data_ptr(), dst.data_ptr()), L.cn_last_error(), flush=True)
print("predict again", p.predict(st), flush=True)
