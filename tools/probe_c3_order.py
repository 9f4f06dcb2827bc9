"""Diagnostic (-DCN_STAMPS library): per-workgroup start / end of consecutive C3 launches on the device-wide
100 MHz clock, saved for an offline list-scheduling model (how much of the launch is the order in which
workgroups start, and how well one launch's workgroup durations predict the next one's).

    CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so python tools/probe_c3_order.py OUT.npz
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(out, E=4096, N=25, W=300, K=6):
    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
    c.action_space.kinematics = "holonomic"
    c.robot.FOV = c.humans.FOV = 1.0
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    a = torch.randn((W + K, E, 2), generator=g, device="cuda:0") * 0.5
    eng.reset()
    for s in range(W):
        eng.step(a[s])
    L = _lib.lib()
    L.cn_debug_stamps_r.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.cn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    runs, phases = [], []
    for k in range(K):
        eng.step(a[W + k])
        torch.cuda.synchronize()
        r = np.zeros(8192 * 2, np.uint64)
        L.cn_debug_stamps_r(r.ctypes.data_as(ctypes.c_void_p), None)
        runs.append(r.reshape(-1, 2)[:8192 - 7].astype(np.int64))
        sa, sb = np.zeros(4096 * 24, np.uint64), np.zeros(8192 * 24, np.uint64)
        L.cn_debug_stamps(sa.ctypes.data_as(ctypes.c_void_p), sb.ctypes.data_as(ctypes.c_void_p))
        phases.append(sa.reshape(-1, 24)[:, :7].astype(np.int64))   # per step workgroup: phase boundaries (cycles)
    st = eng.spawn_stats()
    np.savez(out, runs=np.stack(runs), phases=np.stack(phases), E=E, N=N)
    R = runs[-1]
    live = np.nonzero(R[:, 1] > 0)[0]
    nb = live.max() + 1
    t0 = R[:nb, 0].min()
    print("workgroups %d, last launch span %.1f us, stats %s" % (nb, (R[:nb, 1].max() - t0) / 100.0, st))
    eng.close()


if __name__ == "__main__":
    main(sys.argv[1])
