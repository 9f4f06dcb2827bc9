"""Diagnostic: the fixed cost of bench.py's short window (--steps 20 --warmup 5) under the HIP runtime's host
synchronisation modes. A window's wall time = the K launches' span on the GPU (HIP events) + a fixed part:
host -> first kernel, last kernel -> host wake-up. `spin` calls hipSetDeviceFlags(hipDeviceScheduleSpin) on
torch's HIP runtime before the device is initialised, so synchronisation polls instead of sleeping.

    python tools/probe_sync.py [auto|spin|yield|blocking] [windows]
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

MODE = sys.argv[1] if len(sys.argv) > 1 else "auto"
FLAGS = {"auto": None, "spin": 1, "yield": 2, "blocking": 4}
if FLAGS[MODE] is not None:
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    print("hipSetDeviceFlags(%d) -> %d" % (FLAGS[MODE], hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[MODE]))))

from crowdnav_dsrnn_amd import _lib  # noqa: E402
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config  # noqa: E402
from crowdnav_dsrnn_amd.engine import CrowdNavEngine  # noqa: E402


def main(windows=8, K=20, W=5, E=4096):
    c = clone_config(Config())
    c.sim.human_num = 10
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E, nenv=E, phase="train"), "cuda:0")
    L = _lib.lib()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = (torch.rand((W + K, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1).contiguous()
    walls, spans = [], []
    for w in range(windows + 1):
        eng.reset()
        eng.step_seq(acts[:W])
        _lib.check(L.cn_profile(eng._h, 1, K))
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step_seq(acts[W:])
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        _lib.check(L.cn_profile(eng._h, 0, 0))
        walls.append(wall * 1e6)   # (window 0 included: it shows the first window's extra cost)
        spans.append(a.value * 1e3)
    print("windows in order (wall / span us): " + ", ".join("%.0f/%.0f" % (a, b) for a, b in zip(walls, spans)))
    walls, spans = sorted(walls), sorted(spans)
    fixed = sorted(x - y for x, y in zip(walls, spans))
    print("%s: wall us median %.1f min %.1f | kernel span median %.1f | fixed median %.1f min %.1f | value median %.2f M"
          % (MODE, walls[len(walls) // 2], walls[0], spans[len(spans) // 2], fixed[len(fixed) // 2], fixed[0],
             E * K / walls[len(walls) // 2]))


if __name__ == "__main__":
    main(int(sys.argv[2]) if len(sys.argv) > 2 else 8)
