"""Diagnostic (GPU box): count the norm-zone reward flips and path_violation mismatches between the HIP
engine and the oracle in the teacher-forced configurations of tests/test_gpu_parity.py, and dump the
pre-step state of every mismatching env (gpurun_out/flips_<name>.npz) for analysis on the CPU."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from crowdnav_dsrnn_amd import abi  # noqa: E402
from crowdnav_dsrnn_amd.engine import NumpyEngine  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from tests.test_gpu_parity import _cfg  # noqa: E402

CASES = [
    ("c5_traffic_normzones", "holonomic", 5, ("parallel_traffic", "perpendicular_traffic"), {"reward__norm_zones": True}),
    ("c5_side_pref", "holonomic", 1, ("side_pref_passing", "side_pref_overtaking", "side_pref_crossing"),
     {"test__side_preference": True, "sim__circle_radius": 4}),
    ("c2", "unicycle", 10, "circle_crossing", {}),
    ("c1", "holonomic", 5, "circle_crossing", {}),
    ("c3", "holonomic", 25, "square_crossing", {"robot__FOV": 1.0, "humans__FOV": 1.0}),
]


def main():
    out_dir = os.path.join(REPO, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    for name, kin, N, scen, over in CASES:
        cfg = _cfg(N, kin, scen, "orca", 1024, 2.0 if "FOV" not in str(over) else 1.0, **over)
        ref, g = cpu_ref.RefEngine(cfg), NumpyEngine(cfg, "cuda:0")
        ref.reset()
        rng = np.random.RandomState(5)
        flips = pv = 0
        dumps = []
        for t in range(60):  # noqa: B007
            a = (rng.uniform(-0.15, 0.15, (cfg.num_envs, 2)) if kin == "unicycle"
                 else rng.normal(0, 0.8, (cfg.num_envs, 2))).astype(np.float32)
            st = ref.get_state()
            g.set_state(st)
            r_out, g_out = ref.step(a), g.step(a)
            bad = np.zeros(cfg.num_envs, bool)
            if cfg.norm_zones:
                dr = np.abs(g_out[1].astype(np.float64) - r_out[1])
                f = np.abs(dr - abs(cfg.norm_zone_penalty)) < 1e-5
                flips += int(f.sum())
                bad |= f
            p = g_out[4][:, abi.INFO_PATH_VIOLATION] != r_out[4][:, abi.INFO_PATH_VIOLATION]
            pv += int(p.sum())
            bad |= p
            for e in np.nonzero(bad)[0][:50]:
                one = {}
                for n, _, _ in abi.STATE_FIELDS:
                    v = np.asarray(getattr(st, n))
                    if n != "mt" and v.size % cfg.num_envs == 0:
                        one[n] = v.reshape(cfg.num_envs, -1)[e]
                dumps.append((t, e, a[e], one,
                              g_out[4][e], r_out[4][e], g_out[1][e], r_out[1][e]))
        print("%-24s envs %d x 60 steps: norm-zone flips %d, path_violation mismatches %d"
              % (name, cfg.num_envs, flips, pv), flush=True)
        if dumps:
            np.savez(os.path.join(out_dir, "flips_%s.npz" % name),
                     t=np.array([d[0] for d in dumps]), e=np.array([d[1] for d in dumps]),
                     a=np.array([d[2] for d in dumps]), info_gpu=np.array([d[4] for d in dumps]),
                     info_ref=np.array([d[5] for d in dumps]), rew_gpu=np.array([d[6] for d in dumps]),
                     rew_ref=np.array([d[7] for d in dumps]),
                     **{"state_" + k: np.array([d[3][k] for d in dumps]) for k in dumps[0][3]})


if __name__ == "__main__":
    main()
