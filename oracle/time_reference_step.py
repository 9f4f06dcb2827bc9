"""Time the REFERENCE's own CrowdSimDict.step() in this container; build
container only (the reference never travels to the GPU box). Writes profiles/cpu_reference_step.json.

    python oracle/time_reference_step.py [--seconds 20]

What is timed, on ONE core of this container (taskset is not used; the process is single-threaded:
OMP/MKL threads pinned to 1 before numpy loads):
  (ii)  the reference's CrowdSimDict.step() (crowd_sim_dict.py:205-271) of ONE env, with the VecEnv
        worker's auto-reset (shmem_vec_env.py:164-168) — social-force humans, because ORCA needs the
        absent RVO2 C++ library (its Python stand-in in oracle/shims would time a Python restatement, not
        the reference); N = 10, circle_crossing, holonomic robot (the unicycle path crashes in calc_reward
        at HEAD), reference config defaults otherwise. shapely is absent too: its calls run
        through the analytic shim (oracle/shims/shapely), and the share of step time spent inside the
        shim is measured with cProfile and reported so the reader can discount it.
  (iii) the build's C restatement (oracle/cpu_ref.c) of the same step on the same config, 1 thread,
        256 envs: the calibration ratio (ii)/(iii) lets bench.py's GPU-box timing of cpu_ref stand for
        the reference's Python step on that host.
"""
import argparse
import cProfile
import json
import os
import pstats
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import gen_golden as G  # noqa: E402  (imports the reference through the shims)


def ref_steps(cfg, seconds, seed=1):
    env = G.make_ref_env(cfg, 0, 16)
    G.env_reset(env)
    rng = np.random.RandomState(seed)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        G.env_step(env, rng.normal(0, 0.5, 2).astype(np.float32))
        n += 1
    return n, time.perf_counter() - t0


def oracle_rate(N, seconds):
    from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config
    from oracle import cpu_ref

    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "social_force"
    c.action_space.kinematics = "holonomic"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    E = 256
    cfg = make_cn_config(c, num_envs=E, nenv=E, phase="train")
    cpu_ref.lib().cnref_set_threads(1)
    eng = cpu_ref.RefEngine(cfg)
    eng.reset()
    rng = np.random.RandomState(0)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        eng.step(rng.normal(0, 0.5, (E, 2)).astype(np.float32))
        n += 1
    return E * n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--humans", type=int, default=10)
    args = ap.parse_args()
    cfg = G.make_ref_config(kin="holonomic", policy="social_force", N=args.humans)
    n, el = ref_steps(cfg, args.seconds)
    ref_rate = n / el
    # shim share: profile a shorter run and sum the time spent in oracle/shims/shapely
    prof = cProfile.Profile()
    prof.enable()
    n2, el2 = ref_steps(cfg, min(5.0, args.seconds / 4), seed=2)
    prof.disable()
    st = pstats.Stats(prof)
    shim = sum(v[2] for k, v in st.stats.items() if "shims" in k[0] and "shapely" in k[0])   # tottime
    total = sum(v[2] for v in st.stats.values())
    orc = oracle_rate(args.humans, args.seconds / 2)
    doc = {
        "what": "reference CrowdSimDict.step() (social-force humans, N=%d, circle_crossing, holonomic, 1 env, "
                "auto-reset) timed in the build container on 1 core; oracle/cpu_ref.c on the same config "
                "(1 thread, 256 envs) for calibration" % args.humans,
        "host_nproc": os.cpu_count(),
        "cores": 1,
        "reference_env_steps_per_s": ref_rate,
        "reference_ms_per_step": 1e3 / ref_rate,
        "reference_steps_timed": n,
        "shapely_shim_time_frac": shim / total if total else None,
        "oracle_env_steps_per_s_1thread": orc,
        "ratio_oracle_over_reference": orc / ref_rate,
        "note": "ORCA cannot be timed here (RVO2 absent); shapely runs through the analytic Python shim "
                "(its share of step time is shapely_shim_time_frac; GEOS would be faster).",
    }
    out = os.path.join(REPO, "profiles", "cpu_reference_step.json")
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
