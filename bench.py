"""bench.py — env-steps/sec of the batched CrowdSimDict hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--humans H] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): per GPU 4096 envs x 10 humans, circle_crossing,
ORCA humans, unicycle robot, dt = 0.25, reference config defaults (randomize_attributes, goal
changing, auto-reset). A "step" is one cn_step of every env: clip_action, ORCA for every human,
calc_reward, kinematics, observation, goal changes, auto-reset of finished envs. Actions: synthetic
U[-0.1, 0.1]^2 (dv, dtheta), generated on the device (torch Philox, seed = rank) BEFORE the timed
region, so the timed region only runs the env hot path with inputs resident in HBM.
Multi-GPU: envs shard with no collective (env g of rank r is global env r*E+g; thisSeed/nenv are
global) -> weak scaling; timing = max over ranks between barriers.
One JSON line on rank 0 (bench contract in the task statement).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def algorithmic_bytes_per_env_step(N):
    """B_step(N) = 2*(S_r + N*S_h) + 8 (action) + 4*(9 + 2N) (obs) + 4 (reward) + 2 (done, event),
    S_r = 112 B, S_h = 96 B  ->  2,274 B at N = 10."""
    return 2 * (112 + 96 * N) + 8 + 4 * (9 + 2 * N) + 4 + 2


def make_config(E, N, env_offset, nenv):
    from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.sim.test_sim = ["circle_crossing"]
    c.humans.policy = "orca"
    c.action_space.kinematics = "unicycle"
    return make_cn_config(c, num_envs=E, env_offset=env_offset, nenv=nenv, phase="train")


def cpu_baseline(N, budget_s=12.0):
    """The oracle (C restatement of the reference step, oracle/cpu_ref.c) on ONE host core, bounded
    sample of the same workload: 256 envs, steps until ~budget_s of CPU time."""
    from oracle import cpu_ref

    cpu_ref.lib().cnref_set_threads(1)
    E = 256
    cfg = make_config(E, N, 0, 4096)
    eng = cpu_ref.RefEngine(cfg)
    eng.reset()
    rng = np.random.RandomState(0)
    steps = 0
    t0 = time.perf_counter()
    while True:
        eng.step(rng.uniform(-0.1, 0.1, (E, 2)).astype(np.float32))
        steps += 1
        el = time.perf_counter() - t0
        if el > budget_s or steps >= 50000:
            break
    return {"value": E * steps / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "oracle/cpu_ref.c (C restatement of CrowdSimDict.step incl. RVO2 ORCA), 1 thread, "
                      "%d envs x %d steps of the same C2 workload (%.1f s)" % (E, steps, el)}


def load_pmc_traffic():
    """HBM bytes per step-kernel launch from the committed rocprofv3 --pmc summary (profiles/), or None."""
    p = os.path.join(REPO, "profiles", "pmc_step_kernel.json")
    if not os.path.exists(p):
        return None
    try:
        return float(json.load(open(p))["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--humans", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    from crowdnav_dsrnn_amd import _lib
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    E, N, K, W = args.envs, args.humans, args.steps, args.warmup
    cfg = make_config(E, N, env_offset=rank * E, nenv=E * world)
    eng = CrowdNavEngine(cfg, device)
    gen = torch.Generator(device=device)
    gen.manual_seed(rank)
    actions = (torch.rand((K + W, E, 2), generator=gen, device=device) * 0.2 - 0.1).contiguous()
    eng.reset()
    for s in range(W):
        eng.step(actions[s])
    L = _lib.lib()

    def barrier():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)

    _lib.check(L.cn_profile(eng._h, 1, K))
    barrier()
    t0 = time.perf_counter()
    for s in range(K):
        eng.step(actions[W + s])
    barrier()
    elapsed = time.perf_counter() - t0
    a_ms, b_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a_ms), ctypes.byref(b_ms), ctypes.byref(n)))
    _lib.check(L.cn_profile(eng._h, 0, 0))
    done_frac = float(eng.done.float().mean().item())
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        value = world * E * K / elapsed
        kernel_s = a_ms.value / 1e3 / max(n.value, 1)
        bpl = algorithmic_bytes_per_env_step(N) * E
        achieved = bpl / kernel_s / 1e9
        traffic = load_pmc_traffic()
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(elapsed / K * 1e3, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": "C2: %d envs/GPU x %d humans, circle_crossing, ORCA humans (RVO2 f32), unicycle robot, "
                            "dt=0.25, actions U[-0.1,0.1]^2, auto-reset" % (E, N),
                "envs_per_gpu": E, "humans": N, "global_envs": E * world,
                "parallelism": "env-sharded x%d (no collective)" % world,
                "step_kernel_ms": round(kernel_s * 1e3, 5),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "kernel": "cn_step_kernel",
                "algorithmic_bytes_per_launch": bpl,
            },
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(N, args.cpu_budget)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
