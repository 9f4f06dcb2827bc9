"""Attribute C4's GPU time to the operations that launch it.

Runs bench.py's C4 trainer (4096 envs x 10 humans, PPO 128 x 5 x 2) for one warmup update, then one update
under torch.profiler with shapes recorded, and prints, per (aten op, input shapes) -> kernel: calls, total
and mean device time, and for the GEMM-type ops the algorithmic FLOP and TFLOP/s. The innermost aten op
that launched a kernel is the one it is charged to; the Python call sites are in the stack column.

    python tools/prof_c4_ops.py [--envs 4096] [--top 40] > gpurun_out/c4_ops.log
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gemm_flop(name, shapes):
    try:
        if name in ("aten::mm", "aten::addmm"):
            a, b = (shapes[0], shapes[1]) if name == "aten::mm" else (shapes[1], shapes[2])
            return 2.0 * a[0] * a[1] * b[1]
        if name in ("aten::bmm", "aten::baddbmm"):
            a, b = (shapes[0], shapes[1]) if name == "aten::bmm" else (shapes[1], shapes[2])
            return 2.0 * a[0] * a[1] * a[2] * b[2]
    except (IndexError, TypeError):
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--part", choices=["all", "rollout"], default="all",
                    help="rollout: profile one eager rollout (collect) only")
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner import PPO
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer
    from crowdnav_dsrnn_amd.policy import Policy

    device = "cuda:0"
    E, N = args.envs, 10
    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.action_space.kinematics = "holonomic"
    c.training.num_processes = E
    c.ppo.num_steps, c.ppo.epoch, c.ppo.num_mini_batch = 128, 5, 2
    c.training.lr, c.training.eps, c.training.max_grad_norm = 4e-5, 1e-5, 0.5
    torch.manual_seed(0)
    envs = CrowdNavVecEnv(c, E, c.env.seed, device)
    pol = Policy(envs.observation_space.spaces, envs.action_space, base="srnn", base_kwargs=c).to(device)
    agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, c.ppo.num_mini_batch, c.ppo.value_loss_coef,
                c.ppo.entropy_coef, lr=c.training.lr, eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
    tr = RolloutTrainer(c, envs, pol, agent, graphs=args.part == "all")
    tr.update()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        if args.part == "rollout":
            tr.collect()
            torch.cuda.synchronize()
        else:
            st = tr.update()
            torch.cuda.synchronize()
            print("profiled update: rollout %.3f s, ppo %.3f s" % (st["rollout_s"], st["update_s"]))
    rows = collections.defaultdict(lambda: [0, 0.0, None])
    total = 0.0
    for ev in prof.events():
        ks = getattr(ev, "kernels", None) or []
        if not ks:
            continue
        shp = tuple(tuple(s) if isinstance(s, (list, tuple)) else s for s in (ev.input_shapes or []))
        for k in ks:
            key = (ev.name, str(shp)[:90], k.name[:70])
            r = rows[key]
            r[0] += 1
            r[1] += k.duration   # us
            r[2] = gemm_flop(ev.name, ev.input_shapes)
            total += k.duration
    print("device time attributed: %.1f ms" % (total / 1e3))
    print("%-16s %-90s %-70s %6s %10s %9s %8s" % ("op", "shapes", "kernel", "calls", "total ms", "mean us",
                                                  "TFLOP/s"))
    for key, (n, t, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:args.top]:
        tf = "%.1f" % (fl / (t / n * 1e-6) / 1e12) if fl else "-"
        print("%-16s %-90s %-70s %6d %10.2f %9.1f %8s" % (key[0][:16], key[1], key[2], n, t / 1e3, t / n, tf))
    envs.close()


if __name__ == "__main__":
    main()
