"""bench.py — env-steps/sec of the batched CrowdSimDict hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--humans H] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`python bench.py --gpus N` (N > 1) without WORLD_SIZE launches the N rank processes itself (a child
torch.distributed.run on 127.0.0.1, before this process touches the GPU) and exits with its code -- the
reference builds its whole worker pool from one make_vec_envs call (envs.py:120-139). Under a launcher,
--gpus must equal WORLD_SIZE.

Workload (BASELINE.json configs[1]): per GPU 4096 envs x 10 humans, circle_crossing,
ORCA humans, unicycle robot, dt = 0.25, reference config defaults (randomize_attributes, goal
changing, auto-reset). A "step" is one cn_step of every env: clip_action, ORCA for every human,
calc_reward, kinematics, observation, goal changes, auto-reset of finished envs. Actions: synthetic
U[-0.1, 0.1]^2 (dv, dtheta), generated on the device (torch Philox, seed = rank) BEFORE the timed
region, so the timed region only runs the env hot path with inputs resident in HBM.
Multi-GPU: envs shard with no collective (env g of rank r is global env r*E+g; thisSeed/nenv are
global) -> weak scaling; timing = max over ranks between barriers.
One JSON line on rank 0 (bench contract in the task statement). The main window is the K launches after
W warm-up launches after cn_reset (the driver's --steps 20 --warmup 5: launches 6-25 of the first
episodes, few auto-resets); `steady_state` in the same line is SURVEY §8d's window on the same engine:
100 more warm-up launches, then 2,000 timed ones including all their auto-resets (`resets` = episodes
ended and restarted inside the window, counted from the engine's per-env reset counters).
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
WORKLOAD_DESC = {
    "c2": "C2: %d envs/GPU x %d humans, circle_crossing, ORCA humans (RVO2 f32), unicycle robot, dt=0.25, "
          "actions U[-0.1,0.1]^2, auto-reset",
    "c3": "C3: %d envs/GPU x %d humans, square_crossing, robot/human FOV pi, ORCA humans (kd-tree path), "
          "holonomic robot, actions N(0,0.5^2), auto-reset",
    "c4": "C4: %d envs/GPU x %d humans, circle_crossing, ORCA humans, holonomic robot, DSRNN act() in the loop "
          "(sampled actions), PPO num_steps=128 epochs=5 minibatches=2",
    "c5": "C5: %d envs/GPU in ONE mixed engine, per-env scenario dispatch round-robin over parallel / "
          "perpendicular traffic (%s humans) and the 3 side_pref scenarios (1 human, padded), norm-zone reward, "
          "holonomic, ORCA",
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def algorithmic_bytes_per_env_step(N):
    """B_step(N) = 2*(S_r + N*S_h) + 8 (action) + 4*(9 + 2N) (obs) + 4 (reward) + 2 (done, event),
    S_r = 112 B, S_h = 96 B  ->  2,274 B at N = 10."""
    return 2 * (112 + 96 * N) + 8 + 4 * (9 + 2 * N) + 4 + 2


DIAG = None   # --diag (counter attribution runs only, never the line of record): "nogoal" = no goal changing


def make_config(E, N, env_offset, nenv, workload="c2", rng="mt19937"):
    """SURVEY.md §8d workloads. c2 (default, the BASELINE metric): circle_crossing, ORCA, unicycle.
    c3: square_crossing ("random crossing"), robot/human FOV = pi, holonomic. c5: c5_mixed."""
    from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    if DIAG == "nogoal":
        c.humans.random_goal_changing = c.humans.end_goal_changing = False
    if workload == "c3":
        c.sim.train_val_sim = c.sim.test_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
    else:
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        c.action_space.kinematics = "unicycle"
    return make_cn_config(c, num_envs=E, env_offset=env_offset, nenv=nenv, phase="train", rng=rng)


C5_SCENARIOS = ["parallel_traffic", "perpendicular_traffic", "side_pref_passing", "side_pref_overtaking",
                "side_pref_crossing"]


def c5_scenario_configs():
    """{scenario: reference-style config}. Traffic scenarios: N = 5; the side-preference
    scenarios: N = 1, circle radius 4, fixed robot (0, -4) -> (0, 4), no goal changing (config.py:37-40,
    95,99; crowd_sim.py:642-651). Norm-zone reward ("social-metric reward") everywhere,
    holonomic robot, ORCA humans."""
    from crowdnav_dsrnn_amd.config import Config, clone_config

    out = {}
    for scen, n in (("traffic", 5), ("side_pref", 1)):
        c = clone_config(Config())
        c.sim.human_num = n
        c.humans.policy = "orca"
        c.action_space.kinematics = "holonomic"
        c.reward.norm_zones = True
        if n == 1:
            c.test.side_preference = True
            c.sim.circle_radius = 4
            c.humans.random_goal_changing = False
            c.humans.end_goal_changing = False
        for s in C5_SCENARIOS:
            if s.startswith("side_pref") == (scen == "side_pref"):
                out[s] = c
    return out


def c5_mixed(E, env_offset, nenv, rng="mt19937"):
    """(group cn_configs, env_group) of the C5 mixed engine: env r runs C5_SCENARIOS[(env_offset + r) % 5]
    (round-robin by global env index) with that scenario's human count."""
    from crowdnav_dsrnn_amd.config import make_mixed_cn_configs

    return make_mixed_cn_configs(c5_scenario_configs(), C5_SCENARIOS, E, env_offset=env_offset, nenv=nenv,
                                 phase="train", rng=rng)


def _oracle_rate(cfg, budget_s, threads, kind="uniform"):
    """env-steps/s of oracle/cpu_ref.c on `cfg` with `threads` OpenMP threads over envs, ~budget_s."""
    from oracle import cpu_ref

    cpu_ref.lib().cnref_set_threads(threads)
    E = cfg.num_envs
    eng = cpu_ref.RefEngine(cfg)
    eng.reset()
    rng = np.random.RandomState(0)
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = rng.uniform(-0.1, 0.1, (E, 2)) if kind == "uniform" else rng.normal(0, 0.5, (E, 2))
        eng.step(a.astype(np.float32))
        steps += 1
        el = time.perf_counter() - t0
        if el > budget_s or steps >= 50000:
            break
    return E * steps / el, steps, el


def host_threads():
    """CPU threads this process may use: the box's share (OMP_NUM_THREADS = 16 there), else the affinity."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else n


def cpu_baseline(N, budget_s=12.0):
    """SURVEY §8d CPU legs on the GPU box's host, bounded samples of the same C2 workload:
    value = oracle/cpu_ref.c (C restatement of CrowdSimDict.step incl. RVO2 ORCA) with an OpenMP loop
    over envs on all the host threads this job may use; one_thread = the same on 1 thread; and the
    reference's own Python step, estimated as cpu_ref(social force, 1 thread, timed here) / the
    cpu_ref-over-reference ratio measured in the build container (profiles/cpu_reference_step.json,
    oracle/time_reference_step.py: ORCA needs the absent RVO2, so the reference is timed with social force)."""
    from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

    T = host_threads()
    E_all = 4096   # the C2 workload itself: the OpenMP loop over envs amortises its per-step fork/join
    all_rate, all_steps, all_el = _oracle_rate(make_config(E_all, N, 0, 4096), budget_s * 0.5, T)
    one_rate, one_steps, one_el = _oracle_rate(make_config(256, N, 0, 4096), budget_s * 0.3, 1)
    out = {"value": all_rate, "unit": "env-steps/s", "cores": T, "kind": "port",
           "sample": "oracle/cpu_ref.c (C restatement of CrowdSimDict.step incl. RVO2 ORCA), OpenMP over envs on "
                     "%d threads, %d envs x %d steps of the same C2 workload (%.1f s)" % (T, E_all, all_steps, all_el),
           "one_thread": {"value": one_rate, "cores": 1,
                          "sample": "same, 1 thread, 256 envs x %d steps (%.1f s)" % (one_steps, one_el)}}
    cal = os.path.join(REPO, "profiles", "cpu_reference_step.json")
    if os.path.exists(cal):
        doc = json.load(open(cal))
        c = clone_config(Config())
        c.sim.human_num = 10
        c.humans.policy = "social_force"
        c.action_space.kinematics = "holonomic"
        c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
        sf_rate, _, _ = _oracle_rate(make_cn_config(c, num_envs=256, nenv=256, phase="train"), budget_s * 0.2, 1,
                                     kind="normal")
        out["reference_python_estimate"] = {
            "value": sf_rate / doc["ratio_oracle_over_reference"], "cores": 1,
            "sample": "reference CrowdSimDict.step (social force, N=10, 1 env, 1 core): %.1f env-steps/s timed in the "
                      "build container; scaled to this host by cpu_ref(social force) here / there (ratio %.1f)"
                      % (doc["reference_env_steps_per_s"], doc["ratio_oracle_over_reference"])}
    return out


def load_pmc(kernel="cn_step_kernel", workload="c2", window=None):
    """Counter figures for `kernel` from the newest committed rocprofv3 summary (profiles/pmc_<tag>.json,
    written by profiles/summarize.py) that was measured on a library built from EXACTLY the sources this
    run uses (CN_SRC_HASH) and on the same workload; None when no such profile exists (a stale profile
    is never reported). window = (first, count): the figures of exactly those launches after cn_reset
    (0-based first launch), which the profile must have split out (summarize.py `windows`); a profile of
    another window is not reported for this one."""
    import glob

    from crowdnav_dsrnn_amd import build

    want = build.source_hash()
    best = None
    for p in glob.glob(os.path.join(REPO, "profiles", "pmc_*.json")):
        try:
            doc = json.load(open(p))
        except Exception:
            continue
        if doc.get("lib_src_hash") != want:
            continue
        wl = "c2"
        a = doc.get("bench_args", "").split()
        if "--diag" in a:   # an attribution run of a modified workload: never reported
            continue
        if "--workload" in a:
            wl = a[a.index("--workload") + 1]
        if wl != workload:
            continue
        for k, d in doc.get("kernels", {}).items():
            if kernel not in k:
                continue
            if window is not None:
                d = next((w for w in d.get("windows", []) if (w.get("first"), w.get("count")) == tuple(window)), None)
                if d is None:
                    continue
            if "hbm_bytes_per_launch" in d:
                if best is None or os.path.getmtime(p) > best[0]:
                    best = (os.path.getmtime(p), doc["tag"], d)
    if best is None:
        return None
    _, tag, d = best
    return {"tag": tag, "traffic": d["hbm_bytes_per_launch"], "valu_issue_frac": d.get("valu_issue_frac"),
            "active_inst_frac": d.get("active_inst_frac"), "avg_duration_ns": d.get("avg_duration_ns")}


FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_{32x32x2,16x16x4}_f32, dense, no TF32 on gfx950


def gru_gemm_roofline(torch, device, B, H, reps=50):
    """Roofline of C4's dominant forward kernel: the per-step fused recurrent step of the spatial-edge GRU
    in the PPO update (ops._MaskedGRU -> cn_gru_fwd_fused: gh = hm W_hh^T + b_hh on the f32 MFMA with the
    gate epilogue, B = envs per minibatch x humans rows, K = H = 256, 3H = 768 columns; 128 steps x 5 epochs
    x 2 minibatches per update). The same call on the same shapes (save record and next masked state
    written, as in training) is timed with HIP events on the stream it runs on; algorithmic FLOP per launch
    = 2 B H 3H (the gate arithmetic is not counted). The unfused pair it replaced (hipBLASLt addmm +
    cn_gru_fwd_step) is timed beside it."""
    from crowdnav_dsrnn_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device=device)
    g.manual_seed(1)
    hm = torch.randn((B, H), generator=g, device=device)
    w = torch.randn((3 * H, H), generator=g, device=device) * 0.05
    b = torch.randn((3 * H,), generator=g, device=device)
    gi = torch.randn((B, 3 * H), generator=g, device=device)
    m = torch.ones((B,), device=device)
    h_out = torch.empty((B, H), device=device)
    hm_next = torch.empty((B, H), device=device)
    save = torch.empty((B, 4 * H), device=device)
    gh = torch.empty((B, 3 * H), device=device)
    st = torch.cuda.current_stream(device).cuda_stream

    def fused():
        _lib.check(L.cn_gru_fwd_fused(st, B, H, gi.data_ptr(), hm.data_ptr(), w.data_ptr(), b.data_ptr(),
                                      m.data_ptr(), h_out.data_ptr(), hm_next.data_ptr(), save.data_ptr(), None, 1, 0))

    def pair():
        torch.addmm(b, hm, w.t(), out=gh)
        _lib.check(L.cn_gru_fwd_step(st, B, H, gi.data_ptr(), gh.data_ptr(), hm.data_ptr(), m.data_ptr(),
                                     h_out.data_ptr(), hm_next.data_ptr(), save.data_ptr()))

    def timed(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / reps

    dt, dt_pair = timed(fused), timed(pair)
    flop = 2.0 * B * H * 3 * H
    tf = flop / dt / 1e12
    return {"bound": "mfma", "achieved": round(tf, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tf / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
            "kernel": "spatial-edge GRU fused step cn_gru_fwd_fused (gh = hm W_hh^T + b_hh on the fp32 MFMA + gates), "
                      "%d x %d -> %d" % (B, H, 3 * H),
            "flop_per_launch": flop, "avg_launch_us": round(dt * 1e6, 2),
            "unfused_addmm_plus_gates_us": round(dt_pair * 1e6, 2)}


def dsrnn_flop_per_env_step(N, c):
    """Algorithmic forward FLOP of the DSRNN policy per env-step (srnn_model.py:409-504 with the config's
    sizes): 2*M*K per output of every Linear / GRU gate GEMM (gi and gh), attention scores and pooling;
    the elementwise gate / activation arithmetic is not counted. 6.63 MFLOP at N = 10. This is the
    reference's algorithm: ops.spatial_attention reassociates the spatial_edge_layer term (2*He*A*N of `att`,
    0.33 MFLOP at N = 10) into 2*A*He + 2*He*N, so ~5 % of the count is no longer executed."""
    S = c.SRNN
    He, Hn, emb = S.human_human_edge_rnn_size, S.human_node_rnn_size, S.human_human_edge_embedding_size
    enc = 2 * 2 * emb * (N + 1) + 2 * 7 * 3 + 2 * 3 * S.human_node_embedding_size
    edge_gru = 2 * emb * 3 * He + 2 * He * 3 * He                  # gi + gh per edge row
    att = 2 * He * S.attention_size * (N + 1) + 2 * S.attention_size * N + 2 * He * N
    node_in = 2 * S.human_node_embedding_size
    node = 2 * (2 * He) * S.human_node_embedding_size + 2 * node_in * 3 * Hn + 2 * Hn * 3 * Hn + 2 * Hn * S.human_node_output_size
    out = S.human_node_output_size
    heads = 2 * (2 * out * out) + 2 * (2 * out * out) + 2 * out + 2 * out * 2
    return enc + (N + 1) * edge_gru + att + node + heads


def run_c4(torch, dist, device, rank, world, E, N, K, W):
    """env-steps/s over PPO updates, counted like train.py:342-352 (rollout of num_steps
    steps of every env with DSRNN act() in the loop, then the PPO update, all inside the timed region).
    A "step" here is one update = 128 x E env steps per GPU; W untimed updates first (the first eager,
    the second captures the rollout's HIP graph), then K timed ones. Returns the line's dict on rank 0
    (None elsewhere)."""
    from crowdnav_dsrnn_amd import ops
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner import PPO
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer
    from crowdnav_dsrnn_amd.policy import Policy

    c = clone_config(Config())
    c.sim.human_num = N
    c.humans.policy = "orca"
    c.sim.train_val_sim = c.sim.test_sim = ["circle_crossing"]
    c.action_space.kinematics = "holonomic"
    c.training.num_processes = E
    c.ppo.num_steps = 128
    c.ppo.epoch = 5
    c.ppo.num_mini_batch = 2
    c.training.lr = 4e-5
    c.training.eps = 1e-5
    c.training.max_grad_norm = 0.5
    torch.manual_seed(0)
    envs = CrowdNavVecEnv(c, E, c.env.seed, device, env_offset=rank * E, nenv=E * world)
    pol = Policy(envs.observation_space.spaces, envs.action_space, base="srnn", base_kwargs=c).to(device)
    agent = PPO(pol, c.ppo.clip_param, c.ppo.epoch, c.ppo.num_mini_batch, c.ppo.value_loss_coef,
                c.ppo.entropy_coef, lr=c.training.lr, eps=c.training.eps, max_grad_norm=c.training.max_grad_norm)
    tr = RolloutTrainer(c, envs, pol, agent)

    for _ in range(W):
        tr.update()
    _barrier(torch, dist, device)
    ops.FUSED_TIMING = []   # in-loop HIP events around the spatial-edge GRU's fused steps (its stream)
    t0 = time.perf_counter()
    roll = upd = 0.0
    episodes = 0
    for _ in range(K):
        st = tr.update()
        roll += st["rollout_s"]
        upd += st["update_s"]
        episodes += st["episodes"]
        if rank == 0:
            print("c4 update: rollout %.3f s, ppo %.3f s, episodes %d, mean return %.3f, value_loss %.4f"
                  % (st["rollout_s"], st["update_s"], st["episodes"], st["mean_episode_return"],
                     st["value_loss"]), file=sys.stderr, flush=True)
    _barrier(torch, dist, device)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed, float(episodes)], dtype=torch.float64, device=device)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, episodes = float(t[0].item()), int(t[1].item())
    timing, ops.FUSED_TIMING = ops.FUSED_TIMING, None
    roof = gru_gemm_roofline(torch, device, E // c.ppo.num_mini_batch * N, 256) if rank == 0 else None
    if rank == 0 and timing:
        # the roofline of record: the same kernel timed IN the loop (all its launches of the timed updates)
        n_launch = sum(t[2] for t in timing)
        secs = sum(t[3].elapsed_time(t[4]) for t in timing) / 1e3
        B0, H0, F0 = timing[0][0], timing[0][1], timing[0][5]
        flop = 2.0 * B0 * (H0 + F0) * 3 * H0   # recurrent GEMM + the in-kernel input projection (F0 > 0)
        iso = roof
        tf = flop * n_launch / secs / 1e12
        roof = dict(iso, achieved=round(tf, 3), frac=round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
                    avg_launch_us=round(secs / n_launch * 1e6, 2), launches_timed=n_launch,
                    kernel="edge-RNN fused step of the PPO forward (cn_gru_fwd_seq: the spatial and temporal edge GRUs, "
                           "%d rows per launch; x W_ih^T (F = %d) + hm W_hh^T + b on the fp32 MFMA, gates in the "
                           "epilogue)" % (B0, F0),
                    flop_per_launch=flop,
                    method="HIP events around every training forward's fused-step loop, on its stream, inside "
                           "the timed updates",
                    isolated_kernel=iso["kernel"], isolated_flop_per_launch=iso["flop_per_launch"],
                    isolated_avg_launch_us=iso["avg_launch_us"])
    line = None
    if rank == 0:
        steps_per_update = c.ppo.num_steps * E
        fps = dsrnn_flop_per_env_step(N, c)
        # rollout forward + PPO epochs x (forward + 2x backward) over every env-step of the update
        upd_flop = steps_per_update * fps * (1 + 3 * c.ppo.epoch)
        upd_s = elapsed / K
        whole = {"flop_per_update": upd_flop, "flop_per_env_step_fwd": fps,
                 "achieved": round(upd_flop / upd_s / 1e12, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(upd_flop / upd_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}
        line = {
            "metric": METRIC + " [C4 side measurement: incl. DSRNN act + PPO update]",
            "value": round(world * steps_per_update * K / elapsed, 1),
            "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64 env / fp32 policy", "data": "synthetic",
            "config": {"workload": WORKLOAD_DESC["c4"] % (E, N) + (", grads all-reduced over RCCL" if world > 1 else ""),
                       "envs_per_gpu": E, "humans": N,
                       "global_envs": E * world, "env_steps_per_update": steps_per_update * world,
                       "rollout_s_per_update": round(roll / K, 4), "ppo_s_per_update": round(upd / K, 4),
                       "rollout_timing": "HIP events on the update's stream (rollout = act + cn_step + storage, "
                                         "incl. get_value / compute_returns; ppo = PPO.update)",
                       "resets": episodes,
                       "parallelism": "dp%d (env-sharded%s)" % (world, ", PPO grads all-reduced" if world > 1 else "")},
            "roofline": roof,
            "whole_update_roofline": whole,
        }
    envs.close()
    del tr, agent, pol, envs
    torch.cuda.empty_cache()
    return line


def _barrier(torch, dist, device):
    # (device is the current device, torch.cuda.set_device in main: the plain synchronize skips the
    # device-guard switch; one rank needs no second synchronize -- it ended a timed window with ~5 us of
    # host overhead)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()


def reset_total(eng):
    """Sum over envs of the engine's per-env reset counter (state field reset_count: one per auto-reset
    inside cn_step, crowd_sim_dict.py:105 via shmem_vec_env.py:166-167). Host copy of the state, outside
    any timed region."""
    st = eng.get_state()
    views = [v for _, v in st] if isinstance(st, list) else [st]
    return int(sum(int(v.reset_count.astype(np.int64).sum()) for v in views))


def reset_total_dev(eng):
    """reset_total of a plain engine from its reset_count field alone: the E x 4 bytes of that field are
    copied on the device by the engine library itself (cn_debug_copy64, stream-ordered after the steps) into
    a torch tensor and summed there, so the window that follows does not start behind a 15 MB pageable
    state copy and no second handle on the HIP runtime is needed; mixed engines fall back to reset_total."""
    import torch

    from crowdnav_dsrnn_amd import _lib, abi

    if eng.groups is not None:
        return reset_total(eng)
    off = abi.state_layout(eng.E, eng.N, eng.cfg.robot_visible)[0]["reset_count"][0]
    base = _lib.lib().cn_state_device_ptr(eng._h)
    n64 = (eng.E + 1) // 2   # the field is padded to 256 B: the odd-E tail word stays inside it
    buf = torch.empty((2 * n64,), dtype=torch.int32, device=eng.device)
    with torch.cuda.device(eng.device):
        st = ctypes.c_void_p(torch.cuda.current_stream(eng.device).cuda_stream)
        _lib.check(_lib.lib().cn_debug_copy64(st, n64, 64, ctypes.c_void_p(base + off), ctypes.c_void_p(buf.data_ptr())))
    return int(buf[:eng.E].to(torch.int64).sum().item())


def launch_plan(gpus, environ):
    """How this invocation runs: ("run", world) inside a launcher (or a plain 1-GPU run), ("spawn", N) when
    `--gpus N` > 1 is asked for without WORLD_SIZE (bench.py then starts the N ranks itself), or
    ("error", message) when --gpus and the launcher's WORLD_SIZE disagree (never a silent n_gpus: 1 line)."""
    if gpus < 1:
        return ("error", "--gpus must be >= 1, got %d" % gpus)
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return ("spawn", gpus) if gpus > 1 else ("run", 1)
    if int(ws) != gpus:
        return ("error", "--gpus %d but the launcher started WORLD_SIZE=%s ranks" % (gpus, ws))
    return ("run", gpus)


def spawn_ranks(n, argv):
    """Start `python -m torch.distributed.run --nproc-per-node n ... bench.py argv` as a CHILD process
    (this process has not touched the GPU: no exec after GPU init) and return its exit code."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """--dry-run: the launcher and the rank bookkeeping without a GPU (gloo; CPU tests): every rank joins,
    the max-over-ranks reduction runs, rank 0 prints the line's launcher fields."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "max_over_ranks": float(t.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_env(torch, dist, device, rank, world, workload, E, N, K, W, steady, rng="mt19937", launch="seq"):
    """The env hot path alone (c2 / c3 / c5): W untimed launches after cn_reset, then K timed ones
    (barrier + synchronize on both sides, max over ranks); with `steady` also SURVEY §8d's window on the
    same engine (100 more warm-up launches, then 2,000 timed ones). launch = "seq" (default): each timed
    window is one cn_step_seq call over its K pre-drawn actions (the K launches go out back to back from
    native code, so the window measures the GPU and not the host's Python call rate); "host": Python
    issues the K cn_step calls; "graph": one replay of a HIP graph of the K launches (cn_set_graph_mode).
    Returns the measurements on every rank."""
    from crowdnav_dsrnn_amd import _lib
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    if workload == "c5":
        cfgs, env_group = c5_mixed(E, rank * E, E * world, rng)
        engs = [CrowdNavEngine.mixed(cfgs, env_group, device)]
    else:
        engs = [CrowdNavEngine(make_config(E, N, rank * E, E * world, workload, rng), device)]
    eng = engs[0]
    SW, SK = 100, 2000   # 100 warm-up steps, then >= 2,000 timed steps incl. all auto-resets
    gen = torch.Generator(device=device)
    gen.manual_seed(rank)

    def actions(T, e_):
        if workload == "c2":   # unicycle (dv, dtheta) ~ U[-0.1, 0.1]^2
            a = torch.rand((T, e_.E, 2), generator=gen, device=device) * 0.2 - 0.1
        else:                  # holonomic (vx, vy) ~ N(0, 0.5^2), clipped by clip_action in the kernel
            a = torch.randn((T, e_.E, 2), generator=gen, device=device) * 0.5
        return a.contiguous()

    def warm(acts, count):
        """count untimed launches, issued the way the timed window issues its own (so the window does not
        pay the first call's host-side setup)"""
        if launch == "seq":
            for e_, a in zip(engs, acts):
                e_.step_seq(a[0:count])
        else:
            for s in range(count):
                for e_, a in zip(engs, acts):
                    e_.step(a[s])

    acts = [actions(K + W, e_) for e_ in engs]
    for e_ in engs:
        e_.reset()
    L = _lib.lib()
    # the warm-up launches also run the window's bracket once (reset-count read, cn_profile's events armed,
    # recorded and read), so the timed window pays none of their first-use costs
    reset_total_dev(eng)
    prof_warm = W > 0 and launch != "graph"
    if prof_warm:
        _lib.check(L.cn_profile(eng._h, 1, W))
    warm(acts, W)
    if prof_warm:
        a_ms, b_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a_ms), ctypes.byref(b_ms), ctypes.byref(n)))
        _lib.check(L.cn_profile(eng._h, 0, 0))
    reset_total_dev(eng)

    use_graph = launch == "graph" and eng.groups is None   # (mixed engines: host-issued, no graph mode)
    if use_graph:
        for e_ in engs:
            e_.set_graph_mode(True)   # the step sequence on the device: launches capturable (synchronises)

    win_issue = [0.0]

    def timed_window(acts, first, count):
        """count launches of every engine, timed between barriers (max over ranks). launch == "seq": one
        cn_step_seq call issues the count launches back to back from native code; "host": Python issues every
        launch; in both the kernel time comes from the two HIP events cn_step records around the window on its
        stream. "graph": the count launches are captured into one HIP graph first (recorded, not run) and the
        timed region is its replay; the kernel time is the span of two HIP events around the replay."""
        r0 = reset_total_dev(eng)
        g = None
        if use_graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for s in range(count):
                    for e_, a in zip(engs, acts):
                        e_.step(a[first + s])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        else:
            _lib.check(L.cn_profile(eng._h, 1, count))
        _barrier(torch, dist, device)
        t0 = time.perf_counter()
        if g is not None:
            ev[0].record()
            g.replay()
            ev[1].record()
        elif launch == "seq":
            for e_, a in zip(engs, acts):
                e_.step_seq(a[first:first + count])
        else:
            for s in range(count):
                for e_, a in zip(engs, acts):
                    e_.step(a[first + s])
        t_issued = time.perf_counter()
        _barrier(torch, dist, device)
        elapsed = time.perf_counter() - t0
        win_issue[0] = t_issued - t0
        if g is not None:
            kernel_s = ev[0].elapsed_time(ev[1]) / 1e3 / count
            del g
        else:
            a_ms, b_ms, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
            _lib.check(L.cn_profile_read(eng._h, ctypes.byref(a_ms), ctypes.byref(b_ms), ctypes.byref(n)))
            _lib.check(L.cn_profile(eng._h, 0, 0))
            kernel_s = a_ms.value / 1e3 / max(n.value, 1)
        resets = reset_total_dev(eng) - r0
        if dist is not None:
            t = torch.tensor([elapsed, float(resets)], dtype=torch.float64, device=device)
            dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
            dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
            elapsed, resets = float(t[0].item()), int(t[1].item())
        return elapsed, kernel_s, resets, win_issue[0]

    out = {"workload": workload, "W": W, "K": K,
           "launch": "hipGraph replay" if use_graph else ("cn_step_seq (native loop of cn_step launches)"
                                                          if launch == "seq" else "host-issued cn_step per step")}
    out["main"] = timed_window(acts, W, K)
    out["done_frac"] = float(eng.done.float().mean().item())   # envs that ended an episode at the last step
    out["steady"] = None
    if steady:
        del acts
        sacts = [actions(SW + SK, e_) for e_ in engs]
        warm(sacts, SW)
        out["steady"] = timed_window(sacts, SW, SK)
        out["SW"], out["SK"] = SW, SK
        del sacts
    out["E_total"] = sum(e_.E for e_ in engs)
    out["N"] = N
    if workload == "c5":   # per group: its envs x B_step(its own N) (padding rows not counted)
        hum = eng.env_humans.cpu().numpy()
        out["bpl"] = int(sum(algorithmic_bytes_per_env_step(int(n)) for n in hum))
    else:
        out["bpl"] = algorithmic_bytes_per_env_step(eng.N) * eng.E
    for e_ in engs:
        e_.close()
    return out


def env_window_obj(m, world, which="main"):
    """The line's object for one window of run_env (value, timing, resets, roofline)."""
    el, ks, resets, issue = m[which]
    W, K = (m["W"], m["K"]) if which == "main" else (m["W"] + m["K"] + m["SW"], m["SK"])
    pmc = load_pmc("cn_step_kernel", m["workload"], window=(W, K))
    return {"value": round(world * m["E_total"] * K / el, 1), "unit": "env-steps/s", "warmup": W, "steps": K,
            "ms_per_step": round(el / K * 1e3, 6), "step_kernel_ms": round(ks * 1e3, 5),
            "window": "launches %d..%d after cn_reset" % (W + 1, W + K), "launches": [W, K], "resets": resets,
            "launch": m["launch"],
            # where the window's wall time goes: the host's time to issue the K launches, the GPU span of the
            # K step kernels (the two HIP events around them), the rest (first-launch latency + final sync)
            "window_ms": {"wall": round(el * 1e3, 4), "host_issue": round(issue * 1e3, 4),
                          "step_kernels": round(ks * K * 1e3, 4), "other": round((el - ks * K) * 1e3, 4)},
            "roofline": roofline_obj(m["bpl"] / ks / 1e9, m["bpl"], pmc)}


# SURVEY §8d side measurements carried by the default line (driver-observed C3 / C4 / C5):
# (workload, warm-up, timed steps); C4 counts PPO updates (the first warm-up update runs eagerly, the second
# captures the rollout's HIP graph)
SIDE_WINDOWS = (("c3", 100, 200), ("c5", 100, 200), ("c4", 2, 2))
SIDE_DEADLINE_S = 300.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--humans", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-steady", action="store_true", help="skip the steady_state window (100 + 2000 launches)")
    ap.add_argument("--no-side", action="store_true", help="skip the C3 / C4 / C5 side windows of the c2 line")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--launch", choices=["seq", "host", "graph"], default="seq",
                    help="timed env windows as one cn_step_seq call (default: K launches back to back from "
                         "native code), K host-issued cn_step calls, or one HIP-graph replay of the K launches")
    ap.add_argument("--rng", choices=["mt19937", "philox"], default="mt19937",
                    help="reset / goal-change stream: mt19937 = the reference's numpy draws (default, the "
                         "BASELINE line), philox = fast mode (SURVEY §8f-2)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2 = BASELINE metric (default); c3 / c4 / c5 are the SURVEY §8d side measurements "
                         "(c4: --steps / --warmup count PPO updates)")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--diag", choices=["nogoal"], default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    global DIAG
    DIAG = args.diag

    kind, val = launch_plan(args.gpus, os.environ)
    if kind == "error":
        print("bench.py: " + val, file=sys.stderr, flush=True)
        sys.exit(2)
    if kind == "spawn":
        sys.exit(spawn_ranks(val, sys.argv[1:]))
    world = val
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch

    # rehearsal knobs for the multi-rank path on a box with fewer GPUs than ranks (never set by the driver):
    # CN_BENCH_SHARE_DEVICE=1 puts every rank on cuda:0, CN_BENCH_DIST_BACKEND=gloo replaces RCCL (which
    # refuses two ranks on one GPU)
    dev_index = 0 if os.environ.get("CN_BENCH_SHARE_DEVICE") == "1" else local_rank
    backend = os.environ.get("CN_BENCH_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)

    E, N, K, W = args.envs, args.humans, args.steps, args.warmup
    if args.workload == "c4":
        line = run_c4(torch, dist, device, rank, world, E, N, K if K != 2000 else 10, W if W != 100 else 2)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    if args.workload == "c3" and N == 10:
        N = 25
    if args.workload == "c5" and E == 4096:
        E = 8192
    if args.workload == "c5":
        N = 5
    steady = not args.no_steady and (K < 2000 or W < 100)
    m = run_env(torch, dist, device, rank, world, args.workload, E, N, K, W, steady, args.rng, args.launch)
    line = None
    if rank == 0:
        main_w = env_window_obj(m, world)
        line = {
            "metric": METRIC,
            "value": main_w["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": main_w["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": WORKLOAD_DESC[args.workload] % (m["E_total"], N) + (
                    " [DIAGNOSTIC %s: not the metric's workload]" % DIAG if DIAG else ""),
                "envs_per_gpu": m["E_total"], "humans": N if args.workload != "c5" else "5 (traffic) / 1 (side_pref)",
                "global_envs": m["E_total"] * world,
                "parallelism": "env-sharded x%d (no collective)" % world,
                "rng": args.rng,
                "step_kernel_ms": main_w["step_kernel_ms"],
                "launch": main_w["launch"],
                "window_ms": main_w["window_ms"],
                "window": main_w["window"],
                "launches": main_w["launches"],
                "resets": main_w["resets"],
                "done_frac_last_step": round(m["done_frac"], 5),
            },
            "roofline": main_w["roofline"],
        }
        if m["steady"] is not None:
            st = env_window_obj(m, world, "steady")
            st["window"] += " (SURVEY 8d: 100 warm-up + 2000 timed, incl. auto-resets)"
            line["steady_state"] = st
    if args.workload == "c2" and not args.no_side:
        run_side_windows(torch, dist, device, rank, world, args.rng, line, args.launch)
    if rank == 0:
        if not args.no_cpu_baseline and world == 1 and args.workload == "c2":
            line["cpu_baseline"] = cpu_baseline(N, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_side_windows(torch, dist, device, rank, world, rng, line, launch="seq"):
    """SIDE_WINDOWS into line["side_c3"], ["side_c4"], ["side_c5"] (rank 0), each workload at its SURVEY §8d
    per-GPU shape on the same ranks. A watchdog bounds them: past SIDE_DEADLINE_S every rank stops, rank 0
    prints the line with what it has (the side windows never cost the main line)."""
    import threading

    t_start = time.perf_counter()
    # side results enter `line` only under this lock, so the watchdog serialises a consistent snapshot
    lock = threading.Lock()

    def bail():
        # a side window that hangs (or a rank stuck in a collective after another rank's exception) ends the
        # process with a non-zero status: the main measurement is printed first, but the run did not finish
        if rank == 0 and line is not None:
            got = lock.acquire(timeout=5.0)
            try:
                snap = dict(line)
            finally:
                if got:
                    lock.release()
            snap["side_timeout_s"] = SIDE_DEADLINE_S
            print(json.dumps(snap), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)

    timer = threading.Timer(SIDE_DEADLINE_S, bail)
    timer.daemon = True
    timer.start()
    try:
        for wl, w, k in SIDE_WINDOWS:
            t0 = time.perf_counter()
            try:
                if wl == "c4":
                    obj = run_c4(torch, dist, device, rank, world, 4096, 10, k, w)
                    if obj is not None:
                        obj = {"workload": obj["config"]["workload"], "value": obj["value"], "unit": obj["unit"],
                               "warmup": w, "steps": k, "step": "one rollout of 128 steps of every env + one PPO update",
                               "ms_per_step": obj["ms_per_step"], "resets": obj["config"]["resets"],
                               "rollout_s_per_update": obj["config"]["rollout_s_per_update"],
                               "ppo_s_per_update": obj["config"]["ppo_s_per_update"],
                               "roofline": obj["roofline"], "whole_update_roofline": obj["whole_update_roofline"]}
                else:
                    E, N = (4096, 25) if wl == "c3" else (8192, 5)
                    m = run_env(torch, dist, device, rank, world, wl, E, N, k, w, False, rng, launch)
                    obj = None
                    if rank == 0:
                        obj = dict(env_window_obj(m, world), workload=WORKLOAD_DESC[wl] % (m["E_total"], N))
            except Exception as e:   # reported in the line; the main measurement stands
                obj = {"error": "%s: %s" % (type(e).__name__, e)}
            torch.cuda.empty_cache()
            if rank == 0:
                obj["wall_s"] = round(time.perf_counter() - t0, 2)
                with lock:
                    line["side_" + wl] = obj
    finally:
        timer.cancel()
    if rank == 0:
        with lock:
            line["side_wall_s"] = round(time.perf_counter() - t_start, 2)


def roofline_obj(achieved, bpl, pmc):
    """The line's roofline object for the step kernel (SURVEY §8d B_step bytes per launch / its average
    launch time); traffic / VALU issue from a hash-matched profile of the same window, else null."""
    return {
        "bound": "hbm",
        "achieved": round(achieved, 3),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 6),
        "traffic": round(pmc["traffic"]) if pmc and pmc.get("traffic") else None,
        "kernel": "cn_step_kernel",
        "algorithmic_bytes_per_launch": bpl,
        # what actually limits the kernel: dependent per-lane chains, not bandwidth
        "limiter": "latency / issue (dependent f64 + f32 chains per lane; not HBM)",
        "valu_issue_frac": round(pmc["valu_issue_frac"], 4) if pmc and pmc.get("valu_issue_frac") else None,
        "pmc_profile": ("profiles/pmc_%s.json" % pmc["tag"]) if pmc else None,
        "pmc_avg_duration_us": round(pmc["avg_duration_ns"] / 1e3, 3) if pmc and pmc.get("avg_duration_ns") else None,
    }


if __name__ == "__main__":
    main()
