"""Diagnostic: phase breakdown of the step and RNG kernels from the -DCN_STAMPS build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DCN_STAMPS \
        -o crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so crowdnav_dsrnn_amd/csrc/cn_engine.hip crowdnav_dsrnn_amd/csrc/cn_gru.hip

    CN_LIB_PATH=crowdnav_dsrnn_amd/lib/libcrowdnav_hip_stamps.so python tools/probe_stamps.py [variant]
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


def run(variant, E=4096, N=10, steps=300):
    if variant.endswith("_301"):   # a last step that is not a multiple of 20 (random goal changes every 5 s)
        variant, steps = variant[:-4], 301
    if variant == "c2w":   # the crowded circle centre of bench.py's --steps 20 --warmup 5 window
        steps = 16
    c = clone_config(Config())
    c.sim.human_num = N
    c.sim.train_val_sim = ["circle_crossing"]
    c.action_space.kinematics = "unicycle"
    if variant == "nogoal":
        c.humans.random_goal_changing = False
        c.humans.end_goal_changing = False
    if variant == "sf":
        c.humans.policy = "social_force"
    if variant in ("c3", "c3nogoal"):
        N = 25
        c.sim.human_num = N
        c.sim.train_val_sim = ["square_crossing"]
        c.action_space.kinematics = "holonomic"
        c.robot.FOV = c.humans.FOV = 1.0
        if variant == "c3nogoal":
            c.humans.random_goal_changing = False
            c.humans.end_goal_changing = False
    if variant in ("c5a", "c5b", "c5a_nonorm", "c5b_nonorm"):   # the two C5 engines (bench.engines_for)
        c.humans.policy = "orca"
        c.action_space.kinematics = "holonomic"
        c.reward.norm_zones = not variant.endswith("nonorm")
        if variant.startswith("c5a"):
            N = 5
            c.sim.train_val_sim = c.sim.test_sim = ["parallel_traffic", "perpendicular_traffic"]
        else:
            N = 1
            c.sim.train_val_sim = c.sim.test_sim = ["side_pref_passing", "side_pref_overtaking", "side_pref_crossing"]
            c.test.side_preference = True
            c.sim.circle_radius = 4
            c.humans.random_goal_changing = False
            c.humans.end_goal_changing = False
        c.sim.human_num = N
    eng = CrowdNavEngine(make_cn_config(c, num_envs=E), "cuda:0")
    eng.reset()
    L = _lib.lib()
    L.cn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    a = np.zeros(4096 * 24, np.uint64)
    b = np.zeros(8192 * 24, np.uint64)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0)
    acts = torch.rand((steps, E, 2), generator=g, device="cuda:0") * 0.2 - 0.1
    _lib.check(L.cn_profile(eng._h, 1, steps))
    for s in range(steps):
        eng.step(acts[s])
    torch.cuda.synchronize()
    ta, tb, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    L.cn_profile_read(eng._h, ctypes.byref(ta), ctypes.byref(tb), ctypes.byref(n))
    L.cn_debug_stamps(a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p))
    blocks = (E + (64 // N) - 1) // (64 // N)
    A = a.reshape(-1, 24)[:blocks].astype(np.int64)
    d = np.diff(A[:, :7], axis=1)
    print("[%s] kernel A avg %.1f us, kernel B avg %.1f us over %d steps" % (variant, ta.value * 1e3 / n.value,
                                                                          tb.value * 1e3 / n.value, n.value))
    names = ["load", "visibility", "policy+reward terms", "reward ladder", "kinematics+obs", "rng work (phase 5)"]
    tot = (A[:, 6] - A[:, 0])
    print("  kernel A cycles per workgroup (last step): total median %d max %d" % (np.median(tot), tot.max()))
    for k, nm in enumerate(names):
        print("    %-26s median %8d  max %8d  (%.0f%%)" % (nm, np.median(d[:, k]), d[:, k].max(),
                                                            100 * np.median(d[:, k]) / np.median(tot)))
    slow = tot >= np.percentile(tot, 95)
    print("  slowest 5%% workgroups (total >= %d): mean per phase %s" % (
        np.percentile(tot, 95), ", ".join("%s %d" % (nm.split()[0], d[slow, k].mean()) for k, nm in enumerate(names))))
    # the slowest workgroups of the last launch: phases, and each env's phase-5 item (kind, cycles from the
    # workgroup's phase-5 start; per-env stamps of the same workgroup share its XCD's clock)
    Bx = b.reshape(-1, 24).astype(np.int64)
    epb_ = 64 // N
    nbk = len(tot)
    xq, xr = nbk >> 3, nbk & 7
    for k in np.argsort(-tot)[:8]:
        items = []
        xi = k & 7
        blk = xi * xq + min(xi, xr) + (k >> 3)   # the kernel's XCD-aware env placement
        for e in range(blk * epb_, min((blk + 1) * epb_, E)):
            st_, rs, gl = Bx[e, 0], Bx[e, 5], Bx[e, 4]
            if A[k, 5] <= st_ <= A[k, 6]:
                kind = "reset" if A[k, 5] <= rs <= A[k, 6] and rs >= st_ else "goal"
                end = rs if kind == "reset" else gl
                items.append("%s %d-%d" % (kind, st_ - A[k, 5], end - A[k, 5]))
        print("    WG %d total %d: %s | phase 5: wave 0 past its item count %d; %s" % (
            k, tot[k], " ".join("%d" % d[k, j] for j in range(6)), A[k, 22] - A[k, 5], ", ".join(items) or "-"))
    span = A[:, 6].max() - A[:, 0].min()
    print("  launch span (first start -> last end) %d cycles; start skew max %d" % (span, A[:, 0].max() - A[:, 0].min()))
    # the whole grid on the device-wide 100 MHz clock (s_memtime above is per XCD: durations only)
    L.cn_debug_stamps_r.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    r = np.zeros(8192 * 2, np.uint64)
    L.cn_debug_stamps_r(r.ctypes.data_as(ctypes.c_void_p), None)
    print("  lp3 sub-problems over all launches: solved %d, visited by RVO2's loop %d" % (int(r[-14]), int(r[-13])))
    r[-14:] = 0
    R = r.reshape(-1, 2).astype(np.int64)
    live = np.nonzero(R[:, 1] > 0)[0]
    if len(live):
        R = R[:live.max() + 1]
        t0r = R[R[:, 0] > 0, 0].min()
        st, en = (R[:, 0] - t0r) * 10, (R[:, 1] - t0r) * 10     # ns
        kd = variant in ("c3", "c3nogoal")
        nb = len(R)
        is_step = np.zeros(nb, bool)
        if kd:
            is_step[nb - blocks:] = True
        else:
            is_step[:blocks] = True
        print("  grid timeline (ns from the first workgroup's start; %d step + %d spawn workgroups):" % (
            is_step.sum(), (~is_step).sum()))
        for nm, sel in (("step", is_step), ("spawn", ~is_step)):
            if sel.any():
                print("    %-5s start median %6d max %6d | end median %6d p95 %6d max %6d | duration median %6d max %6d" % (
                    nm, np.median(st[sel]), st[sel].max(), np.median(en[sel]), np.percentile(en[sel], 95), en[sel].max(),
                    np.median(en[sel] - st[sel]), (en[sel] - st[sel]).max()))
        last = np.argsort(-en)[:8]
        print("    last to end: " + ", ".join("%s#%d [%d, %d]" % ("step" if is_step[k] else "spawn", k, st[k], en[k])
                                              for k in last))
    B = b.reshape(-1, 24).astype(np.int64)[:E]
    t0 = A[:, 0].min()
    sub = [("p0 human loads", A[:, 12] - A[:, 0]), ("p0 env loads", A[:, 13] - A[:, 12]), ("p0 clip", A[:, 10] - A[:, 13]), ("p0 robot VR", A[:, 11] - A[:, 10]), ("p0 barrier", A[:, 1] - A[:, 11]),
           ("lines+sort", A[:, 7] - A[:, 2]), ("LP2", A[:, 8] - A[:, 7]), ("LP3", A[:, 9] - A[:, 8]), ("VR+terms", A[:, 3] - A[:, 9])]
    if (A[:, 14] > A[:, 2]).all():
        sub += [("kd: table", A[:, 15] - A[:, 2]), ("kd: walk", A[:, 14] - A[:, 15]),
                ("kd: rank+lines", A[:, 7] - A[:, 14])]
    if variant in ("c3", "c3nogoal"):
        it = A[:, 13]
        print("      kd walk iterations (thread 0's human, round 2): median %d max %d mean %.2f" % (np.median(it), it.max(), it.mean()))
        sub = [x for x in sub if not x[0].startswith("p0")]
    for nm, v in sub:
        print("      wave0 %-12s median %8d  max %8d" % (nm, np.median(v), v.max()))
    if variant not in ("c3", "c3nogoal"):   # linearProgram3 sub-problems of the workgroup (lp3_tasks): count, cycles B1 -> B2
        cyc = A[:, 23]
        print("      lp3 task rounds (lp3_tasks + replays) cycles: median %d max %d" % (np.median(cyc), cyc.max()))
    if variant not in ("c3", "c3nogoal"):   # per-wave ends of phases 0-2 (-DCN_STAMPS lanes 0 / 64 / 128), from the phase start
        per = [("p0 wave1 env load+clip+VR", A[:, 16] - A[:, 0]), ("p1 wave0 visibility", A[:, 19] - A[:, 1]),
               ("p1 wave1 reward terms", A[:, 17] - A[:, 1]), ("p1 wave2 robot terms", A[:, 18] - A[:, 1]),
               ("p2 wave1 quads done", A[:, 21] - A[:, 2]), ("p2 wave1 +ladder", A[:, 20] - A[:, 2])]
        for nm, v in per:
            print("      %-26s median %8d  max %8d" % (nm, np.median(v), v.max()))
    cur = B[:, 0] >= t0                      # items of the last step only
    res = B[cur & (B[:, 5] >= B[:, 0])]
    goal = B[cur & (B[:, 4] >= B[:, 0]) & (B[:, 5] < B[:, 0])]
    if len(res):
        r = res[:, 5] - res[:, 0]
        print("  phase-5 resets (last step, %d envs): cycles median %d p90 %d max %d" % (len(res), np.median(r), np.percentile(r, 90), r.max()))
    if len(goal):
        gg = np.diff(goal[:, :5], axis=1)
        tot = goal[:, 4] - goal[:, 0]
        print("  phase-5 goal items (last step, %d envs): mt load %d  random %d  end %d  write %d (median); total median %d p90 %d max %d"
              % (len(goal), *np.median(gg, axis=0), np.median(tot), np.percentile(tot, 90), tot.max()))
        for slot, nm in ((6, "random"), (7, "end")):
            v = goal[:, slot]
            rounds, chg, elig = v // 1000, (v % 1000) // 100, v % 100
            part = gg[:, 1] if slot == 6 else gg[:, 2]
            print("     %s pass: eligible mean %.2f, rounds mean %.2f max %d, changes (1st round) mean %.2f" % (
                nm, elig.mean(), rounds.mean(), rounds.max(), chg.mean()))
            k0 = 8 if slot == 6 else 11
            for r in range(int(rounds.max()) + 1):
                sel = rounds == r
                if sel.any():
                    print("        %d rounds: %4d envs, cycles median %d max %d | walk %d first-tries %d reject-loop %d (mean)" % (
                        r, sel.sum(), np.median(part[sel]), part[sel].max(), goal[sel, k0].mean(), goal[sel, k0 + 1].mean(),
                        goal[sel, k0 + 2].mean()))
    if len(goal) or len(res):   # the slowest 5 % workgroups' envs: what their RNG waves did (last step)
        epb = 64 // N
        slow_b = np.nonzero(slow)[0]
        sel = np.zeros(E, bool)
        for b in slow_b:
            sel[b * epb:(b + 1) * epb] = True
        rows = np.nonzero(cur)[0]
        ss = rows[sel[rows]]
        kinds = {"reset": ss[B[ss, 5] >= B[ss, 0]], "goal": ss[(B[ss, 4] >= B[ss, 0]) & (B[ss, 5] < B[ss, 0])]}
        print("  slowest 5%% workgroups' envs (%d WGs, %d env items): resets %d, goal items %d" % (
            len(slow_b), len(ss), len(kinds["reset"]), len(kinds["goal"])))
        gi = kinds["goal"]
        if len(gi):
            gg = np.diff(B[gi, :5], axis=1)
            print("    goal items: mt load %d random %d end %d write %d (mean); random changes mean %.2f, end changes mean %.2f" % (
                *gg.mean(axis=0), ((B[gi, 6] % 1000) // 100).mean(), ((B[gi, 7] % 1000) // 100).mean()))
    if variant in ("c3", "c3nogoal"):
        L.cn_debug_stamps_c.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        cc = np.zeros(8192 * 4, np.uint64)
        pp = np.zeros(8192 * 2, np.uint64)
        L.cn_debug_stamps_c(cc.ctypes.data_as(ctypes.c_void_p), pp.ctypes.data_as(ctypes.c_void_p))
        P = pp.reshape(-1, 2).astype(np.int64)[:E]
        ok = P[:, 1] > P[:, 0]
        if ok.any():
            dur = P[ok, 1] - P[ok, 0]    # the latest spawn of each env (s_memtime differs across XCDs: durations only)
            print("  spawn waves (latest spawn per env, %d envs): cycles median %d p90 %d max %d" % (
                ok.sum(), np.median(dur), np.percentile(dur, 90), dur.max()))
        C = cc.reshape(-1, 4).astype(np.float64)[:E]
        n = C[:, 3].sum()
        if n:
            print("  crowded rejection, all steps: %d passes; per pass cycles: ensure (MT gen) %.0f, candidates %.0f, "
                  "tests + ballot %.0f" % (n, C[:, 0].sum() / n, C[:, 1].sum() / n, C[:, 2].sum() / n))
    eng.close()


if __name__ == "__main__":
    for v in (sys.argv[1:] or ["c2", "nogoal", "sf"]):
        run(v)
