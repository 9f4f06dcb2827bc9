// cn_engine.hip — MI355X (gfx950) batched CrowdSimDict engine: kernels + C ABI (include/crowdnav.h).
//
// Hot path: ONE kernel launch per cn_step (no host synchronisation, no second kernel):
//   cn_step_kernel, step workgroups: one lane per (env, human), 256-lane workgroups holding
//       floor(256/N) whole envs. Phases 0-4: SRNN.clip_action, the human policies (ORCA LP / social
//       force) on the PRE-move state, calc_reward, kinematics, observation, Monitor. Phase 5: the
//       workgroup's own RNG work, one wave per env needing it — goal changes (numpy-legacy MT19937 in
//       LDS) and the VecEnv auto-reset, which copies a spawn drawn ahead of time.
//   cn_step_kernel, spare workgroups: spawn waves. CrowdSimDict.reset is a pure function of the seed
//       schedule, so each env's NEXT episode is drawn (reseed + spawn with rejection) by these spare
//       workgroups right after its reset, concurrently with the step. On the kd-tree path they come
//       first in the grid so that they are dispatched first: a crowded spawn (25 humans in
//       square_crossing) runs ~1M cycles, longer than the step workgroups' rounds, and started last it
//       would add its whole latency to the launch. On the quad path (cheap spawns) they come last, so
//       the step workgroups start without waiting for their dispatch.
//   cn_reset_kernel: cn_reset (every env), one wave per env.
// Reference: crowd_sim/envs/crowd_sim_dict.py:105-271, crowd_sim/envs/crowd_sim.py:296-1161,
// crowd_sim/envs/utils/agent.py:172-218, crowd_nav/policy/{orca,social_force,srnn}.py; RVO2 v2.0
// (third-party) restated in float32. Numerics: see cn_math.h.
#include <hip/hip_runtime.h>
#include <vector>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/crowdnav.h"
#include "../../include/crowdnav_state.h"
#include "cn_math.h"

using namespace cn;

// LDS ordering among the lanes of ONE wave (kernel B workgroups are a single wave; the spawn waves of
// kernel A run independently of the other waves of their workgroup): no s_barrier needed, only the
// compiler/LDS ordering a release/acquire pair at wavefront scope gives.
__device__ __forceinline__ void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#define CN_BLK 256

// Diagnostic build only (-DCN_STAMPS): per-workgroup s_memtime stamps at phase boundaries, read back
// with cn_debug_stamps(). The shipped library is built without it (no stamp executes).
#ifdef CN_STAMPS
#define CN_NSTAMP 24
__device__ unsigned long long cn_stamp_a[4096 * CN_NSTAMP];
__device__ unsigned long long cn_stamp_b[8192 * CN_NSTAMP];
__device__ unsigned long long cn_stamp_c[8192 * 4];   // crowded rejection: ensure / cand / test / passes
__device__ unsigned long long cn_stamp_p[8192 * 2];   // spawn waves: start / end of each env's latest spawn
__device__ unsigned long long cn_stamp_r[8192 * 2];   // every workgroup: start / end on the device-wide 100 MHz clock
__device__ unsigned long long cn_lp3_cnt[2 + 12];   // lp3 sub-problems solved / visited by the replay (all launches)
__device__ unsigned long long cn_stamp_s[8192 * 16];   // spawn_env: start, seeded, robot, after human i (3 + i)
#define STAMP_S(e, k) do { if (lane == 0 && (e) >= 0 && (e) < 8192) cn_stamp_s[(e) * 16 + (k)] = clock64(); } while (0)
#define STAMP_R(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) cn_stamp_r[blockIdx.x * 2 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define STAMP_A(k) do { const unsigned sb_ = (unsigned)sb; if (threadIdx.x == 0 && sb_ < 4096) cn_stamp_a[sb_ * CN_NSTAMP + (k)] = clock64(); } while (0)
#define STAMP_B(w, k) do { if ((threadIdx.x & 63) == 0 && (w) < 8192) cn_stamp_b[(w) * CN_NSTAMP + (k)] = clock64(); } while (0)
// stamp k by thread t (a lane of another wave than thread 0's)
#define STAMP_T(k, t) do { const unsigned sb_ = (unsigned)sb; if (threadIdx.x == (t) && sb_ < 4096) cn_stamp_a[sb_ * CN_NSTAMP + (k)] = clock64(); } while (0)
#else
#define STAMP_T(k, t) do { } while (0)
#define STAMP_A(k) do { } while (0)
#define STAMP_B(w, k) do { } while (0)
#define STAMP_R(k) do { } while (0)
#define STAMP_S(e, k) do { } while (0)
#endif
#define CN_MAX_A 32
#ifndef CN_LP3_W
#define CN_LP3_W 12   // linearProgram3 sub-problems solved ahead per infeasible human (lp3_tasks); the rest inline
#endif
#define CN_DUMMY_POS 7.0
#define CN_CTL_NSTEP 12   // work_count words of the device-side step sequence (StepArgs::ctl)
#define CN_CTL_ALL 13
#define CN_CTL_DONE 14

// ------------------------------------------------------------------------------------------------
// launch geometry + LDS plan of kernel A
// ------------------------------------------------------------------------------------------------
struct StepPlan {
    int T;       // threads per workgroup (256)
    int H;       // human-lane stride (64: the humans of EPB envs sit on wave 0's lanes)
    int NH;      // per-human stride of the ORCA scratch arrays (kd-tree path: EPB * N humans; quad path: H)
    int EPB;     // envs per workgroup
    int M;       // observed slots per human (ORCA lines upper bound)
    int A;       // agents per RVO2 simulator
    int kd;      // A > 10: RVO2's KdTree order decides ties between equally distant neighbours
    // LDS byte offsets
    int o_renv, o_racts, o_rflag, o_rvr, o_hum, o_lane, o_orad, o_vis, o_nv, o_eg, o_lines, o_proj, o_nd, o_ns, o_perm,
        o_hvr, o_hst, o_l3b, o_l3r, o_l3k,
        total;
    int rng_waves;   // phase-5 RNG regions (rng_stride bytes each), laid over o_lines
    int rng_stride;  // CN_PEND_LDS, + CN_GRID_LDS when the plan has room for the spawn's DiscGrid
};

#define CN_RENV_F 27   // robot/env doubles per env in LDS
#define CN_HUM_F 14    // human doubles per lane in LDS
#define CN_PEND_LDS (2 * CN_MT_N * 4 + 7 * 32 * 8 + 6 * 64 * 8)   // per RNG wave: MT ring, agent table, try slots
#ifndef CN_COVER_RANDGOAL
#define CN_COVER_RANDGOAL 1   // diagnostic switch: the candidate-box cover for random goals on the circle
#endif
#ifndef CN_QUAD_PARK
// the quad path's spawning waves park their spawns after a budget too (and cn_reset pre-draws the next two
// spawns, as on the kd-tree path): round 6's timeline (stamps build without contended atomics) had the
// spawn workgroups end last in 78 % of steady C2 launches, one circle_crossing spawn being ~82 k cycles
#define CN_QUAD_PARK 1
#endif
#ifndef CN_QUAD_BUDGET
#define CN_QUAD_BUDGET 70000   // clock cycles a quad-path spawning wave works per launch before parking
#endif
#ifndef CN_QUAD_SPAWN_WAVES
#define CN_QUAD_SPAWN_WAVES 128   // spawning waves of the quad path's spare workgroups
#endif
#ifndef CN_SLOT_FENCE
// device-scope fences around the pending-slot handshake inside a step launch (write_pending / reset_env), the
// round-5 protocol (ok zeroed and fenced before a slot's new key; key, fence, ok on the reader's side). On gfx950
// each is buffer_wbl2 sc1 + buffer_inv sc1: a write-back AND invalidation of the XCD's whole L2, once per spawn
// written and per reset. Round 6 replaces them by a key-tagged ok word (PendPtrs::ok, reset_env), which needs none.
#define CN_SLOT_FENCE 0
#endif
#ifndef CN_SPAWN_PRIO
#define CN_SPAWN_PRIO 0     // issue priority of the quad path's spawning waves (0: normal)
#endif
#ifndef CN_RNG_PRIO_ALL
#define CN_RNG_PRIO_ALL 0   // diagnostic: raise the RNG waves' priority on the quad path too
#endif
#define CN_GRID 16
#define CN_GRID_LDS (96 * 8 + CN_GRID * CN_GRID * 4 + 4 * 8 + 4 * 8)   // + spawn DiscGrid: agent table, masks, cover, box

__host__ __device__ inline int cn_align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline StepPlan cn_step_plan(int N, int robot_visible)
{
    StepPlan p;
    p.A = N + (robot_visible ? 1 : 0);
    p.M = p.A - 1;
    p.kd = p.A > 10;
    // 4 waves: the humans of EPB = 64 / N envs on wave 0's lanes for the per-human phases, the env lanes
    // on wave 1, all 256 lanes (4 per human) for ORCA. A > 10 adds the KdTree build / query (one lane of
    // each quad) that fixes RVO2's neighbour order.
    p.T = CN_BLK;
    p.H = 64;
    // at most 16 envs per workgroup: with 1-3 humans per env (side-preference scenarios) 64 / N envs would
    // put up to 64 env lanes' divergent reward / norm-zone work on one wave (C5: 16 -> +6 %; 8 -> -2 %)
    p.EPB = p.H / N < 16 ? p.H / N : 16;
    const int H = p.H;
    const int ML = p.M > 0 ? p.M : 1;
    // the kd-tree path sizes its ORCA scratch for the workgroup's EPB * N humans (quads past them never
    // touch it), so that three workgroups fit a CU's LDS
    p.NH = p.kd ? p.EPB * N : H;
    const int NH = p.NH;
    int o = 0;
    p.o_renv = o;  o = cn_align16(o + CN_RENV_F * p.EPB * 8);
    p.o_racts = o; o = cn_align16(o + 2 * p.EPB * 4);
    p.o_rflag = o; o = cn_align16(o + (3 * p.EPB + 2) * 4);   // + the 64-bit mask of envs with RNG work
    p.o_rvr = o;   o = cn_align16(o + 8 * p.EPB * 8);
    p.o_hum = o;   o = cn_align16(o + CN_HUM_F * H * 8);
    p.o_lane = o;  o = cn_align16(o + H * 8 + H * 4);      // closest distance (f64) + flag word
    p.o_orad = o;  o = cn_align16(o + H * 4);
    p.o_vis = o;   o = cn_align16(o + 3 * H * 4);          // visible mask, dummy mask, frozen max speed
    p.o_nv = o;    o = cn_align16(o + H * 16);             // post-move positions (x [H], y [H])
    p.o_eg = o;    o = cn_align16(o + H * 4);              // goal-reached / NaN flags
    // ORCA, per human: sorted lines [NH][M], projected lines [NH][M], neighbour distances (quad path); kd:
    // neighbour slots [M][NH], KdTree agent order [A][NH]
    p.o_lines = o; o = cn_align16(o + ML * NH * 16);
    p.o_proj = o;  o = cn_align16(o + ML * NH * 16);
    p.o_nd = o;    o = cn_align16(o + (p.kd ? 0 : ML * H * 4));
    p.o_ns = o;    o = cn_align16(o + (p.kd ? (ML + 1) * NH : 0));      // + a dummy row (the KdTree walk)
    p.o_perm = o;  o = cn_align16(o + (p.kd ? (p.A + 1) * NH : 0));     // + a dummy row
    // human velocity rectangles [8][H] (phases 1-2) + the human values human_post stages for the contiguous
    // state / observation stores after phase 2 [7][H]: over the quad path's projected-line / distance
    // scratch, unused there since the linear programs keep their lines in registers. The kd-tree path keeps
    // both in each human's own projected-line block instead (hvr_ref / hst_ref below): the rectangle is
    // consumed at the start of phase 2, before that block holds the KdTree exchange, and the staged values
    // are written after the human's linearProgram3, its last use of the block.
    if (p.kd) { p.o_hvr = p.o_proj; p.o_hst = p.o_proj; }
    else if ((p.o_ns - p.o_proj) >= 15 * H * 8) { p.o_hvr = p.o_proj; p.o_hst = p.o_proj + 8 * H * 8; }
    else { p.o_hvr = o; p.o_hst = o + 8 * H * 8; o = cn_align16(o + 15 * H * 8); }
    // quad path: the workgroup's linearProgram3 sub-problems (lp3_tasks): per human fail | n << 8, results
    // [H][12] (phase 2 only: under the RNG regions)
    p.o_l3b = o;   o = cn_align16(o + (p.kd ? 0 : H * 4));
    p.o_l3r = o;   o = cn_align16(o + (p.kd ? 0 : H * 12 * 8));
    p.o_l3k = o;   o = cn_align16(o + (p.kd ? 0 : H * 12));
    // one RNG wave per env of the workgroup, at most 4 (kd-tree path: EPB = 2 or 5 envs)
    p.rng_waves = p.EPB < 4 ? p.EPB : 4;
    // the DiscGrid region only where it costs no LDS (the kd-tree path's ORCA scratch is larger than the
    // RNG regions it hosts); the quad path keeps its 3 workgroups per CU
    p.rng_stride = p.o_lines + p.rng_waves * (CN_PEND_LDS + CN_GRID_LDS) <= o ? CN_PEND_LDS + CN_GRID_LDS : CN_PEND_LDS;
    const int rng_end = p.o_lines + p.rng_waves * p.rng_stride;
    p.total = o > rng_end ? o : rng_end;
    return p;
}

// kernel-A LDS views
struct SL {
    int T;            // lane stride of the per-lane arrays
    double *r;        // [CN_RENV_F][EPB]
    float *act;       // [2][EPB] clipped action (holonomic vx,vy / unicycle v,r)
    uint32_t *rflag;  // [EPB] flags ; [EPB] aux ; [EPB] humans the reward loop visited (first collision + 1)
    double *rvr;      // [8][EPB] robot VelocityRectangle corners
    double *hvr;      // [8][H] human VelocityRectangle corners (x0..x3, y0..y3)
    double *hst;      // [7][H] human_post's results (vx, vy, belief px, py, vx, vy, r), stored after phase 2
    double *h;        // [CN_HUM_F][T]
    double *cd;       // [T]
    uint32_t *lf;     // [T]
    float *orad;      // [T]
    uint32_t *vis;    // [H] visible-now mask of the human's observed slots (quad path)
    uint32_t *dm;     // [H] dummy-at-creation mask
    float *vmax;      // [H] frozen RVO2 max speed
    double *npx, *npy; // [H] each: post-move human positions (the phase-5 goal changes read them)
    uint32_t *eg;     // [H] goal reached (LF_ENDGOAL) / non-finite position (bit 31) after the move
    float4 *lines;    // [M][T]  (kd-tree path)
    float4 *proj;     // [M][T]  linearProgram3's projected lines (kd-tree path)
    float *nd;        // [M][T]
    uint8_t *ns;      // [M][T]
    uint8_t *perm;    // [A][T]
};
enum { R_PX, R_PY, R_GX, R_GY, R_VX, R_VY, R_TH, R_RAD, R_VP, R_POT, R_GT, R_DV, R_NX, R_NY, R_LAX, R_LAY, R_EPR,
       // robot terms of calc_reward / kinematics computed early (phase 1), applied in phase 3
       R_CVX, R_CVY, R_NTH, R_JERK, R_D2G, R_SPD, R_SL, R_SR, R_SEP, R_BITS };
enum { H_PX, H_PY, H_GX, H_GY, H_VX, H_VY, H_R, H_VP, H_TH, H_BPX, H_BPY, H_BVX, H_BVY, H_BR };
#define RF(sl, f, el, EPB) ((sl).r[(f) * (EPB) + (el)])
#define HF(sl, f, t) ((sl).h[(f) * (sl).T + (t)])

// lane flag bits
#define LF_VR 1u
#define LF_NOTREACHED 2u
#define LF_ENDGOAL 4u

// ------------------------------------------------------------------------------------------------
// FOV (CrowdSim.detect_visible, crowd_sim.py:820-847)
// With fov >= 2*pi (the reference default, FOV = 2) the arccos test always passes: an agent is visible
// iff the normalised dot product is not NaN. Away from under/overflow of |v|^2 that is "heading finite
// and the agents not coincident", decided without atan2/cos/sin/sqrt/division; `vis360` returns -1
// where the full computation must decide (|v|^2 outside [1e-300, 1e300]).
// ------------------------------------------------------------------------------------------------
// unit FOV direction of an agent with float64 heading
__device__ inline void fov_dir64(double th, double &fx, double &fy)
{
    fx = cos(th); fy = sin(th);
    const double nf = np_norm2(fx, fy);
    fx = ddiv(fx, nf); fy = ddiv(fy, nf);
}
// float32 heading (np.float32 robot state): float32 cos/sin/norm, promoted for the dot
__device__ inline void fov_dir32(float th, double &fx, double &fy)
{
    float cx = np_cosf(th), cy = np_sinf(th);
    const float nf = np_norm2f(cx, cy);
    fx = (double)fdiv(cx, nf); fy = (double)fdiv(cy, nf);
}
__device__ __forceinline__ int vis360(bool heading_finite, double px1, double py1, double px2, double py2)
{
    if (!heading_finite) return 0;
    const double dx = px2 - px1, dy = py2 - py1;
    const double n2 = __fma_rn(dy, dy, dx * dx);
    return (n2 > 1e-300 && n2 < 1e300) ? 1 : -1;
}
// arccos(d) <= fov / 2, the reference's test, out of line: only cosines within the band below reach it
__device__ __noinline__ bool acos_within(double d, double fov) { return fabs(acos(d)) <= fov / 2; }
// `cth` = cos(fov / 2) (any accurate evaluation): arccos is decreasing with |d arccos / dd| >= 1, so for
// |d - cth| > 1e-12 the arccos of d is farther than 1e-12 from fov / 2 -- orders of magnitude beyond the
// few-ulp error of any arccos or cosine -- and the comparison of d with cth gives the arccos test's
// answer; only the 2e-12-wide band around cth evaluates the arccos itself.
__device__ inline bool in_fov(double fx, double fy, double px1, double py1, double px2, double py2, double fov,
                              double cth)
{
    double vx = px2 - px1, vy = py2 - py1;
    const double nv = np_norm2(vx, vy);
    vx = ddiv(vx, nv); vy = ddiv(vy, nv);
    double d = np_dot2(fx, fy, vx, vy);
    if (d != d) return false;  // coincident agents: arccos(nan) -> not visible
    if (fov >= 2.0 * CN_PI) return true;
    d = d < -1.0 ? -1.0 : (d > 1.0 ? 1.0 : d);
    if (d > cth + 1e-12) return true;
    if (d < cth - 1e-12) return false;
    return acos_within(d, fov);
}

// in_fov decided without square roots or divisions where that is exact (FOV < 2 pi; the pair loops of
// phase 1 and the robot's belief test): d = (f . v) / |v| against thresholds 4e-12 either side of cth, as
// sign tests of dp = f . v and of dp^2 - t^2 |v|^2 (d > t <=> dp > t |v|). These are within a few 1e-16 of
// the exact values, and the reference's d (correctly rounded norm, divisions and dot product, in_fov)
// within a few 1e-16 of the exact d too, so outside the +-4e-12 band both sides of cth are decided alike;
// inside it (and for |v|^2 near under/overflow or zero: coincident agents) in_fov itself runs.
__device__ inline bool in_fov_fast(double fx, double fy, double px1, double py1, double px2, double py2, double fov,
                                   double cth)
{
    const double dx = px2 - px1, dy = py2 - py1;
    const double n2 = __fma_rn(dy, dy, dx * dx);
    if (n2 > 1e-200 && n2 < 1e200) {
        const double dp = __fma_rn(fy, dy, fx * dx), dp2 = dp * dp;
        const double hi = cth + 4e-12, lo = cth - 4e-12;
        const bool above = hi >= 0.0 ? (dp > 0.0 && dp2 > hi * hi * n2) : (dp >= 0.0 || dp2 < hi * hi * n2);
        if (above) return true;
        const bool below = lo > 0.0 ? (dp <= 0.0 || dp2 < lo * lo * n2) : (dp < 0.0 && dp2 > lo * lo * n2);
        if (below) return false;
    }
    return in_fov(fx, fy, px1, py1, px2, py2, fov, cth);
}

// the robot's FOV test of a freshly spawned human (generate_ob(reset=True)), out of line: inlined into the
// step kernel's RNG phase, the acos polynomial's f64 constants were hoisted to the loop preheader and
// spilled to scratch by every wave with RNG work; only FOV < 2 pi configurations call it
__device__ __noinline__ int reset_fov_test(double th, double rpx, double rpy, double px, double py, double fov)
{
    double fx, fy;
    fov_dir64(th, fx, fy);
    return in_fov(fx, fy, rpx, rpy, px, py, fov, cos(fov / 2)) ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// shapely restatements (parity unpinned)
// ------------------------------------------------------------------------------------------------
__device__ inline void vel_rect(double px, double py, double vx, double vy, double r, bool f32, double *cx,
                                double *cy)
{
    const double w = 2 * r * 1;
    double len, dth, xos, yos;
    if (f32) {
        const float fvx = (float)vx, fvy = (float)vy;
        len = (double)(3.0f * fsqrt(fvx * fvx + fvy * fvy));
        const float h = atan2f(fvy, fvx);
        dth = (double)(h - (float)(CN_PI / 2));
        xos = px + (double)((float)r * np_cosf(h));
        yos = py + (double)((float)r * np_sinf(h));
    } else {
        len = 3 * dsqrt(vx * vx + vy * vy);
        const double heading = atan2(vy, vx);
        dth = heading - CN_PI / 2;
        xos = px + r * cos(heading);
        yos = py + r * sin(heading);
    }
    double c = cos(dth), s = sin(dth);
    if (fabs(c) < 2.5e-16) c = 0.0;
    if (fabs(s) < 2.5e-16) s = 0.0;
    const double bx[4] = {w / 2, w / 2, -w / 2, -w / 2};
    const double by0[4] = {-len / 2, len / 2, len / 2, -len / 2};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double x = bx[k], y = by0[k] + len / 2;
        cx[k] = (c * x - s * y) + xos;
        cy[k] = (s * x + c * y) + yos;
    }
}

__device__ inline bool quads_intersect(const double *ax, const double *ay, const double *bx, const double *by)
{
    for (int p = 0; p < 2; ++p) {
        const double *qx = p ? bx : ax, *qy = p ? by : ay;
        for (int k = 0; k < 4; ++k) {
            const double ex = qx[(k + 1) & 3] - qx[k], ey = qy[(k + 1) & 3] - qy[k];
            if (ex == 0.0 && ey == 0.0) continue;
            for (int t = 0; t < 2; ++t) {
                const double nx = t ? ex : -ey, ny = t ? ey : ex;
                double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const double pa = ax[v] * nx + ay[v] * ny, pb = bx[v] * nx + by[v] * ny;
                    amin = pa < amin ? pa : amin; amax = pa > amax ? pa : amax;
                    bmin = pb < bmin ? pb : bmin; bmax = pb > bmax ? pb : bmax;
                }
                if (amax < bmin || bmax < amin) return false;
            }
        }
    }
    return true;
}

__device__ __forceinline__ int quad_or(int x);
// quads_intersect split over the 4 lanes of a quad: lane s tests the 4 axes of edges 2(s & 1), 2(s & 1) + 1 of
// quad s >> 1 and the quad ORs "separated" (a separating axis exists iff some lane found one: the same
// boolean as the sequential early-out loop). Lanes of the quad must run it together.
__device__ __forceinline__ bool quads_intersect_q(const double *ax, const double *ay, const double *bx, const double *by,
                                                  int s)
{
    // the lane's quad and edges by register selects (no lane-dependent indexing)
    const bool qb = (s >> 1) != 0, hi = (s & 1) != 0;
    double Qx[4], Qy[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) { Qx[v] = qb ? bx[v] : ax[v]; Qy[v] = qb ? by[v] : ay[v]; }
    double ex[2], ey[2];
    ex[0] = hi ? Qx[3] - Qx[2] : Qx[1] - Qx[0]; ey[0] = hi ? Qy[3] - Qy[2] : Qy[1] - Qy[0];   // edge k0
    ex[1] = hi ? Qx[0] - Qx[3] : Qx[2] - Qx[1]; ey[1] = hi ? Qy[0] - Qy[3] : Qy[2] - Qy[1];   // edge k0 + 1
    int sep = 0;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        if (ex[kk] == 0.0 && ey[kk] == 0.0) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const double nx = t ? ex[kk] : -ey[kk], ny = t ? ey[kk] : ex[kk];
            double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const double pa = ax[v] * nx + ay[v] * ny, pb = bx[v] * nx + by[v] * ny;
                amin = pa < amin ? pa : amin; amax = pa > amax ? pa : amax;
                bmin = pb < bmin ? pb : bmin; bmax = pb > bmax ? pb : bmax;
            }
            if (amax < bmin || bmax < amin) sep = 1;
        }
    }
    return quad_or(sep) == 0;
}

__device__ inline bool inside_world(double px, double py, double r, double half)
{
    const bool right = (px + r >= half) && (px - r <= half);
    const bool left = (px - r <= -half) && (px + r >= -half);
    const bool top = (py + r >= half) && (py - r <= half);
    const bool bottom = (py - r <= -half) && (py + r >= -half);
    return !(right || left || top || bottom);
}

// The robot's heading frame of its norm zones (both zones share it): offset point and rotation by dth
struct ZoneFrame {
    double dth, xos, yos, c, s;
};

__device__ __forceinline__ ZoneFrame zone_frame(double px, double py, double vx, double vy, double r, bool f32)
{
    ZoneFrame f;
    if (f32) {
        const float h = atan2f((float)vy, (float)vx);
        f.dth = (double)(h - (float)(CN_PI / 2));
        f.xos = px + (double)((float)r * np_cosf(h));
        f.yos = py + (double)((float)r * np_sinf(h));
    } else {
        const double heading = atan2(vy, vx);
        f.dth = heading - CN_PI / 2;
        f.xos = px + r * cos(heading);
        f.yos = py + r * sin(heading);
    }
    f.c = cos(f.dth); f.s = sin(f.dth);
    if (fabs(f.c) < 2.5e-16) f.c = 0.0;
    if (fabs(f.s) < 2.5e-16) f.s = 0.0;
    return f;
}

__device__ inline void norm_zone(const ZoneFrame &f, double r, int lhs, int left, double *cx, double *cy)
{
    const double w = 2 * r * 1.5, len = 1.5 * 1.2;
    const double xos = f.xos, yos = f.yos, c = f.c, s = f.s;
    double tx, ty;
    if (lhs) { if (left) { tx = -w / 2; ty = len / 2 + 0.6; } else { tx = w / 2; ty = len / 2; } }
    else { if (left) { tx = -w / 2; ty = len / 2; } else { tx = w / 2; ty = len / 2 + 0.6; } }
    const double bx[4] = {w / 2, w / 2, -w / 2, -w / 2};
    const double by[4] = {-len / 2, len / 2, len / 2, -len / 2};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double x = bx[k] + tx, y = by[k] + ty;
        cx[k] = (c * x - s * y) + xos;
        cy[k] = (s * x + c * y) + yos;
    }
}

// robot disc (GEOS 64-gon buffer) vs convex quad; unit circle table precomputed on the host
__constant__ double c_circ_cos[64];
__constant__ double c_circ_sin[64];

// GEOS's 64-gon buffer of the robot disc (Point.buffer(r)): vertex k at angle -k*pi/32
__device__ __forceinline__ double gon_x(double px, double r, int k)
{
    k &= 63;
    return k == 0 ? px + r : px + r * c_circ_cos[k];
}
__device__ __forceinline__ double gon_y(double py, double r, int k)
{
    k &= 63;
    return k == 0 ? py : py + r * c_circ_sin[k];
}

// Extents of the 64-gon on axis n: the vertex projections V_k.n = P.n + r|n|cos(theta_k - phi) peak at
// the vertex nearest phi (kmax) and bottom out opposite (kmax + 32); vertices two or more steps away
// are smaller by >= ~r|n|*pi^2/1024 relative to the extreme, ~10^12 times any rounding of a projection,
// so the extremes over a +-2 window equal those over all 64 vertices exactly (min / max are
// order-independent).
__device__ __forceinline__ void gon_extent(double px, double py, double r, double nx, double ny, int kmax,
                                           double &amin, double &amax)
{
    amin = INFINITY; amax = -INFINITY;
#pragma unroll
    for (int d = -2; d <= 2; ++d) {
        const double t = gon_x(px, r, kmax + d) * nx + gon_y(py, r, kmax + d) * ny;
        const double u = gon_x(px, r, kmax + 32 + d) * nx + gon_y(py, r, kmax + 32 + d) * ny;
        amax = t > amax ? t : amax;
        amin = u < amin ? u : amin;
    }
}

// One 64-gon edge axis of disc_quad_sat's second loop (edge k -> k + 1, extents over the +-2 vertex windows
// of gon_extent): true if it separates the 64-gon from the quad. Same vertices, same operations as the loop.
__device__ __forceinline__ bool gon_axis_separates(double px, double py, double r, const double *qx, const double *qy, int k)
{
    auto vx = [&](int idx) { idx &= 63; return idx == 0 ? px + r : px + r * c_circ_cos[idx]; };
    auto vy = [&](int idx) { idx &= 63; return idx == 0 ? py : py + r * c_circ_sin[idx]; };
    const double ex = vx(k + 1) - vx(k), ey = vy(k + 1) - vy(k);
    if (ex == 0.0 && ey == 0.0) return false;
    const double nx = -ey, ny = ex;
    double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const double t = vx(k - 2 + d) * nx + vy(k - 2 + d) * ny;
        const double u = vx(k + 30 + d) * nx + vy(k + 30 + d) * ny;
        amax = t > amax ? t : amax;
        amin = u < amin ? u : amin;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) { const double t = qx[v] * nx + qy[v] * ny; bmin = t < bmin ? t : bmin; bmax = t > bmax ? t : bmax; }
    return amax < bmin || bmax < amin;
}

// Separating-axis test over the edge normals of the quad and of the 64-gon (the predicate the oracle,
// oracle/cpu_ref.c:disc_quad_intersect, evaluates with all 64 vertices per axis): identical boolean. Only the
// fallback for degenerate quads / radii (and the test hook's mode 1), so written for few registers: loops
// not unrolled.
__device__ __forceinline__ bool disc_quad_sat(double px, double py, double r, const double *qx, const double *qy)
{
    const double step = CN_PI / 32;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {   // quad edges: the 64-gon's extreme vertex from the axis angle
        const int k1 = (k + 1) & 3;
        const double ex = qx[k1] - qx[k], ey = qy[k1] - qy[k];
        if (ex == 0.0 && ey == 0.0) continue;
        const double nx = -ey, ny = ex;
        const int kmax = ((int)rint(-atan2(ny, nx) / step) % 64 + 64) % 64;
        double amin, amax, bmin = INFINITY, bmax = -INFINITY;
        gon_extent(px, py, r, nx, ny, kmax, amin, amax);
#pragma unroll
        for (int v = 0; v < 4; ++v) { const double t = qx[v] * nx + qy[v] * ny; bmin = t < bmin ? t : bmin; bmax = t > bmax ? t : bmax; }
        if (amax < bmin || bmax < amin) return false;
    }
#pragma unroll 1
    for (int k = 0; k < 64; ++k)   // 64-gon edge k -> k+1 (its normal points at -(k + 1/2) pi/32)
        if (gon_axis_separates(px, py, r, qx, qy, k)) return false;
    return true;
}

// disc_quad_sat for a centre P OUTSIDE the quad within the boundary band (r cos(pi/64) - eps <= d <= r + eps,
// d = |c - P|, c the quad's closest point, (cx, cy) = c - P): the same boolean from the 4 quad axes and only
// the 64-gon edge axes whose direction lies within 3 steps of c - P or of P - c. Why no other axis can
// separate: an axis of unit direction u separates (amax < bmin) only if min_q (q - P).u exceeds the 64-gon's
// support (v - P).u, which is at least the apothem r cos(pi/64) for every u; but min_q (q - P).u <=
// (c - P).u = d cos(angle(u, c - P)) <= (r + eps) cos(angle). Edge k's normal points at -(k + 1/2) pi/32;
// ks, the nearest such edge to c - P, is within pi/64 (+ rounding of atan2 / rint) of it, so an edge 4 or
// more steps away is >= 3.5 pi/32 off: (r + eps) cos(3.5 pi/32) = 0.941 (r + eps) < 0.9988 r -- a margin of
// ~0.057 r against eps = 1e-9 and the ~1e-15 r rounding of the projections (r > 1e-6 here). The other
// condition (bmax < amin) is separation along -u: the window around ks + 32. SURVEY §9-7; the 100 k predicate
// cases of tests/test_norm_zone.py (the zones' corner-on-circle geometry included) check it against the
// oracle's all-axes test.
// kq >= 0: the quad is a norm zone (a rectangle rotated by dth, norm_zone), whose edge k's normal points at
// dth + pi + k pi/2, so the 64-gon's extreme vertex for it is (kq - 16 k) & 63 with kq = rint(-dth / step) - 32
// -- the vertex nearest the normal up to one step where the rounded edge vector's atan2 would round the other
// way, which gon_extent's +-2 window absorbs (its extremes are those of all 64 vertices for any kmax within one
// step of the nearest vertex): the same amin / amax, without four f64 atan2. kq < 0: atan2 per edge.
__device__ __forceinline__ bool disc_quad_sat_band(double px, double py, double r, const double *qx, const double *qy,
                                                   double cx, double cy, int kq)
{
    const double step = CN_PI / 32;
#pragma unroll 1
    for (int k = 0; k < 4; ++k) {   // quad edges, as in disc_quad_sat
        const int k1 = (k + 1) & 3;
        const double ex = qx[k1] - qx[k], ey = qy[k1] - qy[k];
        if (ex == 0.0 && ey == 0.0) continue;
        const double nx = -ey, ny = ex;
        const int kmax = kq >= 0 ? (kq - 16 * k) & 63 : ((int)rint(-atan2(ny, nx) / step) % 64 + 64) % 64;
        double amin, amax, bmin = INFINITY, bmax = -INFINITY;
        gon_extent(px, py, r, nx, ny, kmax, amin, amax);
#pragma unroll
        for (int v = 0; v < 4; ++v) { const double t = qx[v] * nx + qy[v] * ny; bmin = t < bmin ? t : bmin; bmax = t > bmax ? t : bmax; }
        if (amax < bmin || bmax < amin) return false;
    }
    const int ks = (int)rint(-atan2(cy, cx) / step - 0.5);
#pragma unroll 1
    for (int j = -3; j <= 3; ++j) {
        if (gon_axis_separates(px, py, r, qx, qy, (ks + j) & 63)) return false;
        if (gon_axis_separates(px, py, r, qx, qy, (ks + 32 + j) & 63)) return false;
    }
    return true;
}

__device__ __forceinline__ int disc_quad_classify(double px, double py, double r, const double *qx, const double *qy,
                                                  double sgn, double eps, double &cx, double &cy)
{
    bool inside = true;
    double d2 = INFINITY;   // squared distance from P to the quad's boundary segments
    cx = 0.0; cy = 0.0;     // closest boundary point - P
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int k1 = (k + 1) & 3;
        const double ex = qx[k1] - qx[k], ey = qy[k1] - qy[k];
        const double wx = px - qx[k], wy = py - qy[k];
        if (sgn * (ex * wy - ey * wx) < 0) inside = false;
        const double ee = ex * ex + ey * ey;
        double t = ee > 0 ? (wx * ex + wy * ey) / ee : 0.0;
        t = t < 0 ? 0 : (t > 1 ? 1 : t);
        const double dx = wx - t * ex, dy = wy - t * ey;
        const double dd = dx * dx + dy * dy;
        if (dd < d2) { d2 = dd; cx = -dx; cy = -dy; }
    }
    if (inside) return 1;
    const double d = sqrt(d2);
    if (d < r * 0.99879545620517241 - eps) return 1;   // cos(pi/64)
    if (d > r + eps) return 0;
    return -1;
}

// robot 64-gon vs a norm-zone quad (Point.buffer(r).intersects(zone), crowd_sim.py norm-zone penalty).
// Away from the boundary the answer is geometric: the 64-gon lies between the discs of radius
// r cos(pi/64) and r about P, so a centre distance to the (convex) quad below r cos(pi/64) - eps means
// intersecting and above r + eps disjoint (eps = 1e-9 >> rounding of the inputs); only the thin band in
// between runs the separating-axis test (disc_quad_sat_band's axes). Returns 1 / 0, or -1 for a degenerate
// quad or radius, which the full separating-axis test (disc_quad_sat) decides.
__device__ __forceinline__ int disc_quad_intersect3(double px, double py, double r, const double *qx, const double *qy,
                                                    int kq = -1)
{
    const double eps = 1e-9;
    double area2 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) area2 += qx[k] * qy[(k + 1) & 3] - qx[(k + 1) & 3] * qy[k];
    if (!(fabs(area2) > 1e-12 && r > 1e-6)) return -1;
    double cx, cy;
    // 1 / 0 decided by the distance classification, -1: the centre is in the band, outside the quad
    const int cls = disc_quad_classify(px, py, r, qx, qy, area2 > 0 ? 1.0 : -1.0, eps, cx, cy);
    return cls >= 0 ? cls : (int)disc_quad_sat_band(px, py, r, qx, qy, cx, cy, kq);
}

__device__ __forceinline__ bool disc_quad_intersect(double px, double py, double r, const double *qx, const double *qy)
{
    const int v = disc_quad_intersect3(px, py, r, qx, qy);
    return v >= 0 ? v != 0 : disc_quad_sat(px, py, r, qx, qy);
}

// crowd_sim.py:918-926,957-960 (norm zones on): both zones are built around the robot and
// tested against its own disc. Out of line: the separating-axis tests would otherwise raise the step
// kernel's register pressure (and scratch) for every workload, norm zones on or off. Returns 1 / 0, or -1
// when a zone is degenerate (a robot radius <= 1e-6): robot_norm_zone_violation then decides with the full
// separating-axis test. Two callees, each without calls of its own: a callee's VGPR count (the highest
// register it touches, callee-saved ones included when it calls further) is charged to every kernel that
// calls it, beyond the kernel's launch bounds.
__device__ __noinline__ int robot_norm_zone_fast(double px, double py, double vx, double vy, double rr, bool f32, int lhs)
{
    double zx[4], zy[4];
    const ZoneFrame f = zone_frame(px, py, vx, vy, rr, f32);   // the heading's trigonometry once for both zones
    const int kq = ((int)rint(-f.dth / (CN_PI / 32)) - 32) & 63;
#pragma unroll 1
    for (int z = 0; z < 2; ++z) {
        norm_zone(f, rr, lhs, z == 0, zx, zy);
        const int v = disc_quad_intersect3(px, py, rr, zx, zy, kq);
        if (v != 0) return v;
    }
    return 0;
}

__device__ __noinline__ bool robot_norm_zone_full(double px, double py, double vx, double vy, double rr, bool f32, int lhs)
{
    double zx[4], zy[4];
    const ZoneFrame f = zone_frame(px, py, vx, vy, rr, f32);
#pragma unroll 1
    for (int z = 0; z < 2; ++z) {
        norm_zone(f, rr, lhs, z == 0, zx, zy);
        if (disc_quad_sat(px, py, rr, zx, zy)) return true;
    }
    return false;
}

__device__ __forceinline__ bool robot_norm_zone_violation(double px, double py, double vx, double vy, double rr, bool f32,
                                                          int lhs)
{
    const int v = robot_norm_zone_fast(px, py, vx, vy, rr, f32, lhs);
    return v >= 0 ? v != 0 : robot_norm_zone_full(px, py, vx, vy, rr, f32, lhs);
}

// ------------------------------------------------------------------------------------------------
// RVO2 v2.0 agent-0 solve (float32) with ORCA lines in LDS ([line][lane] float4: point.xy, dir.xy)
// ------------------------------------------------------------------------------------------------
#define RVO_EPSILON 0.00001f

__device__ inline float det2(float ax, float ay, float bx, float by) { return ax * by - ay * bx; }

// a / b, IEEE-rounded, for the linear programs' quotients: |b| > RVO_EPSILON (the callers ignore the
// quotient when |b| <= RVO_EPSILON, RVO2's parallel-line branch) and |b| <= 2 (determinants of unit
// direction vectors). This is the compiler's correctly rounded f32 division (v_div_scale, rcp, one
// reciprocal and two quotient refinements by FMA, v_div_fmas, v_div_fixup) without the steps that are
// identities on that domain: v_div_scale only rescales a denormal divisor or an exponent gap of >= 96
// (so VCC = 0 and v_div_fmas is a plain FMA), and v_div_fixup only rewrites zero / inf / NaN operands and
// over/underflowed quotients. The FMA residuals a - b*q are exact only while they stay above the denormal
// range, i.e. for |a| >= ~2^-100: a numerator below 2^-96 (zero included) takes the full division instead
// (a rarely taken branch). tools/fdiv_lp_check.hip compares this with `/` bit for bit over numerators of
// every exponent (denormals included) and that divisor domain.
__device__ __forceinline__ float fdiv_lp(float a, float b)
{
    if (__builtin_expect(__builtin_fabsf(a) < 0x1p-96f, 0)) return a / b;
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
    const float q0 = a * y1;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y1, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), y1, q1);
}

// projected line of LP3's line li against lj (`valid` false when RVO2 skips it: parallel, same direction)
__device__ __forceinline__ float4 proj_line(const float4 li, const float4 lj, bool &valid)
{
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    const float determinant = det2(li.z, li.w, lj.z, lj.w);
    valid = true;
    if (fabsf(determinant) <= RVO_EPSILON) {
        if (li.z * lj.z + li.w * lj.w > 0.0f) { valid = false; return r; }
        r.x = 0.5f * (li.x + lj.x);
        r.y = 0.5f * (li.y + lj.y);
    } else {
        const float s = fdiv_lp(det2(lj.z, lj.w, li.x - lj.x, li.y - lj.y), determinant);
        r.x = li.x + s * li.z;
        r.y = li.y + s * li.w;
    }
    const float ddx = lj.z - li.z, ddy = lj.w - li.w;
    const float inv = fdiv(1.0f, fsqrt(ddx * ddx + ddy * ddy));
    r.z = ddx * inv; r.w = ddy * inv;
    return r;
}

// ------------------------------------------------------------------------------------------------
// ORCA linear programs on a QUAD of lanes per human (A <= 10). The lines live in LDS ([human][M]);
// every quad-uniform quantity (the result, loop indices, branch conditions) is computed redundantly by
// the 4 lanes, and the inner loop of linearProgram1 over the earlier lines is split across them: lane s
// takes lines s, s+4, ... and the quad combines tLeft = max, tRight = min and the parallel-line failure.
// tLeft only grows and tRight only shrinks in RVO2's sequential loop, and its exits ("tLeft > tRight",
// "parallel line with numerator < 0") are order independent, so the combined result is RVO2's.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float quad_xor1(float x)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float quad_xor2(float x)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ int quad_xor1i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_xor2i(int x) { return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ float quad_min(float x)
{
    float y = quad_xor1(x); x = y < x ? y : x;
    y = quad_xor2(x); return y < x ? y : x;
}
__device__ __forceinline__ float quad_max(float x)
{
    float y = quad_xor1(x); x = x < y ? y : x;
    y = quad_xor2(x); return x < y ? y : x;
}
__device__ __forceinline__ int quad_or(int x)
{
    x |= quad_xor1i(x);
    return x | quad_xor2i(x);
}

// 64-bit quad OR (MT = uint64_t masks: simulators of more than 32 agents, cn_orca_predict_kd only)
__device__ __forceinline__ uint32_t quad_or_m(uint32_t x) { return (uint32_t)quad_or((int)x); }
__device__ __forceinline__ uint64_t quad_or_m(uint64_t x)
{
    return (uint64_t)(uint32_t)quad_or((int)(uint32_t)x) | ((uint64_t)(uint32_t)quad_or((int)(uint32_t)(x >> 32)) << 32);
}

// linearProgram1 on line `no` of Lb (valid lines: bits of vmask), quad-cooperative. MT: the line mask type
// (uint32_t: <= 32 lines, the step kernel; uint64_t: <= 64, the plugin's large simulators)
template <typename MT = uint32_t>
__device__ __forceinline__ bool lp1_q(const float4 *Lb, MT vmask, int no, float radius, int s, float &tL,
                                      float &tR)
{
    const float4 ln = Lb[no];
    const float dot = ln.x * ln.z + ln.y * ln.w;
    const float disc = dot * dot + radius * radius - (ln.x * ln.x + ln.y * ln.y);
    const float sd = fsqrt(disc);
    float ptl = -INFINITY, ptr = INFINITY;
    for (int j = s; j < no; j += 4) {
        if (!((vmask >> j) & (MT)1)) continue;
        const float4 li = Lb[j];
        const float den = det2(ln.z, ln.w, li.z, li.w);
        const float num = det2(li.z, li.w, ln.x - li.x, ln.y - li.y);
        const bool par = fabsf(den) <= RVO_EPSILON;
        const float t = fdiv_lp(num, den);
        if (!par && den >= 0.0f && t < ptr) ptr = t;
        if (!par && !(den >= 0.0f) && ptl < t) ptl = t;
        if (par && num < 0.0f) ptl = INFINITY;   // RVO2's parallel-line failure (as in lp1_r)
    }
    ptr = quad_min(ptr);
    ptl = quad_max(ptl);
    float tr = -dot + sd, tl = -dot - sd;
    tr = ptr < tr ? ptr : tr;
    tl = tl < ptl ? ptl : tl;
    tL = tl; tR = tr;
    return !(disc < 0.0f || tl > tr);
}

// linearProgram2 (optimize closest to (ox, oy)); returns the index of the failing line or n
template <typename MT = uint32_t>
__device__ __forceinline__ int lp2_q(const float4 *Lb, int n, float radius, float ox, float oy, int s, float &rx,
                                     float &ry)
{
    if (ox * ox + oy * oy > radius * radius) {
        const float inv = fdiv(1.0f, fsqrt(ox * ox + oy * oy));
        rx = (ox * inv) * radius; ry = (oy * inv) * radius;
    } else { rx = ox; ry = oy; }
    for (int i = 0; i < n; ++i) {
        const float4 li = Lb[i];
        if (det2(li.z, li.w, li.x - rx, li.y - ry) > 0.0f) {
            float tL, tR;
            if (!lp1_q<MT>(Lb, ~(MT)0, i, radius, s, tL, tR)) return i;
            const float t = li.z * (ox - li.x) + li.w * (oy - li.y);
            if (t < tL) { rx = li.x + tL * li.z; ry = li.y + tL * li.w; }
            else if (t > tR) { rx = li.x + tR * li.z; ry = li.y + tR * li.w; }
            else { rx = li.x + t * li.z; ry = li.y + t * li.w; }
        }
    }
    return n;
}

// linearProgram3 from line `begin` (agents only); Pb = the human's projected-line scratch
template <typename MT = uint32_t>
__device__ __forceinline__ void lp3_q(const float4 *Lb, float4 *Pb, int n, int begin, float radius, int s, float &rx,
                                      float &ry)
{
    float distance = 0.0f;
    for (int i = begin; i < n; ++i) {
        const float4 li = Lb[i];
        if (det2(li.z, li.w, li.x - rx, li.y - ry) > distance) {
            MT pv = 0;
            for (int j = s; j < i; j += 4) {
                bool v;
                const float4 pj = proj_line(li, Lb[j], v);
                Pb[j] = pj;
                if (v) pv |= (MT)1 << j;
            }
            pv = quad_or_m(pv);
            wsync();
            const float tx = rx, ty = ry;
            const float ox = -li.w, oy = li.z;   // linearProgram2(projLines, radius, (-d.y, d.x), true)
            rx = ox * radius; ry = oy * radius;
            bool fail = false;
            for (int k = 0; k < i && !fail; ++k) {
                if (!((pv >> k) & (MT)1)) continue;
                const float4 pk = Pb[k];
                if (det2(pk.z, pk.w, pk.x - rx, pk.y - ry) > 0.0f) {
                    float tL, tR;
                    if (!lp1_q<MT>(Pb, pv, k, radius, s, tL, tR)) fail = true;
                    else if (ox * pk.z + oy * pk.w > 0.0f) { rx = pk.x + tR * pk.z; ry = pk.y + tR * pk.w; }
                    else { rx = pk.x + tL * pk.z; ry = pk.y + tL * pk.w; }
                }
            }
            if (fail) { rx = tx; ry = ty; }
            distance = det2(li.z, li.w, li.x - rx, li.y - ry);
            wsync();
        }
    }
}

// ------------------------------------------------------------------------------------------------
// The same linear programs with the lines in REGISTERS (quad path, <= 4 * NU lines): lane s of the quad
// holds lines s, s+4, ..., s+4(NU-1) (R[u] = line s + 4u) and line i reaches the whole quad by a DPP
// quad_perm broadcast from lane i & 3 -- the loops over lines are unrolled, so every broadcast has a
// compile-time source lane and no LDS round trip sits on the linear programs' dependent chain. Same
// operations in the same order as lp1_q / lp2_q / lp3_q, so the same bits.
// ------------------------------------------------------------------------------------------------
template <int T>
__device__ __forceinline__ float qbc(float x)   // quad_perm(T, T, T, T): lane T of the quad to all four
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), T * 0x55, 0xF, 0xF, false));
}
__device__ __forceinline__ float4 qbc4(const float4 v, int t)   // t folds to a constant once unrolled
{
    switch (t & 3) {
    case 0: return make_float4(qbc<0>(v.x), qbc<0>(v.y), qbc<0>(v.z), qbc<0>(v.w));
    case 1: return make_float4(qbc<1>(v.x), qbc<1>(v.y), qbc<1>(v.z), qbc<1>(v.w));
    case 2: return make_float4(qbc<2>(v.x), qbc<2>(v.y), qbc<2>(v.z), qbc<2>(v.w));
    default: return make_float4(qbc<3>(v.x), qbc<3>(v.y), qbc<3>(v.z), qbc<3>(v.w));
    }
}
__device__ __forceinline__ float qbcf(const float v, int t)
{
    switch (t & 3) {
    case 0: return qbc<0>(v);
    case 1: return qbc<1>(v);
    case 2: return qbc<2>(v);
    default: return qbc<3>(v);
    }
}

// linearProgram1 on line `no` (= ln, already broadcast) against the valid (vmask) lines j < no of R
template <int NU>
__device__ __forceinline__ bool lp1_r(const float4 (&R)[NU], uint32_t vmask, int no, const float4 ln, float radius,
                                      int s, float &tL, float &tR)
{
    const float dot = ln.x * ln.z + ln.y * ln.w;
    const float disc = dot * dot + radius * radius - (ln.x * ln.x + ln.y * ln.y);
    const float sd = fsqrt(disc);
    float ptl = -INFINITY, ptr = INFINITY;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int j = s + 4 * u;
        if (j < no && ((vmask >> j) & 1u)) {
            const float4 li = R[u];
            const float den = det2(ln.z, ln.w, li.z, li.w);
            const float num = det2(li.z, li.w, ln.x - li.x, ln.y - li.y);
            const bool par = fabsf(den) <= RVO_EPSILON;
            const float t = fdiv_lp(num, den);
            if (!par && den >= 0.0f && t < ptr) ptr = t;
            if (!par && !(den >= 0.0f) && ptl < t) ptl = t;
            // RVO2 fails on a parallel line with numerator < 0: tLeft = +inf (> any tRight, t is finite)
            // fails the same test below, and rides the max reduction instead of a third quad reduction
            if (par && num < 0.0f) ptl = INFINITY;
        }
    }
    ptr = quad_min(ptr);
    ptl = quad_max(ptl);
    float tr = -dot + sd, tl = -dot - sd;
    tr = ptr < tr ? ptr : tr;
    tl = tl < ptl ? ptl : tl;
    tL = tl; tR = tr;
    return !(disc < 0.0f || tl > tr);
}

// linearProgram2 (optimize closest to (ox, oy)) over the n lines of R; returns the failing line or n
template <int NU>
__device__ __forceinline__ int lp2_r(const float4 (&R)[NU], int n, float radius, float ox, float oy, int s, float &rx,
                                     float &ry)
{
    if (ox * ox + oy * oy > radius * radius) {
        const float inv = fdiv(1.0f, fsqrt(ox * ox + oy * oy));
        rx = (ox * inv) * radius; ry = (oy * inv) * radius;
    } else { rx = ox; ry = oy; }
    int fail = n;
#pragma unroll
    for (int i = 0; i < 4 * NU; ++i) {
        if (i < n && fail == n) {   // quad-uniform
            const float4 li = qbc4(R[i >> 2], i);
            if (det2(li.z, li.w, li.x - rx, li.y - ry) > 0.0f) {
                float tL, tR;
                if (!lp1_r<NU>(R, ~0u, i, li, radius, s, tL, tR)) fail = i;
                else {
                    const float t = li.z * (ox - li.x) + li.w * (oy - li.y);
                    if (t < tL) { rx = li.x + tL * li.z; ry = li.y + tL * li.w; }
                    else if (t > tR) { rx = li.x + tR * li.z; ry = li.y + tR * li.w; }
                    else { rx = li.x + t * li.z; ry = li.y + t * li.w; }
                }
            }
        }
    }
    return fail;
}

// RVO2 linearProgram3's sub-problem for line i: linearProgram2 over the projections of lines 0..i-1 onto
// line i (R: lane s holds lines s + 4u), optimising direction (-d.y, d.x) from result = opt * radius.
// Depends on the lines only. Returns false when it fails (RVO2 then keeps the result it had).
template <int NU>
__device__ __forceinline__ bool lp3_sub(const float4 (&R)[NU], const float4 li, int i, float radius, int s, float &rx,
                                        float &ry)
{
    float4 P[NU];
    uint32_t pv = 0;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int j = s + 4 * u;
        P[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < i) {
            bool v;
            P[u] = proj_line(li, R[u], v);
            if (v) pv |= 1u << j;
        }
    }
    pv = (uint32_t)quad_or((int)pv);
    const float ox = -li.w, oy = li.z;   // linearProgram2(projLines, radius, (-d.y, d.x), true)
    rx = ox * radius; ry = oy * radius;
    bool fail = false;
#pragma unroll
    for (int k = 0; k < 4 * NU; ++k) {
        if (k < i && !fail && ((pv >> k) & 1u)) {   // quad-uniform
            const float4 pk = qbc4(P[k >> 2], k);
            if (det2(pk.z, pk.w, pk.x - rx, pk.y - ry) > 0.0f) {
                float tL, tR;
                if (!lp1_r<NU>(P, pv, k, pk, radius, s, tL, tR)) fail = true;
                else if (ox * pk.z + oy * pk.w > 0.0f) { rx = pk.x + tR * pk.z; ry = pk.y + tR * pk.w; }
                else { rx = pk.x + tL * pk.z; ry = pk.y + tL * pk.w; }
            }
        }
    }
    return !fail;
}

// linearProgram3 from line `begin`; Lb = the same lines in LDS (line i of the outer loop is read from
// there: its index is dynamic), the projected lines stay in registers (lane s: j = s + 4u)
template <int NU>
__device__ __forceinline__ void lp3_r(const float4 (&R)[NU], const float4 *Lb, int n, int begin, float radius, int s,
                                      float &rx, float &ry)
{
    float distance = 0.0f;
    for (int i = begin; i < n; ++i) {
        const float4 li = Lb[i];
        if (det2(li.z, li.w, li.x - rx, li.y - ry) > distance) {
            float qx, qy;
            if (lp3_sub<NU>(R, li, i, radius, s, qx, qy)) { rx = qx; ry = qy; }
            distance = det2(li.z, li.w, li.x - rx, li.y - ry);
        }
    }
}

// The linearProgram3 sub-problems of a whole workgroup, spread over all its quads (the quad path's step
// kernel). Sub-problem (h, i) -- human h's line i -- depends on h's lines only, not on the result RVO2's
// loop has reached when it visits line i, so every one that the loop may visit (i in [fail, n) of each
// human whose linearProgram2 failed at `fail`) is solved up front, by any quad: sorted by i (descending),
// so the 16 quads of a wave run sub-problems of about the same size side by side, and one human's
// sub-problems run on different quads at once. Each human's quad then replays RVO2's loop (lp3_replay).
// The serial version puts a human's whole loop on its own quad, and the wave runs the union of its 16
// humans' control flow: for crowded circle crossings that was half of the C2 launch.
// bn[h] = fail | n << 8 (0: no linearProgram3); results to res / rok [h][12].
template <int NU>
__device__ __forceinline__ void lp3_tasks(const float4 *lines, int M, const float *vmax, const uint32_t *bn,
                                          float2 *res, uint8_t *rok, int tid)
{
    const int q = tid >> 2, sq = tid & 3;
    const uint32_t b = bn[tid & 63];
    const int b0 = (int)(b & 0xffu), b1 = (int)(b >> 8);
    uint64_t mk[4 * NU];
    int cn[4 * NU], T = 0;
#pragma unroll
    for (int i = 0; i < 4 * NU; ++i) {   // humans with sub-problem i (wave-uniform)
        mk[i] = __ballot(b0 <= i && i < b1);
        cn[i] = __popcll(mk[i]);
        T += cn[i];
    }
    for (int t = q; t < T; t += 64) {   // quad-uniform
        int i = 0, k = 0, acc = 0;
        uint64_t m = 0;
        bool found = false;
#pragma unroll
        for (int ii = 4 * NU - 1; ii >= 0; --ii) {
            if (!found && t < acc + cn[ii]) { found = true; i = ii; k = t - acc; m = mk[ii]; }
            acc += cn[ii];
        }
        for (int z = 0; z < k; ++z) m &= m - 1;   // the k-th human with sub-problem i
        const int h = __ffsll((long long)m) - 1;
        const float4 *Lh = lines + h * M;
        float4 R[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) R[u] = sq + 4 * u < i ? Lh[sq + 4 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
        float qx, qy;
        const bool ok = lp3_sub<NU>(R, Lh[i], i, vmax[h], sq, qx, qy);
        if (sq == 0) { res[h * 12 + i] = make_float2(qx, qy); rok[h * 12 + i] = ok ? 1 : 0; }
    }
}

// RVO2's linearProgram3 loop over the sub-problems lp3_tasks solved (lines < `end`), quad-uniform; a visited
// line >= end has its sub-problem solved here, by the human's own quad (R: its lines, lane s: s + 4u)
template <int NU>
__device__ __forceinline__ int lp3_replay(const float4 (&R)[NU], const float4 *Lb, int n, int begin, int end,
                                          float radius, int s, const float2 *res, const uint8_t *rok, float &rx,
                                          float &ry)
{
    float distance = 0.0f;
    int vis = 0;
    for (int i = begin; i < n; ++i) {
        const float4 li = Lb[i];
        if (det2(li.z, li.w, li.x - rx, li.y - ry) > distance) {
            ++vis;
            if (i < end) {
                if (rok[i]) { const float2 r2 = res[i]; rx = r2.x; ry = r2.y; }
            } else {
                float qx, qy;
                if (lp3_sub<NU>(R, li, i, radius, s, qx, qy)) { rx = qx; ry = qy; }
            }
            distance = det2(li.z, li.w, li.x - rx, li.y - ry);
        }
    }
    return vis;
}

// one ORCA line (Agent::computeNewVelocity, agent branch) of self vs another agent
__device__ __forceinline__ float4 orca_line(float X0, float Y0, float VX0, float VY0, float R0, float ox, float oy,
                                           float ovx, float ovy, float orr, float invTH, float invTS)
{
    const float rpx = ox - X0, rpy = oy - Y0;
    const float rvx = VX0 - ovx, rvy = VY0 - ovy;
    const float distSq = rpx * rpx + rpy * rpy;
    const float cr = R0 + orr;
    const float crSq = cr * cr;
    float ux, uy, dx, dy;
    if (distSq > crSq) {
        const float wx = rvx - invTH * rpx, wy = rvy - invTH * rpy;
        const float wLenSq = wx * wx + wy * wy;
        const float dot1 = wx * rpx + wy * rpy;
        if (dot1 < 0.0f && dot1 * dot1 > crSq * wLenSq) {
            const float wLen = fsqrt(wLenSq);
            const float inv = fdiv(1.0f, wLen);
            const float uwx = wx * inv, uwy = wy * inv;
            dx = uwy; dy = -uwx;
            const float s = cr * invTH - wLen;
            ux = s * uwx; uy = s * uwy;
        } else {
            const float leg = fsqrt(distSq - crSq);
            const float inv = fdiv(1.0f, distSq);
            if (det2(rpx, rpy, wx, wy) > 0.0f) {
                dx = (rpx * leg - rpy * cr) * inv;
                dy = (rpx * cr + rpy * leg) * inv;
            } else {
                dx = -((rpx * leg + rpy * cr) * inv);
                dy = -((-rpx * cr + rpy * leg) * inv);
            }
            const float dot2 = rvx * dx + rvy * dy;
            ux = dot2 * dx - rvx; uy = dot2 * dy - rvy;
        }
    } else {
        const float wx = rvx - invTS * rpx, wy = rvy - invTS * rpy;
        const float wLen = fsqrt(wx * wx + wy * wy);
        const float inv = fdiv(1.0f, wLen);
        const float uwx = wx * inv, uwy = wy * inv;
        dx = uwy; dy = -uwx;
        const float s = cr * invTS - wLen;
        ux = s * uwx; uy = s * uwy;
    }
    return make_float4(VX0 + 0.5f * ux, VY0 + 0.5f * uy, dx, dy);
}

// Agent::computeNeighbors + the agent loop of Agent::computeNewVelocity for a simulator of <= 13 agents
// (RVO2's KdTree is a single leaf for <= 10: the neighbours are the in-range slots stably sorted by distSq
// in slot order), quad-cooperative: lane sq builds the lines of slots sq, sq+4, sq+8 and ranks them itself
// against the quad's distances, gathered by DPP broadcasts (no LDS round trip).
// `slot(k, x, y, vx, vy, r)` gives observed slot k (agent k + 1) in float32. Lines land in Lb[rank].
// Returns the number of lines. Shared by cn_step_kernel and cn_debug_orca.
template <typename SlotF>
__device__ __forceinline__ int orca_lines_quad(const SlotF &slot, int M, int sq, float X0, float Y0, float VX0,
                                               float VY0, float R0, float rangeSq, float invTH, float invTS,
                                               float4 *Lb)
{
    float4 rawv[3];
    float dv[3];
    uint32_t inm = 0;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int k = sq + 4 * u;
        rawv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        dv[u] = 0.0f;
        if (k < M) {
            float x, y, vx, vy, r;
            slot(k, x, y, vx, vy, r);
            const float dx = X0 - x, dy = Y0 - y;
            dv[u] = dx * dx + dy * dy;
            if (dv[u] < rangeSq) inm |= 1u << k;
            rawv[u] = orca_line(X0, Y0, VX0, VY0, R0, x, y, vx, vy, r, invTH, invTS);
        }
    }
    inm = (uint32_t)quad_or((int)inm);
    float dq[12];   // distSq of slot q = 4u + t (lane t's dv[u]), broadcast with the whole quad active
#pragma unroll
    for (int q = 0; q < 12; ++q) dq[q] = qbcf(dv[q >> 2], q);
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int k = sq + 4 * u;
        if (k < M && ((inm >> k) & 1u)) {
            int rank = 0;
#pragma unroll
            for (int q = 0; q < 12; ++q)
                if (((inm >> q) & 1u) && (dq[q] < dv[u] || (dq[q] == dv[u] && q < k))) ++rank;
            Lb[rank] = rawv[u];
        }
    }
    return __popc(inm);
}

// ------------------------------------------------------------------------------------------------
// RNG work (goal changes, spawn): numpy legacy MT19937 per env, one wave per env
// ------------------------------------------------------------------------------------------------
// Pending next-episode spawns. CrowdSimDict.reset (crowd_sim_dict.py:105-203) is a pure function of the
// seed schedule (offset + case_counter + thisSeed) and the scenario, both fixed as soon as the previous
// reset has run, so the spawn of env e's NEXT episode is drawn ahead of time by spare waves of kernel A
// (off the critical path) and kernel B's auto-reset only copies it. (case_counter, reset_count) is
// the validity key: a stale entry (e.g. after cn_set_state) is never used, the reset is then drawn inline.
// Two slots per env (slot = reset_count & 1): the spawn of the env's next reset and of the one after, so
// an env that ends an episode one step after a reset (common where spawns overlap, e.g. 25 humans in
// square_crossing) finds its spawn drawn instead of drawing it inline. Arrays are [2][...].
struct PendPtrs {
    uint32_t *mt;   // [E][624] key words after the spawn draws
    int32_t *pos;   // [E] stream position
    uint32_t *ovf;  // [E] bounded-rejection overflows of the spawn
    int32_t *sc;    // [E] scenario
    int64_t *cc;    // [E] key: case_counter the spawn was drawn for
    int32_t *rc;    // [E] key: reset_count (sequential scenario mode)
    uint64_t *ok;   // [E] (reset_count key << 32) | id of the launch that completed the entry (0: parked / none);
                    // one 8-byte store, written last: consumed only by a LATER launch, and only for its own key
    int32_t *prog;  // [E] humans placed so far by a spawn parked mid-way (resumable spawns)
    double *r;      // [5][E] robot px, py, gx, gy, theta
    double *h;      // [7][E*N] human px, py, gx, gy, radius, v_pref, theta
};
__host__ __device__ inline PendPtrs pend_slot(const PendPtrs &P, int s, int64_t E, int64_t EN)
{
    PendPtrs q = P;
    q.mt += s * E * CN_MT_N; q.pos += s * E; q.ovf += s * E; q.sc += s * E; q.cc += s * E; q.rc += s * E;
    q.ok += s * E; q.prog += s * E; q.r += s * 5 * E; q.h += s * 7 * EN;
    return q;
}

// Output view of a group engine inside a mixed engine (cn_create_mixed): local env e of
// the group is row `row[e]` of the caller's (E_total, ...) buffers, whose spatial_edges have NS human
// slots (NS >= N; slots N..NS-1 are padding). row == nullptr: identity, NS == N (a plain engine).
struct OutView {
    const int32_t *row;
    int NS;
};
__device__ __forceinline__ int64_t orow(const OutView &v, int64_t e) { return v.row ? (int64_t)v.row[e] : e; }
// padding slot of a mixed engine's spatial_edges: a human that is never seen, i.e. the belief the
// reference gives an unseen human at reset (crowd_sim.py:437-455: [15, 15, 0, 0, 0.3], zero velocity, so
// it never moves), relative to the robot
#define CN_PAD_POS 15.0

// where a reset writes: state + the first observation of the new episode
struct ResetOut {
    cn_state_ptrs s;
    float *robot_node, *temporal, *spatial;
    int64_t case_size;
    OutView ov;
};

// pending-spawn modes of a step launch (PendLaunch::all): after cn_set_state every env's next spawn and the one
// after are drawn (resets of that launch draw inline); after cn_reset the reset kernel drew both (ok word
// CN_OK_RESET, never a step launch's id) and the launch draws none -- both modes ignore the spawn and resume
// lists of launches before them
#define PEND_BOTH 1
#define PEND_FRESH 2
#define CN_OK_RESET 0xffffffffu

struct RngArgs {   // cn_reset_kernel
    ResetOut o;
    PendPtrs pend;
    int E;
    int64_t counter_offset;
    int draw_next;   // also draw the spawns of every env's next two resets (then PEND_FRESH)
};


// numpy MT19937 stream over a two-block LDS ring: block 0 = current key words, block 1 = the key after
// the next mt19937_gen. Every lane of the (single-wave) workgroup keeps the same stream position `p`;
// "sequential" draws are read by all lanes (LDS broadcast), and rejection loops evaluate up to 64
// consecutive tries speculatively, one per lane, since each try consumes a fixed number of words.

// wave-cooperative mt19937_gen: n = gen(o) (all 64 lanes of the workgroup must call it). Three
// sections, each with all its LDS loads issued before its stores: new[k] for k < 227 needs old words
// only; k in [227, 454) needs new[k - 227] of the first section, k in [454, 624) new words of the second
// (k = 623 wraps to new[0], and its new[396] is second-section too).
__device__ __forceinline__ void mt_gen_wave_inl(const uint32_t *__restrict__ o, uint32_t *__restrict__ n, int lane)
{
    constexpr int S = CN_MT_N - 397;   // 227
#pragma unroll
    for (int sec = 0; sec < 3; ++sec) {
        const int lo = sec * S, hi = sec == 2 ? CN_MT_N : (sec + 1) * S;
        uint32_t a[4], b[4], cc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = lo + lane + 64 * j;
            if (k < hi) {
                a[j] = o[k];
                b[j] = k + 1 < CN_MT_N ? o[k + 1] : n[0];
                cc[j] = sec == 0 ? o[k + 397] : n[k - S];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = lo + lane + 64 * j;
            if (k < hi) n[k] = mt_mix(a[j], b[j], cc[j]);
        }
        wsync();
    }
}

// out of line for the many rarely-taken call sites (inlined everywhere, the step kernel's code grew by
// half and ran slower); the crowded rejection loop, which twists a block per pass, inlines it
__device__ __noinline__ void mt_gen_wave(const uint32_t *__restrict__ o, uint32_t *__restrict__ n, int lane)
{
    mt_gen_wave_inl(o, n, lane);
}

__device__ __forceinline__ double mt_dbl(const uint32_t *w, int q)
{
    const int32_t a = (int32_t)(mt_temper(w[q]) >> 5), b = (int32_t)(mt_temper(w[q + 1]) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}
// the same over the ping-pong ring: logical word q lives at (q + off) mod 2*624
__device__ __forceinline__ double mt_dbl_ring(const uint32_t *w, int q, int off)
{
    int i = q + off;
    i -= i >= 2 * CN_MT_N ? 2 * CN_MT_N : 0;
    const int i1 = i + 1 == 2 * CN_MT_N ? 0 : i + 1;
    const int32_t a = (int32_t)(mt_temper(w[i]) >> 5), b = (int32_t)(mt_temper(w[i1]) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

// CN_RNG_PHILOX (`phx`): word q is philox(q >> 2) under the episode key (`key`, also kept in w[0] for the
// state write-back); the ring is unused, p counts words from the reset and ensure() is a no-op.
struct WRng {
    double *sl;    // LDS [6][64] per-try candidate slots (wave_reject2)
    uint32_t *w;   // LDS [2*624], a ping-pong ring: logical block 0 (the key) starts at word `off`
    int off;       // 0 or 624
    int p;         // stream position (wave-uniform), 0 .. 2*624 (MT19937) / words since the reset (Philox)
    bool have1;    // block 1 generated
    bool slid;     // the key advanced by at least one whole block (key words must be written back)
    bool phx;      // CN_RNG_PHILOX
    int64_t edbg;  // env index for the -DCN_STAMPS diagnostics
    char *grid;    // CN_GRID_LDS bytes of LDS for the spawn's crowded rejection (DiscGrid + agent table), or null
    uint32_t key;  // Philox key word 0 (the episode seed)
    int lane;
    __device__ double dbl(int q) const { return phx ? philox_dbl(key, q) : mt_dbl_ring(w, q, off); }
    // logical block i (0 = the key, 1 = the key after the next mt19937_gen)
    __device__ uint32_t *blk(int i) const { return w + ((off + i * CN_MT_N) % (2 * CN_MT_N)); }
    // R * cos(angle) with angle = rnd() * pi * 2 (crowd_sim.py:361, 736), for cand_attributes
    __device__ double cos2pi(int q) const { return cos(dbl(q) * CN_PI * 2); }
    __device__ double sin2pi(int q) const { return sin(dbl(q) * CN_PI * 2); }
    // make words [p, p + need) readable (need <= 624); all lanes call it together
    template <bool INL = false>
    __device__ void ensure(int need)
    {
        if (phx) return;
        if (p + need > CN_MT_N && !have1) {
            if (INL) mt_gen_wave_inl(blk(0), blk(1), lane); else mt_gen_wave(blk(0), blk(1), lane);
            have1 = true;
        }
        if (p + need > 2 * CN_MT_N) {   // slide: block 1 becomes the key, the next block overwrites block 0
            wsync();
            off = off ? 0 : CN_MT_N;
            if (INL) mt_gen_wave_inl(blk(0), blk(1), lane); else mt_gen_wave(blk(0), blk(1), lane);
            p -= CN_MT_N;
            slid = true;
        }
    }
    __device__ double rnd() { ensure(2); const double d = dbl(p); p += 2; return d; }
    __device__ double unif(double lo, double hi) { return lo + (hi - lo) * rnd(); }
};

// words one try of create_agent_attributes(scenario) consumes (crowd_sim.py:296-357)
__host__ __device__ inline int cand_words(int scenario)
{
    switch (scenario) {
    case CN_SC_CIRCLE_CROSSING: return 6;
    case CN_SC_SQUARE_CROSSING: return 12;
    case CN_SC_PARALLEL_TRAFFIC: case CN_SC_PERPENDICULAR_TRAFFIC: return 10;
    default: return 6;
    }
}

// create_agent_attributes from the words starting at q
template <typename Src>
__device__ void cand_attributes(const cn_config &c, const Src &w, int q, int scenario, double agent_vpref,
                                double agent_radius, double robot_radius, double &px, double &py, double &gx,
                                double &gy, double &heading, double &vp)
{
    double v_pref = agent_vpref == 0 ? 1.0 : agent_vpref;
    const double pxn = (w.dbl(q) - 0.5) * v_pref;
    const double pyn = (w.dbl(q + 2) - 0.5) * v_pref;
    q += 4;
    const double R = c.circle_radius;
    auto rwp = [&](int qq) { return (w.dbl(qq) - 0.5) * c.square_width / 2; };
    heading = 0;
    switch (scenario) {
    case CN_SC_CIRCLE_CROSSING:
        px = R * w.cos2pi(q) + pxn; py = R * w.sin2pi(q) + pyn;
        gx = -px; gy = -py;
        break;
    case CN_SC_SQUARE_CROSSING:
        px = rwp(q) * 0.4 + pxn;
        py = rwp(q + 2) * 0.4 + pyn;
        gx = rwp(q + 4) * 0.4 + pxn;
        gy = rwp(q + 6) * 0.4 + pyn;
        break;
    case CN_SC_PARALLEL_TRAFFIC: {
        const double sign = w.dbl(q) >= 0.5 ? 1 : -1;
        px = rwp(q + 2) * 0.4 + pxn;
        py = sign * (w.dbl(q + 4) * 3 + 1 + pyn);
        gx = px; gy = -py;
    } break;
    case CN_SC_PERPENDICULAR_TRAFFIC: {
        const double sign = w.dbl(q) >= 0.5 ? 1 : -1;
        px = sign * (w.dbl(q + 2) * 3 + 1 + pxn);
        gx = -px;
        py = rwp(q + 4) * 0.4 + pyn;
        gy = py;
    } break;
    case CN_SC_SIDE_PREF_PASSING:
    case CN_SC_SIDE_PREF_OVERTAKING: {
        const double min_x = -(robot_radius + agent_radius), max_x = -min_x;
        const double hx = (max_x - min_x) * w.dbl(q) + min_x;
        px = hx; gx = hx;
        if (scenario == CN_SC_SIDE_PREF_PASSING) { py = R; gy = -R; heading = -CN_PI / 2; }
        else { py = -R + 2; gy = R + 2; heading = CN_PI / 2; v_pref = 0.3; }
    } break;
    default: {
        const double min_x = -(R + robot_radius + agent_radius), max_x = -(R - robot_radius - agent_radius);
        const double hx = (max_x - min_x) * w.dbl(q) + min_x;
        px = hx; gx = -hx; py = 0; gy = 0;
    } break;
    }
    vp = v_pref;
}

struct Env1 {  // one env's agents in LDS (kernel B)
    double rpx, rpy, rgx, rgy, rr;
    double *hpx, *hpy, *hgx, *hgy, *hr, *hvp, *hth;  // [N]
};

// One agent test of the goal rejection loops (crowd_sim.py:744-760, 792-806): does goal candidate
// (gx, gy) of human `self` (radius r_self) come within r_self + r_agent + discomfort_dist of agent a's
// position or goal? a = 0 is the robot, a >= 1 the other humans in index order (self skipped).
__device__ __forceinline__ bool goal_hit(const cn_config &c, const Env1 &en, int self, double r_self, double gx,
                                         double gy, int a)
{
    double ax, ay, agx, agy, ar;
    if (a == 0) { ax = en.rpx; ay = en.rpy; agx = en.rgx; agy = en.rgy; ar = en.rr; }
    else {
        const int j = a - 1 < self ? a - 1 : a;
        ax = en.hpx[j]; ay = en.hpy[j]; agx = en.hgx[j]; agy = en.hgy[j]; ar = en.hr[j];
    }
    const double md = r_self + ar + c.discomfort_dist;
    return norm_lt(gx - ax, gy - ay, md) || norm_lt(gx - agx, gy - agy, md);
}

// Rejection loop of the reference (`while True: draw; if not collide: break`), speculative over the
// wave. Each try consumes W words, so try t's words start at p + W*t. The first pass spreads the tries
// AND the agent tests: lane = (try t, agent a), t = lane / NA, a = lane % NA, J = 64 / NA tries; later
// passes (crowded scenes, where early tries keep failing) put one try per lane, 64 per pass, each lane
// testing the agents in turn. `cand(q, t)` leaves try t's candidate in slot t of m.sl; `hit(t, a)` is
// one agent test (true = collision). The first try without a hit wins, as in the reference. Bounded by
// max_tries (the reference loops forever; after max_tries the last try is accepted and `ovf` counts
// it). Returns the winning slot; m.p is after its words.
template <typename FC, typename FT>
__device__ int wave_reject2(WRng &m, int W, int NA, int max_tries, uint32_t &ovf, FC cand, FT hit)
{
    const int lane = m.lane;
    const uint64_t gmask = NA >= 64 ? ~0ull : ((1ull << NA) - 1ull);
    int t0 = 0;
    {   // first pass, lane = (try, agent): the common case (an early try is accepted) in one short pass
        const int J = min(64 / NA, CN_MT_N / W);
        const int t = lane / NA, a = lane - t * NA;
        m.ensure(W * J);
        const int nt = min(J, max_tries);
        const bool valid = t < nt;
        if (valid && a == 0) cand(m.p + W * t, t);
        wsync();
        const uint64_t badm = __ballot(valid && hit(t, a));
        for (int k = 0; k < nt; ++k)
            if (((badm >> (k * NA)) & gmask) == 0) { m.p += W * (k + 1); return k; }
        if (J >= max_tries) { m.p += W * nt; ++ovf; return nt - 1; }
        m.p += W * J;
        t0 = J;
        wsync();
    }
    // crowded: lane = try (64 per pass), each lane tests the agents in turn
    const int J = min(64, CN_MT_N / W);
    for (;; t0 += J) {
        m.ensure(W * J);
        const int nt = min(J, max_tries - t0);
        const bool valid = lane < nt;
        if (valid) cand(m.p + W * lane, lane);
        wsync();
        bool bad = !valid;
        for (int a = 0; a < NA && !bad; ++a) bad = hit(lane, a);
        const uint64_t okm = __ballot(!bad);
        if (okm) {
            const int first = __ffsll((long long)okm) - 1;
            m.p += W * (first + 1);
            return first;
        }
        if (t0 + J >= max_tries) { m.p += W * nt; ++ovf; return nt - 1; }
        m.p += W * J;
        wsync();   // slots are rewritten by the next pass
    }
}

// Binned disc test for the crowded passes of the spawn's rejection loops (wave_reject_discs): a try is
// rejected iff its point lies strictly inside one of the agents' discs; the discs except agent 0's (the
// robot, often far from the crowd, tested exactly) are binned once per call into a 16 x 16 grid over their
// bounding box (4 cells per lane, float32 with a 1e-4 m margin, so the binning is conservative): a cell
// lying inside some disc rejects every try that lands in it, a try outside the box hits nothing, and
// otherwise only the agents overlapping its cell are tested exactly (norm_lt). Same result as testing
// every agent. The crowded goal rejection (goal_reject_crowded<GRID>) uses it on the kd-tree path only
// (the quad path's scenes are sparse and its code stays smaller).
struct DiscGrid {
    uint32_t *mask;   // [256] per cell: bit a = agent a's position or goal disc overlaps the cell (NA <= 32)
    uint64_t *cov;    // [4] bit = cell entirely inside some disc
    double *par;      // x0, y0, 16 / width, 16 / height
};

template <bool GOALS = true>
__device__ __forceinline__ void disc_grid_build(const DiscGrid &gr, const double *tx, const double *ty, const double *tgx,
                                                const double *tgy, const double *tmd, int NA, int lane)
{
    // bounding box of every disc (wave-uniform: each lane scans the table)
    // agent 0 (the robot, often far from the crowd) stays out of the grid: disc_grid_hit tests it exactly
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    for (int a = 1; a < NA; ++a) {
        const double d = tmd[a] + 1e-3;
        const double ax = tx[a], ay = ty[a], bx = GOALS ? tgx[a] : ax, by = GOALS ? tgy[a] : ay;
        x0 = fmin(x0, fmin(ax, bx) - d); x1 = fmax(x1, fmax(ax, bx) + d);
        y0 = fmin(y0, fmin(ay, by) - d); y1 = fmax(y1, fmax(ay, by) + d);
    }
    const double ivx = CN_GRID / (x1 - x0), ivy = CN_GRID / (y1 - y0);
    // cells lane + 64 j (j < 4): column lane & 15, row 4 j + lane / 16; each expanded by 1e-4 m (a try is
    // binned in double precision; near a cell edge it may land in the neighbour, which the expansion covers)
    const float m = 1e-4f;
    const int ix = lane & 15;
    const float cx0 = (float)(x0 + ix / ivx) - m, cx1 = (float)(x0 + (ix + 1) / ivx) + m;
    float cy0[4], cy1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int iy = 4 * j + (lane >> 4);
        cy0[j] = (float)(y0 + iy / ivy) - m; cy1[j] = (float)(y0 + (iy + 1) / ivy) + m;
    }
    uint32_t msk[4] = {0u, 0u, 0u, 0u};
    bool covered[4] = {false, false, false, false};
    for (int a = 1; a < NA; ++a) {
        const float d = (float)tmd[a], dl = d + m, ds = d - m;
#pragma unroll
        for (int g = 0; g < (GOALS ? 2 : 1); ++g) {
            const float px = (float)(g ? tgx[a] : tx[a]), py = (float)(g ? tgy[a] : ty[a]);
            const float nx = fmaxf(0.0f, fmaxf(cx0 - px, px - cx1));
            const float fx = fmaxf(fabsf(px - cx0), fabsf(px - cx1));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float ny = fmaxf(0.0f, fmaxf(cy0[j] - py, py - cy1[j]));
                const float fy = fmaxf(fabsf(py - cy0[j]), fabsf(py - cy1[j]));
                if (nx * nx + ny * ny <= dl * dl) msk[j] |= 1u << a;
                if (ds > 0.0f && fx * fx + fy * fy < ds * ds) covered[j] = true;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        gr.mask[lane + 64 * j] = msk[j];
        const uint64_t cv = __ballot(covered[j]);
        if (lane == 0) gr.cov[j] = cv;
    }
    if (lane == 0) { gr.par[0] = x0; gr.par[1] = y0; gr.par[2] = ivx; gr.par[3] = ivy; }
}

// does the goal (gx, gy) lie strictly inside one of the discs? Exact tests (norm_lt) of the agents
// binned in its cell, two agents (four discs) per round with their loads issued together
template <bool GOALS = true>
__device__ __forceinline__ bool disc_grid_hit(const DiscGrid &gr, const double *tx, const double *ty, const double *tgx,
                                              const double *tgy, const double *tmd, double gx, double gy)
{
    if (norm_lt(gx - tx[0], gy - ty[0], tmd[0]) || (GOALS && norm_lt(gx - tgx[0], gy - tgy[0], tmd[0]))) return true;
    const double fx = (gx - gr.par[0]) * gr.par[2], fy = (gy - gr.par[1]) * gr.par[3];
    if (!(fx >= 0.0 && fx < CN_GRID && fy >= 0.0 && fy < CN_GRID)) return false;   // outside every other disc
    const int cell = (int)fy * CN_GRID + (int)fx;
    if ((gr.cov[cell >> 6] >> (cell & 63)) & 1ull) return true;
    uint32_t msk = gr.mask[cell];
    bool hit = false;
    while (msk && !hit) {
        const int a0 = __ffs(msk) - 1;
        msk &= msk - 1;
        const int a1 = msk ? __ffs(msk) - 1 : a0;
        msk &= msk - 1;
        const double x0 = tx[a0], y0 = ty[a0], d0 = tmd[a0];
        const double x1 = tx[a1], y1 = ty[a1], d1 = tmd[a1];
        hit = norm_lt(gx - x0, gy - y0, d0) | norm_lt(gx - x1, gy - y1, d1);
        if (GOALS) {
            const double u0 = tgx[a0], v0 = tgy[a0], u1 = tgx[a1], v1 = tgy[a1];
            hit = hit | norm_lt(gx - u0, gy - v0, d0) | norm_lt(gx - u1, gy - v1, d1);
        }
    }
    return hit;
}

// Cover of a crowded rejection loop's candidate box (kd-tree path: square_crossing end goals and random goals
// on the circle in goal_reject_crowded, square_crossing spawn positions in wave_reject_discs): the box
// [-hb, hb]^2 that holds every candidate (0.4 * rand_world_pt + noise, crowd_sim.py:313-318; R cos / sin +
// noise, :736-741) in CN_GC x CN_GC
// cells. Per row of cells, `cov` has bit i set where cell i lies inside ONE of the agents' position / goal
// discs (so every try landing there is rejected); `arow` / `acol` are the agents whose discs' bounding boxes
// overlap the row / column strip, so a try in an uncovered cell tests only the agents of arow & acol
// exactly. Built per loop in one short pass (lane = row strip x half of the agents), unlike DiscGrid over the
// discs' bounding box, whose ~0.45 m cells left ~30 % of the tries to the exact test (~2 % here).
#define CN_GC 32
struct GoalCover {
    uint32_t *cov, *arow, *acol;   // [CN_GC] each
    double *par;                   // x0 (= y0), CN_GC / (2 hb)
};

// Built in float32 with a 1e-4 m margin on both the cells (expanded) and the discs (shrunk for coverage,
// grown for overlap), so no rounding of the build can mark a cell that the exact test (norm_lt, f64) would
// not reject everywhere: a try is binned in float64 (at most ~1e-14 m off its cell), float32 coordinates
// are ~1e-6 m off, and a cell can only be covered where the chord half-width w > s / 2 = 0.08 m, where
// sqrtf is well conditioned.
template <bool GOALS = true>
__device__ __forceinline__ void goal_cover_build(const GoalCover &gc, const double *tx, const double *ty,
                                                 const double *tgx, const double *tgy, const double *tmd, int NA,
                                                 double hb, int lane)
{
    const double sd = 2 * hb / CN_GC;
    const int r = lane & (CN_GC - 1), half = lane >> 5;
    const float m = 1e-4f, x0 = (float)-hb, inv = (float)(CN_GC / (2 * hb));
    const float s0 = (float)(-hb + r * sd) - m, s1 = (float)(-hb + (r + 1) * sd) + m;   // strip r, expanded
    uint32_t cov = 0u, arow = 0u, acol = 0u;
    for (int a = half; a < NA; a += 2) {
        const float d = (float)tmd[a], dl = d + m, ds = d - m;
#pragma unroll
        for (int g = 0; g < (GOALS ? 2 : 1); ++g) {
            const float cx = (float)(g ? tgx[a] : tx[a]), cy = (float)(g ? tgy[a] : ty[a]);
            if (cy + dl >= s0 && cy - dl <= s1) arow |= 1u << a;
            if (cx + dl >= s0 && cx - dl <= s1) acol |= 1u << a;
            const float dy = fmaxf(fabsf(s0 - cy), fabsf(s1 - cy));   // farthest point of the strip in y
            if (ds > dy) {
                const float w = sqrtf(ds * ds - dy * dy);
                // cells i with [x0 + i s - m, x0 + (i + 1) s + m] inside (cx - w, cx + w)
                const int lo = max((int)floorf((cx - w - x0 + m) * inv) + 1, 0);
                const int hi = min((int)floorf((cx + w - x0 - m) * inv) - 1, CN_GC - 1);
                if (lo <= hi) cov |= (hi - lo == 31 ? ~0u : ((1u << (hi - lo + 1)) - 1u)) << lo;
            }
        }
    }
    cov |= __shfl_xor(cov, 32); arow |= __shfl_xor(arow, 32); acol |= __shfl_xor(acol, 32);
    if (lane < CN_GC) { gc.cov[lane] = cov; gc.arow[lane] = arow; gc.acol[lane] = acol; }
    if (lane == 0) { gc.par[0] = -hb; gc.par[1] = CN_GC / (2 * hb); }
}

// does the goal (gx, gy) lie strictly inside one of the agents' discs? Same answer as goal_hit over every
// agent (GOALS = false: the position discs only, the spawn's placement test)
template <bool GOALS = true>
__device__ __forceinline__ bool goal_cover_hit(const GoalCover &gc, const double *tx, const double *ty,
                                               const double *tgx, const double *tgy, const double *tmd, int NA,
                                               double gx, double gy)
{
    const double fx = (gx - gc.par[0]) * gc.par[1], fy = (gy - gc.par[0]) * gc.par[1];
    uint32_t msk;
    if (fx >= 0.0 && fx < CN_GC && fy >= 0.0 && fy < CN_GC) {
        const int ix = (int)fx, iy = (int)fy;
        if ((gc.cov[iy] >> ix) & 1u) return true;
        msk = gc.arow[iy] & gc.acol[ix];
    } else msk = NA >= 32 ? ~0u : (1u << NA) - 1u;   // outside the box (not reached by its candidates)
    bool hit = false;
    while (msk && !hit) {
        const int a0 = __ffs(msk) - 1;
        msk &= msk - 1;
        const int a1 = msk ? __ffs(msk) - 1 : a0;
        msk &= msk - 1;
        const double x0 = tx[a0], y0 = ty[a0], d0 = tmd[a0];
        const double x1 = tx[a1], y1 = ty[a1], d1 = tmd[a1];
        hit = norm_lt(gx - x0, gy - y0, d0) | norm_lt(gx - x1, gy - y1, d1);
        if (GOALS) {
            const double u0 = tgx[a0], v0 = tgy[a0], u1 = tgx[a1], v1 = tgy[a1];
            hit = hit | norm_lt(gx - u0, gy - v0, d0) | norm_lt(gx - u1, gy - v1, d1);
        }
    }
    return hit;
}

// wave_reject2 for "the candidate point (m.sl[t], m.sl[64 + t]) lies strictly inside one of NA discs"
// (`disc(a, x, y, md)`: centre and radius of agent a): the spawn's human placement (crowd_sim.py:369-390).
// When the wave has grid space (m.grid) the crowded passes bin the discs once into a DiscGrid (see
// goal_reject_crowded) and test each try against its cell's agents only; same result.
template <bool GRID, typename FC, typename FD>
__device__ int wave_reject_discs(WRng &m, int W, int NA, int max_tries, uint32_t &ovf, FC cand, FD disc, double hb = 0.0)
{
    auto hit = [&](int t, int a) {
        double x, y, md;
        disc(a, x, y, md);
        return norm_lt(m.sl[t] - x, m.sl[64 + t] - y, md);
    };
    if (!GRID || !m.grid || NA < 8) return wave_reject2(m, W, NA, max_tries, ovf, cand, hit);
    const int lane = m.lane;
    const uint64_t gmask = NA >= 64 ? ~0ull : ((1ull << NA) - 1ull);
    int t0 = 0;
    {   // first pass, lane = (try, agent), as wave_reject2
        const int J = min(64 / NA, CN_MT_N / W);
        const int t = lane / NA, a = lane - t * NA;
        m.ensure(W * J);
        const int nt = min(J, max_tries);
        const bool valid = t < nt;
        if (valid && a == 0) cand(m.p + W * t, t);
        wsync();
        const uint64_t badm = __ballot(valid && hit(t, a));
        for (int k = 0; k < nt; ++k)
            if (((badm >> (k * NA)) & gmask) == 0) { m.p += W * (k + 1); return k; }
        if (J >= max_tries) { m.p += W * nt; ++ovf; return nt - 1; }
        m.p += W * J;
        t0 = J;
    }
    double *tx = (double *)m.grid, *ty = tx + 32, *tmd = tx + 64;
    DiscGrid gr;
    GoalCover gc;
    const bool cover = hb > 0.0 && NA <= 32;   // a candidate box: cover it (see GoalCover) instead of the discs' box
    gr.mask = (uint32_t *)(tx + 96); gr.cov = (uint64_t *)(tx + 96 + CN_GRID * CN_GRID / 2); gr.par = (double *)(gr.cov + 4);
    gc.cov = (uint32_t *)(tx + 96); gc.arow = gc.cov + CN_GC; gc.acol = gc.arow + CN_GC; gc.par = (double *)(gc.acol + CN_GC);
    if (lane < NA) { double x, y, md; disc(lane, x, y, md); tx[lane] = x; ty[lane] = y; tmd[lane] = md; }
    wsync();
    if (cover) goal_cover_build<false>(gc, tx, ty, tx, ty, tmd, NA, hb, lane);
    else disc_grid_build<false>(gr, tx, ty, tx, ty, tmd, NA, lane);
    const int J = min(64, CN_MT_N / W);
    for (;; t0 += J) {
        m.template ensure<true>(W * J);
        const int nt = min(J, max_tries - t0);
        const bool valid = lane < nt;
        if (valid) cand(m.p + W * lane, lane);
        wsync();
        const bool bad = !valid || (cover ? goal_cover_hit<false>(gc, tx, ty, tx, ty, tmd, NA, m.sl[lane], m.sl[64 + lane])
                                          : disc_grid_hit<false>(gr, tx, ty, tx, ty, tmd, m.sl[lane], m.sl[64 + lane]));
        const uint64_t okm = __ballot(!bad);
        if (okm) {
            const int first = __ffsll((long long)okm) - 1;
            m.p += W * (first + 1);
            return first;
        }
        if (t0 + J >= max_tries) { m.p += W * nt; ++ovf; return nt - 1; }
        m.p += W * J;
        wsync();   // slots are rewritten by the next pass
    }
}

// Crowded goal rejection (a goal pass whose first batch was all rejected; in square_crossing at N = 25
// most of these loops run to max_tries): one try per lane, 64 at a time, straight from the stream; the
// agents (robot, then the other humans in index order) sit in an LDS table with their minimum distance
// precomputed, and each lane tests them four at a time with the loads of a group issued together (the
// agent-at-a-time loop was bound by dependent LDS latency). Same result as goal_hit over the tries in
// order; returns the winning slot (m.sl[t], m.sl[64 + t]), m.p after its words.
// GRID (the kd-tree path, whose waves have DiscGrid space in m.grid): the position and goal discs of the
// agents are binned once per loop (disc_grid_build<true>) and each try tests only its cell's agents --
// at 25 humans in square_crossing most of these loops run all max_tries = 1000 tries (16 passes), so the
// one-off binning is repaid many times over; same result. With a candidate box (hb > 0: square_crossing's
// end goals) a GoalCover over the box replaces the DiscGrid.
template <bool GRID, typename FC>
__device__ int goal_reject_crowded(const cn_config &c, const Env1 &en, WRng &m, int self, double r_self, int W,
                                   int max_tries, uint32_t &ovf, FC cand, double hb = 0.0)
{
    const int lane = m.lane, NA = c.human_num;
    double *tx = m.sl + 128, *ty = tx + 32, *tgx = tx + 64, *tgy = tx + 96, *tmd = tx + 128;   // [32] each
    if (lane < NA) {
        double ar;
        if (lane == 0) { tx[0] = en.rpx; ty[0] = en.rpy; tgx[0] = en.rgx; tgy[0] = en.rgy; ar = en.rr; }
        else {
            const int j = lane - 1 < self ? lane - 1 : lane;
            tx[lane] = en.hpx[j]; ty[lane] = en.hpy[j]; tgx[lane] = en.hgx[j]; tgy[lane] = en.hgy[j]; ar = en.hr[j];
        }
        tmd[lane] = r_self + ar + c.discomfort_dist;
    }
    wsync();
    DiscGrid gr;
    GoalCover gc;
    const bool cover = GRID && m.grid && NA >= 8 && NA <= 32 && hb > 0.0;
    const bool grid = GRID && m.grid && NA >= 8 && !cover;
    if (cover) {
        gc.cov = (uint32_t *)(m.grid + 96 * 8);
        gc.arow = gc.cov + CN_GC; gc.acol = gc.arow + CN_GC;
        gc.par = (double *)(gc.acol + CN_GC);
        goal_cover_build<true>(gc, tx, ty, tgx, tgy, tmd, NA, hb, lane);
        wsync();
    }
    if (grid) {
        gr.mask = (uint32_t *)(m.grid + 96 * 8);
        gr.cov = (uint64_t *)(m.grid + 96 * 8 + CN_GRID * CN_GRID * 4);
        gr.par = (double *)(gr.cov + 4);
        disc_grid_build<true>(gr, tx, ty, tgx, tgy, tmd, NA, lane);
        wsync();
    }
    const int J = min(64, CN_MT_N / W);
#ifdef CN_STAMPS
    unsigned long long tq = clock64(), tc_e = 0, tc_c = 0, tc_t = 0, tc_n = 0;
#endif
    for (int t0 = 0;; t0 += J) {
        m.template ensure<true>(W * J);
#ifdef CN_STAMPS
        { const unsigned long long t_ = clock64(); tc_e += t_ - tq; tq = t_; ++tc_n; }
#endif
        const int nt = min(J, max_tries - t0);
        double gx = 0, gy = 0;
        if (lane < nt) {
            cand(m.p + W * lane, lane);
            gx = m.sl[lane]; gy = m.sl[64 + lane];
        }
        wsync();
#ifdef CN_STAMPS
        { const unsigned long long t_ = clock64(); tc_c += t_ - tq; tq = t_; }
#endif
        bool bad = lane >= nt;
        if (cover) bad = bad || goal_cover_hit<true>(gc, tx, ty, tgx, tgy, tmd, NA, gx, gy);
        else if (grid) bad = bad || disc_grid_hit<true>(gr, tx, ty, tgx, tgy, tmd, gx, gy);
        else
        for (int a0 = 0; a0 < NA && !bad; a0 += 4) {
            double x[4], y[4], u[4], v[4], d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = min(a0 + k, NA - 1);   // a repeated last agent does not change the outcome
                x[k] = tx[a]; y[k] = ty[a]; u[k] = tgx[a]; v[k] = tgy[a]; d[k] = tmd[a];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                bad = bad | norm_lt(gx - x[k], gy - y[k], d[k]) | norm_lt(gx - u[k], gy - v[k], d[k]);
        }
#ifdef CN_STAMPS
        { const uint64_t bb_ = __ballot(bad); (void)bb_; const unsigned long long t_ = clock64(); tc_t += t_ - tq; tq = t_;
          if (lane == 0 && m.edbg >= 0 && m.edbg < 8192) { cn_stamp_c[m.edbg * 4] += tc_e; cn_stamp_c[m.edbg * 4 + 1] += tc_c; cn_stamp_c[m.edbg * 4 + 2] += tc_t; cn_stamp_c[m.edbg * 4 + 3] += 1; }
          tc_e = tc_c = tc_t = 0; }
#endif
        const uint64_t okm = __ballot(!bad);
        if (okm) {
            const int first = __ffsll((long long)okm) - 1;
            m.p += W * (first + 1);
            return first;
        }
        if (t0 + nt >= max_tries) { m.p += W * nt; ++ovf; return nt - 1; }
        m.p += W * J;
        wsync();   // slots are rewritten by the next batch
    }
}

// The random part of CrowdSimDict.reset (crowd_sim_dict.py:110-156; generate_robot_humans,
// crowd_sim.py:555-663; generate_circle_crossing_human :359-393): reseed the env's stream with
// counter_offset + case_counter + thisSeed, draw the robot and then each human with rejection.
// One wave; the result is left in `en` (LDS), rth, ovf, sc and the stream `m`.
// Resumable (spare-workgroup spawns): i0 > 0 continues a spawn parked after its first i0 humans -- the
// caller restored the stream, the robot, rth, ovf, sc and those humans -- and with a `deadline` (clock64
// value, 0 = none) the spawn parks itself before a human once the deadline has passed (at least one
// human per call). Returns the number of humans placed (N = complete).
template <bool GRID>
__device__ __forceinline__ int spawn_env(const cn_config &c, int64_t gidx, int64_t case_counter, int32_t reset_count,
                          int64_t counter_offset, WRng &m, Env1 &en, double &rth, uint32_t &ovf, int &sc,
                          int i0 = 0, long long deadline = 0)
{
    const int lane = m.lane;
    const int N = c.human_num;
    const double R = c.circle_radius;
    const int W0 = i0;
    STAMP_S(gidx, 0);
    if (i0 == 0) {
    uint32_t *mtw = m.w;
    m.off = 0;   // a fresh stream: the key at the start of the ring
    if (c.scenario_mode == CN_SCMODE_SEQUENTIAL) sc = c.scenarios[reset_count % c.num_scenarios];
    else sc = c.scenarios[gidx % c.num_scenarios];
    const uint32_t seed0 = (uint32_t)(counter_offset + case_counter + (c.seed + gidx));
    if (m.phx) {
        if (lane == 0) mtw[0] = seed0;   // the key is the whole stream state (written back with the reset)
        m.key = seed0;
        m.p = 0;
    } else {
        // mt19937_seed: the sequential Knuth chain, wave-uniform so it runs on the scalar unit (s_mul_i32 /
        // s_xor / s_lshr: a few cycles per word instead of a quarter-rate v_mul_lo_u32 chain on one lane);
        // word j*64 + k is dropped into lane k of a VGPR (v_writelane) and each lane stores its word
        uint32_t seed = __builtin_amdgcn_readfirstlane(seed0);
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) {
            int mine = 0;
#pragma unroll
            for (int k = 0; k < 64; ++k) {
                asm("v_writelane_b32 %0, %1, %2" : "+v"(mine) : "s"(seed), "n"(k));
                seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(j * 64 + k + 1);
            }
            if (j * 64 + lane < CN_MT_N) mtw[j * 64 + lane] = (uint32_t)mine;
        }
        m.p = CN_MT_N;   // numpy: pos = 624 after seeding, the first draw runs mt19937_gen
    }
    wsync();
    STAMP_S(gidx, 1);
    m.have1 = false; m.slid = false;
    ovf = 0;
    en.rr = c.robot_radius;
    if (c.kinematics == CN_UNICYCLE) {
        const double angle = m.unif(0, CN_PI * 2);
        en.rpx = R * cos(angle); en.rpy = R * sin(angle);
        // goal: uniform in the square until >= 6 m away (crowd_sim.py:620-634)
        const int tw = wave_reject2(m, 4, 1, c.max_tries, ovf, [&](int q, int t) {
            m.sl[t] = -R + (R - -R) * m.dbl(q); m.sl[64 + t] = -R + (R - -R) * m.dbl(q + 2);
        }, [&](int t, int) { return norm_lt(en.rpx - m.sl[t], en.rpy - m.sl[64 + t], 6.0); });
        en.rgx = m.sl[tw]; en.rgy = m.sl[64 + tw];
        wsync();
        rth = m.unif(0, 2 * CN_PI);
    } else if (c.social_metrics || c.side_preference) {
        en.rpx = 0; en.rpy = -R; en.rgx = 0; en.rgy = R; rth = CN_PI / 2;
    } else {
        // holonomic robot: start and goal uniform in the square until >= 6 m apart (crowd_sim.py:652-660)
        const int tw = wave_reject2(m, 8, 1, c.max_tries, ovf, [&](int q, int t) {
            m.sl[t] = -R + (R - -R) * m.dbl(q); m.sl[64 + t] = -R + (R - -R) * m.dbl(q + 2);
            m.sl[128 + t] = -R + (R - -R) * m.dbl(q + 4); m.sl[192 + t] = -R + (R - -R) * m.dbl(q + 6);
        }, [&](int t, int) { return norm_lt(m.sl[t] - m.sl[128 + t], m.sl[64 + t] - m.sl[192 + t], 6.0); });
        en.rpx = m.sl[tw]; en.rpy = m.sl[64 + tw]; en.rgx = m.sl[128 + tw]; en.rgy = m.sl[192 + tw];
        wsync();
        rth = CN_PI / 2;
    }
    }   // i0 == 0
    STAMP_S(gidx, 2);
    const int W = cand_words(sc);
    for (int i = i0; i < N; ++i) {
        if (deadline && i > W0 && (long long)clock64() > deadline) return i;   // park (wave-uniform clock)
        double vpref = c.human_vpref, rad = c.human_radius;
        if (c.randomize_attributes) { vpref = m.unif(0.5, 1.5); rad = m.unif(0.3, 0.5); }
        // candidate vs the robot and the humans placed so far (crowd_sim.py:369-390): i + 1 agent tests
        const int tw = wave_reject_discs<GRID>(m, W, i + 1, c.max_tries, ovf, [&](int q, int t) {
            double px, py, gx, gy, hd, vp;
            cand_attributes(c, m, q, sc, vpref, rad, en.rr, px, py, gx, gy, hd, vp);
            m.sl[t] = px; m.sl[64 + t] = py; m.sl[128 + t] = gx; m.sl[192 + t] = gy; m.sl[256 + t] = hd;
            m.sl[320 + t] = vp;
        }, [&](int a, double &ax, double &ay, double &md) {
            if (a == 0) {
                ax = en.rpx; ay = en.rpy;
                md = c.kinematics == CN_UNICYCLE ? R / 2 : rad + en.rr + c.discomfort_dist;
            } else {
                ax = en.hpx[a - 1]; ay = en.hpy[a - 1];
                md = rad + en.hr[a - 1] + c.discomfort_dist;
            }
        }, sc == CN_SC_SQUARE_CROSSING ? 0.1 * c.square_width + 0.5 * fabs(vpref == 0 ? 1.0 : vpref) + 1e-3 : 0.0);
        if (lane == 0) {
            en.hpx[i] = m.sl[tw]; en.hpy[i] = m.sl[64 + tw]; en.hgx[i] = m.sl[128 + tw]; en.hgy[i] = m.sl[192 + tw];
            en.hth[i] = m.sl[256 + tw]; en.hvp[i] = m.sl[320 + tw]; en.hr[i] = rad;
        }
        wsync();
        if (i < 13) STAMP_S(gidx, 3 + i);
    }
    return N;
}

// Store a drawn spawn as env e's pending episode for the reset with key (cc, rc), slot rc & 1.
// okv: the completing launch's id, or 0 with `prog` = humans placed for a spawn parked mid-way (the
// stream at the park point, the robot and the first prog humans are stored; resumed by a later launch).
// FENCE: the round-5 handshake (CN_SLOT_FENCE); the ok word, written last, carries the entry's key and the
// completing launch's id, which is all a reset of a later launch needs (reset_env)
template <bool FENCE>
__device__ __forceinline__ void write_pending(const PendPtrs &P2, const cn_config &c, int64_t E, int64_t e, const Env1 &en, double rth,
                              int sc, uint32_t ovf, const uint32_t *mt_src, int pos, int64_t cc, int32_t rc, int lane,
                              uint32_t okv, int prog)
{
    const int N = c.human_num;
    const PendPtrs P = pend_slot(P2, rc & 1, E, E * N);
    const int nk = c.rng_mode == CN_RNG_PHILOX ? 1 : CN_MT_N;   // key words to copy
    // Invalidate the slot before rewriting it, visible device-wide before any new payload or key store:
    // a reset of the same launch that reads the slot (reset_env: key, fence, then ok) and sees a new key
    // then sees ok == 0 (or this launch's id) and draws inline instead of reading a half-written payload.
    if (FENCE) {
        if (lane == 0) P.ok[e] = 0ull;
        __threadfence();
    }
    {
        uint32_t v[(CN_MT_N + 63) / 64];
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; v[j] = k < nk ? mt_src[k] : 0u; }
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; if (k < nk) P.mt[e * CN_MT_N + k] = v[j]; }
    }
    if (lane < prog) {
        const int64_t h = e * N + lane, EN = E * N;
        P.h[h] = en.hpx[lane]; P.h[EN + h] = en.hpy[lane]; P.h[2 * EN + h] = en.hgx[lane];
        P.h[3 * EN + h] = en.hgy[lane]; P.h[4 * EN + h] = en.hr[lane]; P.h[5 * EN + h] = en.hvp[lane];
        P.h[6 * EN + h] = en.hth[lane];
    }
    if (lane == 0) {
        P.r[e] = en.rpx; P.r[E + e] = en.rpy; P.r[2 * E + e] = en.rgx; P.r[3 * E + e] = en.rgy; P.r[4 * E + e] = rth;
        P.pos[e] = pos; P.ovf[e] = ovf; P.sc[e] = sc; P.cc[e] = cc; P.rc[e] = rc;
        P.prog[e] = okv ? 0 : prog;
    }
    if (FENCE) __threadfence();   // the whole entry before its ok word (release)
    if (lane == 0) P.ok[e] = ((uint64_t)(uint32_t)rc << 32) | okv;
}

// The deterministic rest of CrowdSimDict.reset (crowd_sim_dict.py:136-203): state of the new episode,
// case_counter advance, first observation. `mt_src` = key words after the spawn (LDS or pending buffer).
__device__ __forceinline__ void write_reset(const ResetOut &g, const cn_config &c, int64_t e, const Env1 &en, double rth, int sc,
                            uint32_t ovf, const uint32_t *mt_src, int pos, int lane)
{
    const cn_state_ptrs &S = g.s;
    const int N = c.human_num;
    const int64_t hb = e * N;
    const double rpx = en.rpx, rpy = en.rpy;
    const int64_t orw = orow(g.ov, e);
    if (lane >= N && lane < g.ov.NS) {
        g.spatial[(orw * g.ov.NS + lane) * 2] = (float)(CN_PAD_POS - rpx);
        g.spatial[(orw * g.ov.NS + lane) * 2 + 1] = (float)(CN_PAD_POS - rpy);
    }
    if (lane < N) {
        const int64_t h = hb + lane;
        const double px = en.hpx[lane], py = en.hpy[lane];
        S.h_px[h] = px; S.h_py[h] = py; S.h_gx[h] = en.hgx[lane]; S.h_gy[h] = en.hgy[lane];
        S.h_vx[h] = 0.0; S.h_vy[h] = 0.0; S.h_r[h] = en.hr[lane]; S.h_vpref[h] = en.hvp[lane];
        S.h_theta[h] = en.hth[lane];
        S.o_r[h] = 0.0f; S.o_vmax[h] = 0.0f; S.o_dmask[h] = 0u;
        // generate_ob(reset=True): robot velocity is 0 (ints) -> float64 FOV path
        const double th0 = c.kinematics == CN_HOLONOMIC ? 0.0 : rth;   // atan2(0, 0) = 0
        int v = c.robot_fov >= 2.0 * CN_PI ? vis360(isfinite(th0), rpx, rpy, px, py) : -1;
        if (v < 0) v = reset_fov_test(th0, rpx, rpy, px, py, c.robot_fov);
        double bpx, bpy, bvx, bvy, br;
        if (v) { bpx = px; bpy = py; bvx = 0; bvy = 0; br = en.hr[lane]; }
        else { bpx = 15.0; bpy = 15.0; bvx = 0.0; bvy = 0.0; br = 0.3; }
        S.b_px[h] = bpx; S.b_py[h] = bpy; S.b_vx[h] = bvx; S.b_vy[h] = bvy; S.b_r[h] = br;
        g.spatial[(orw * g.ov.NS + lane) * 2] = (float)(bpx - rpx);
        g.spatial[(orw * g.ov.NS + lane) * 2 + 1] = (float)(bpy - rpy);
    }
    const int A = N + (c.robot_visible ? 1 : 0);
    if (A > 10) for (int k = lane; k < N * A; k += 64) S.o_perm[e * N * A + k] = 0;
    const int nk = c.rng_mode == CN_RNG_PHILOX ? 1 : CN_MT_N;   // key words to copy
    {   // all loads first, then all stores: mt_src may be LDS or global, so the compiler cannot pipeline
        uint32_t v[(CN_MT_N + 63) / 64];
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; v[j] = k < nk ? mt_src[k] : 0u; }
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; if (k < nk) S.mt[e * CN_MT_N + k] = v[j]; }
    }
    if (lane == 0) {
        S.scenario[e] = (int32_t)sc;
        S.gtime[e] = 0.0; S.r_dv[e] = 0.0;
        S.r_px[e] = rpx; S.r_py[e] = rpy; S.r_gx[e] = en.rgx; S.r_gy[e] = en.rgy; S.r_theta[e] = rth;
        S.r_vx[e] = 0.0; S.r_vy[e] = 0.0; S.r_radius[e] = c.robot_radius; S.r_vpref[e] = c.robot_vpref;
        S.case_counter[e] = (S.case_counter[e] + c.nenv) % g.case_size;
        S.potential[e] = -fabs(np_norm2(rpx - en.rgx, rpy - en.rgy));
        S.reset_count[e] += 1;
        S.ep_return[e] = 0.0; S.ep_len[e] = 0;
        S.flags[e] = 0; S.overflow[e] = ovf; S.mt_pos[e] = pos;
        float *rn = g.robot_node + orw * 7;
        rn[0] = (float)rpx; rn[1] = (float)rpy; rn[2] = (float)c.robot_radius;
        rn[3] = (float)en.rgx; rn[4] = (float)en.rgy; rn[5] = (float)c.robot_vpref; rn[6] = (float)rth;
        g.temporal[orw * 2] = 0.0f; g.temporal[orw * 2 + 1] = 0.0f;
    }
}


// Word page of a goal pass: the doubles of the next 128 stream words (64 draws) and, where the pass
// needs angles, cos / sin of 2*pi*draw, computed by the 64 lanes at once (one draw + one f64 sincos per
// lane) so that the sequential walk over the humans only reads tables. Index k holds the draw at word
// pb + 2k. Wave-uniform reads are LDS broadcasts (v_readlane broadcasts of loop-carried values
// miscompiled in this loop nest: wrong winners and NaN goals on the GPU, tools/diag_goal.py).
struct GPage {
    double *d, *cs, *sn;   // LDS [64] each (the wave's try-slot area m.sl, unused by the goal passes)
    int pb;
    __device__ double dbl(int q) const { return d[(q - pb) >> 1]; }
    __device__ double cos2pi(int q) const { return cs[(q - pb) >> 1]; }
    __device__ double sin2pi(int q) const { return sn[(q - pb) >> 1]; }
};

// (re)build the page at the stream position m.p (all lanes)
__device__ __forceinline__ void gpage_build(WRng &m, GPage &pg, bool trig)
{
    wsync();   // earlier reads of the old page are done before it is overwritten
    m.ensure(128);
    pg.pb = m.p;
    const double d = m.dbl(m.p + 2 * m.lane);
    pg.d[m.lane] = d;
    if (trig) {
        const double a = d * CN_PI * 2;
        pg.cs[m.lane] = cos(a);
        pg.sn[m.lane] = sin(a);
    }
    wsync();
}

// One of the two goal-change loops at the end of CrowdSimDict.step:
//   KIND 0  update_human_goals_randomly (crowd_sim.py:724-766): humans with v_pref != 0 draw U; if
//           U <= goal_change_chance a new goal on the circle is rejection-sampled (angle, gx_noise, gy_noise);
//   KIND 1  update_human_goal (crowd_sim.py:769-811): humans within their radius of the goal draw U; if
//           U <= end_goal_change_chance radius / v_pref are jittered and create_agent_attributes'
//           candidate is rejection-sampled.
// Both walk the humans in index order, as the reference does, over a page of precomputed draws (GPage):
// the walk itself is wave-uniform table reads; a changing human tests J tries at once, lane = (try t,
// agent a), against the robot and the other humans (earlier humans already carry their new goals); the
// first try without a hit wins. Bounded by max_tries like every rejection loop.
template <int KIND, bool GRID>
__device__ __forceinline__ int goal_pass(const cn_config &c, Env1 &en, WRng &m, uint32_t &ovf, int sc, double *sp,
                                         int64_t edbg = -1)
{
#ifdef CN_STAMPS
    unsigned long long tq = clock64(), t_walk = 0, t_first = 0, t_rej = 0;
#define GP_LAP(acc) do { const unsigned long long t_ = clock64(); acc += t_ - tq; tq = t_; } while (0)
#else
#define GP_LAP(acc) do { } while (0)
#endif
    (void)sp;
    int dbg = 0;   // diagnostics: 1000 * batches + eligible humans + 100 * changes
    const int N = c.human_num, lane = m.lane;
    const double chance = KIND == 0 ? c.goal_change_chance : c.end_goal_change_chance;
    const int W = KIND == 0 ? 6 : cand_words(sc);
    const bool trig = KIND == 0 || sc == CN_SC_CIRCLE_CROSSING;
    bool elig_l = false;       // eligibility reads only the human's own goal / radius: fixed up front
    if (lane < N) {
        if (KIND == 0) elig_l = en.hvp[lane] != 0;
        else elig_l = norm_lt(en.hgx[lane] - en.hpx[lane], en.hgy[lane] - en.hpy[lane], en.hr[lane]);
    }
    uint64_t rem = __ballot(elig_l);
    dbg += __popcll(rem);
    if (!rem) return dbg;
    GPage pg;
    pg.d = m.sl; pg.cs = m.sl + 64; pg.sn = m.sl + 128;
    gpage_build(m, pg, trig);
    const int NA = N;              // robot + the other N-1 humans
    const int JA = 64 / NA;        // tries per batch the lanes hold
    const int JP = 128 / W;        // tries per batch a fresh page holds
    GP_LAP(t_walk);
    while (rem) {
        // The remaining eligible humans draw U at consecutive stream positions until one of them changes its
        // goal, so all of them are tested at once: lane = human index, rank = its place among them; the
        // first rank with U <= chance (within the page) changes, the draws of the ranks before it are spent.
        if (m.p + 2 > pg.pb + 128) gpage_build(m, pg, trig);
        const int avail = (pg.pb + 128 - m.p) >> 1;   // draws left in the page (>= 1)
        const bool mine = ((rem >> lane) & 1ull) != 0;
        const int rank = __popcll(rem & ((1ull << lane) - 1ull));
        bool hit = false;
        if (mine && rank < avail) hit = pg.dbl(m.p + 2 * rank) <= chance;
        const uint64_t hits = __ballot(hit);
        if (!hits) {   // none of the first min(avail, |rem|) changes: their draws are spent
            const int nr = min(avail, __popcll(rem));
            rem &= ~__ballot(mine && rank < nr);
            m.p += 2 * nr;
            continue;
        }
        const int h = __ffsll((long long)hits) - 1;
        m.p += 2 * (__popcll(rem & ((1ull << h) - 1ull)) + 1);
        rem &= ~((2ull << h) - 1ull);   // h and the humans before it are done
        dbg += 100;
        double r_self = en.hr[h], vpc = en.hvp[h];
        if (KIND == 1) {
            const int jw = 2 * ((c.random_radii ? 1 : 0) + (c.random_v_pref ? 1 : 0));
            if (jw) {
                if (m.p + jw > pg.pb + 128) gpage_build(m, pg, trig);
                if (c.random_radii) { r_self += -0.1 + (0.1 - -0.1) * pg.dbl(m.p); m.p += 2; }
                if (c.random_v_pref) { vpc += -0.1 + (0.1 - -0.1) * pg.dbl(m.p); m.p += 2; }
                if (lane == 0) { en.hr[h] = r_self; en.hvp[h] = vpc; }
            }
        }
        const double vpk = (KIND == 0 && vpc == 0) ? 1.0 : vpc;
        GP_LAP(t_walk);
        for (int t0 = 0;; ) {
            if (t0 > 0) {
                // crowded (the first batch was all rejected): the remaining tries 64 candidates at a time
                // straight from the stream (goal_reject_crowded); its try slots overwrite the page
                const int tw = goal_reject_crowded<GRID>(c, en, m, h, r_self, W, c.max_tries - t0, ovf, [&](int q, int tt) {
                    double gx, gy;
                    if (KIND == 0) {
                        gx = c.circle_radius * m.cos2pi(q) + (m.dbl(q + 2) - 0.5) * vpk;
                        gy = c.circle_radius * m.sin2pi(q) + (m.dbl(q + 4) - 0.5) * vpk;
                    } else {
                        double px, py, hd, vp;
                        cand_attributes(c, m, q, sc, vpc, r_self, en.rr, px, py, gx, gy, hd, vp);
                    }
                    m.sl[tt] = gx; m.sl[64 + tt] = gy;
                }, KIND == 0 ? (CN_COVER_RANDGOAL ? c.circle_radius + 0.5 * fabs(vpk) + 1e-3 : 0.0)
                   : sc == CN_SC_SQUARE_CROSSING ? 0.1 * c.square_width + 0.5 * fabs(vpc == 0 ? 1.0 : vpc) + 1e-3 : 0.0);
                if (lane == 0) { en.hgx[h] = m.sl[tw]; en.hgy[h] = m.sl[64 + tw]; }
                wsync();
                pg.pb = -(1 << 28);   // forces a rebuild before the next read
                GP_LAP(t_rej);
                break;
            }
            if (m.p + W * min(JA, JP) > pg.pb + 128) gpage_build(m, pg, trig);
            const int J = min(min(JA, (pg.pb + 128 - m.p) / W), c.max_tries - t0);   // >= 1
            const int t = lane / NA, a = lane - t * NA;
            const bool valid = t < J;
            double gx = 0, gy = 0;
            bool bad = true;
            if (valid) {
                const int q = m.p + W * t;
                if (KIND == 0) {
                    gx = c.circle_radius * pg.cos2pi(q) + (pg.dbl(q + 2) - 0.5) * vpk;
                    gy = c.circle_radius * pg.sin2pi(q) + (pg.dbl(q + 4) - 0.5) * vpk;
                } else {
                    double px, py, hd, vp;
                    cand_attributes(c, pg, q, sc, vpc, r_self, en.rr, px, py, gx, gy, hd, vp);
                }
                bad = goal_hit(c, en, h, r_self, gx, gy, a);
            }
            dbg += 1000;
            const uint64_t badm = __ballot(bad);
            const uint64_t gmask = NA >= 64 ? ~0ull : ((1ull << NA) - 1ull);
            int win = -1;
            for (int k = 0; k < J; ++k)
                if (((badm >> (k * NA)) & gmask) == 0) { win = k; break; }
            if (win < 0 && t0 + J >= c.max_tries) { win = J - 1; ++ovf; }
            if (win >= 0) {
                if (lane == win * NA) { en.hgx[h] = gx; en.hgy[h] = gy; }   // the winning try's a = 0 lane
                m.p += W * (win + 1);
                wsync();
                break;
            }
            m.p += W * J;
            t0 += J;
        }
        GP_LAP(t_first);
    }
#ifdef CN_STAMPS
    if (lane == 0 && edbg >= 0 && edbg < 8192) {
        cn_stamp_b[edbg * CN_NSTAMP + 8 + 3 * KIND] = t_walk;
        cn_stamp_b[edbg * CN_NSTAMP + 9 + 3 * KIND] = t_first;
        cn_stamp_b[edbg * CN_NSTAMP + 10 + 3 * KIND] = t_rej;
    }
#endif
#undef GP_LAP
    (void)edbg;
    return dbg;
}

// Goal changes at the end of CrowdSimDict.step (crowd_sim_dict.py:260-269) for one env, one wave:
// update_human_goals_randomly when `rgoal`, then update_human_goal when `egoal` (goal_pass).
// `en` holds the post-move agents (LDS); the env's MT19937 stream is loaded from / written back to
// the state; `sp` = wave LDS scratch.
template <bool GRID>
__device__ __forceinline__ void goal_changes(const cn_config &c, const cn_state_ptrs &S, int64_t e, Env1 &en, WRng &m,
                                             bool rgoal, bool egoal, double *sp)
{
    const int N = c.human_num;
    const int lane = m.lane;
    uint32_t *mtw = m.w;
    const int64_t hb = e * N;
    m.off = 0;
    if (m.phx) m.key = S.mt[e * CN_MT_N];
    else {
        uint32_t v[(CN_MT_N + 63) / 64];
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; v[j] = k < CN_MT_N ? S.mt[e * CN_MT_N + k] : 0u; }
#pragma unroll
        for (int j = 0; j < (CN_MT_N + 63) / 64; ++j) { const int k = lane + 64 * j; if (k < CN_MT_N) mtw[k] = v[j]; }
    }
    m.p = S.mt_pos[e];
    m.have1 = false; m.slid = false;
    uint32_t ovf = S.overflow[e];
    const int sc = S.scenario[e];
    wsync();
    STAMP_B(e, 1);
    int dbg0 = 0, dbg1 = 0;
    if (rgoal) dbg0 = goal_pass<0, GRID>(c, en, m, ovf, sc, sp, e);
    STAMP_B(e, 2);
    if (egoal) dbg1 = goal_pass<1, GRID>(c, en, m, ovf, sc, sp, e);
    STAMP_B(e, 3);
#ifdef CN_STAMPS
    if (lane == 0 && e < 8192) { cn_stamp_b[e * CN_NSTAMP + 6] = dbg0; cn_stamp_b[e * CN_NSTAMP + 7] = dbg1; }
#endif
    (void)dbg0; (void)dbg1;
    // numpy twists lazily: a stream that consumed exactly the 624 words is (old key, pos 624)
    const bool in1 = !m.phx && m.p > CN_MT_N;
    if (lane < N) {
        S.h_gx[hb + lane] = en.hgx[lane]; S.h_gy[hb + lane] = en.hgy[lane];
        S.h_r[hb + lane] = en.hr[lane]; S.h_vpref[hb + lane] = en.hvp[lane];
    }
    if (in1 || m.slid)
        for (int k = lane; k < CN_MT_N; k += 64) S.mt[e * CN_MT_N + k] = m.blk(in1 ? 1 : 0)[k];
    if (lane == 0) { S.mt_pos[e] = in1 ? m.p - CN_MT_N : m.p; S.overflow[e] = ovf; }
    wsync();
    STAMP_B(e, 4);
}

// Auto-reset of env e (VecEnv worker, shmem_vec_env.py:164-168 -> CrowdSimDict.reset): copy the pending
// spawn when `may_consume` and it is valid for the current key, else draw it here. One wave.
template <bool GRID, bool FENCE = GRID>
__device__ __forceinline__ void reset_env(const ResetOut &o, const PendPtrs &P2, const cn_config &c, int64_t E, int64_t e,
                          int64_t counter_offset, bool may_consume, uint32_t launch_id, WRng &m, Env1 &en,
                          uint32_t *inline_count = nullptr)
{
    const cn_state_ptrs &S = o.s;
    const int N = c.human_num;
    const int lane = m.lane;
    const int64_t cc = S.case_counter[e];
    const int32_t rc = S.reset_count[e];
    const PendPtrs P = pend_slot(P2, rc & 1, E, E * N);
    // An entry completed by THIS launch (a resumed spawn finishing beside this reset) is not consumed: its
    // stores need not be visible yet; the reset draws inline instead.
    // The ok word carries the key it completes and is read first: only an entry completed by an earlier launch
    // FOR THIS KEY is consumed, and no wave of this launch writes such a slot (a slot is rewritten for key rc + 2
    // only after this reset; a spawn of key rc that is written for the first time in this very launch shows the
    // key in its ok word only with id 0 or this launch's), so the payload read after it needs no fence.
    const uint64_t okw = P.ok[e];
    const uint32_t ok = (uint32_t)okw;
    if (FENCE) __threadfence();
    const bool key_ok = (int32_t)(uint32_t)(okw >> 32) == rc && P.cc[e] == cc && P.rc[e] == rc;
    if (may_consume && ok && ok != launch_id && key_ok) {
        if (lane < N) {
            const int64_t h = e * N + lane, EN = E * N;
            double v[7];
#pragma unroll
            for (int f = 0; f < 7; ++f) v[f] = P.h[f * EN + h];
            asm volatile("" ::: "memory");
            en.hpx[lane] = v[0]; en.hpy[lane] = v[1]; en.hgx[lane] = v[2]; en.hgy[lane] = v[3];
            en.hr[lane] = v[4]; en.hvp[lane] = v[5]; en.hth[lane] = v[6];
        }
        en.rpx = P.r[e]; en.rpy = P.r[E + e]; en.rgx = P.r[2 * E + e]; en.rgy = P.r[3 * E + e];
        const double rth = P.r[4 * E + e];
        wsync();
        write_reset(o, c, e, en, rth, P.sc[e], P.ovf[e], P.mt + e * CN_MT_N, P.pos[e], lane);
    } else {
        double rth;
        uint32_t ovf;
        int sc;
        if (inline_count && lane == 0) atomicAdd(inline_count, 1u);
        spawn_env<GRID>(c, c.env_offset + orow(o.ov, e), cc, rc, counter_offset, m, en, rth, ovf, sc);
        const bool in1 = !m.phx && m.p > CN_MT_N;
        write_reset(o, c, e, en, rth, sc, ovf, m.blk(in1 ? 1 : 0), in1 ? m.p - CN_MT_N : m.p, lane);
    }
    wsync();
}

// Spawn waves of kernel A: draw the next episode of every env reset by the previous kernel A
// (or of every env after cn_reset / cn_set_state). One wave per env, independent of the other waves.
struct PendLaunch {
    PendPtrs P;
    const uint32_t *list;   // envs reset by the previous launch: {e, reset_count, case_counter lo, hi} after it
    const uint32_t *count;
    const uint32_t *rlist;  // spawns parked by the previous launch: {e | 2^31 if not started, key rc, cc lo, cc hi}
    const uint32_t *rcount;
    uint32_t *rlist_w;      // spawns this launch parks
    uint32_t *rcount_w;
    int all;                // PEND_BOTH: every env's two spawns, PEND_FRESH: none (lists ignored); 0: the lists
    int step_blocks, pend_blocks;
    int first;              // 1: workgroups [0, pend_blocks) (kd-tree path); 0: after the step workgroups
    int waves;              // spawning waves per spare workgroup (RNG regions that fit the launch's LDS)
    int stride;             // bytes per spawning wave's region (StepPlan::rng_stride)
    int64_t counter_offset;
    int64_t case_size;
    OutView ov;             // global env index = c.env_offset + orow(ov, e)
    long long budget;       // clock cycles a spawning wave works before parking (0: never parks)
    uint32_t launch_id;     // nonzero id of this launch (pending entries it completes carry it)
    uint32_t *stats;        // [4] cumulative (kd-tree path): parked unstarted, parked mid-way, resumed, completed on
                            // resume; [7] resets of the step workgroups that drew their spawn inline (every path)
};

// GRID: the spawn's crowded rejection through a DiscGrid (the kd-tree path's plans have LDS for it).
// PARK: spawns parked after the launch's budget and resumed later (the kd-tree path; the quad path with
// CN_QUAD_PARK). Items: the envs reset by the previous launch (their spawn for the reset after next), then the spawns
// the previous launch parked. With a budget, a wave parks its spawn between two humans once the budget
// is spent (stream, robot and humans so far go to the pending slot, the item to rlist_w) and parks the
// items it has not started; a later launch resumes them. The pending slot of a spawn is written only by
// the wave that owns the item, and a reset consumes an entry only if an EARLIER launch completed it.
template <bool PHX, bool GRID, bool PARK = GRID>
__device__ __forceinline__ void pend_waves(const PendLaunch &pl, const cn_state_ptrs &S, const cn_config &c, int E, char *smem)
{
    const int nw = pl.waves, w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nw) return;
    if (!GRID && CN_SPAWN_PRIO) __builtin_amdgcn_s_setprio(CN_SPAWN_PRIO);
    const int N = c.human_num;
    char *base = smem + w * pl.stride;
    uint32_t *mtw = (uint32_t *)base;
    double *hb = (double *)(base + 2 * CN_MT_N * 4);
    // envs reset by the previous launch: the reset after next (the next one was drawn earlier); after
    // cn_set_state (PEND_BOTH): both the next (items [0, E)) and the one after ([E, 2E)); after cn_reset
    // (PEND_FRESH, its kernel pre-drew both): none
    const uint32_t nnew = pl.all == PEND_BOTH ? (uint32_t)(2 * E) : pl.all ? 0u : min(*pl.count, (uint32_t)E);
    // parked spawns of the previous launch (PARK)
    const uint32_t nres = (!PARK || pl.all) ? 0u : min(*pl.rcount, (uint32_t)(2 * E));
    const int pb = pl.first ? (int)blockIdx.x : (int)blockIdx.x - pl.step_blocks;
    const long long deadline = (PARK && pl.budget) ? (long long)clock64() + pl.budget : 0;
    bool worked = false;   // a wave always works on its first item of the launch (progress for any budget)
    for (uint32_t it = (uint32_t)(pb * nw + w); it < nnew + nres; it += (uint32_t)(pl.pend_blocks * nw)) {
        int64_t e, cc;
        int32_t rc;
        bool started = false;
        if (it < nnew) {
            const bool ahead2 = pl.all != PEND_BOTH || it >= (uint32_t)E;
            // the key's counters come from a list entry, never from the state: the step workgroups of this
            // same launch reset terminal envs and rewrite reset_count / case_counter while the spawn waves run.
            // PEND_BOTH: cn_keysnap_kernel's snapshot of every env's counters, written (stream-ordered) by
            // cn_set_state / cn_reset before this launch (entry e for items e and e + E); otherwise the
            // counters the previous launch's reset wrote (round 5: read back by the resetting wave)
            const uint32_t *q = pl.list + 4 * (pl.all ? it % (uint32_t)E : it);
            e = (int64_t)q[0];
            rc = (int32_t)q[1];
            cc = (int64_t)((uint64_t)q[2] | ((uint64_t)q[3] << 32));
            if (ahead2) { cc = (cc + c.nenv) % pl.case_size; rc += 1; }   // write_reset's counter update
        } else {
            const uint32_t *q = pl.rlist + 4 * (it - nnew);
            e = (int64_t)(q[0] & 0x7fffffffu);
            started = (q[0] >> 31) == 0u;
            rc = (int32_t)q[1];
            cc = (int64_t)((uint64_t)q[2] | ((uint64_t)q[3] << 32));
            // its reset has come and gone (drawn inline). reset_count may be advanced by a reset of this same
            // launch while it is read; either value is safe: such a reset draws inline (the parked entry is not
            // complete), so the item only turns stale, and the next writer of its slot (key rc + 2, queued by
            // that reset) belongs to the next launch, stream-ordered after this item's stores
            if (rc < S.reset_count[e]) continue;
        }
        if (deadline && worked && (long long)clock64() > deadline) {   // out of budget: park the item unstarted / as is
            if (lane == 0) {
                atomicAdd(pl.stats + (started ? 1 : 0), 1u);
                const uint32_t k = atomicAdd(pl.rcount_w, 1u);
                if (k < (uint32_t)(2 * E)) {
                    uint32_t *q = pl.rlist_w + 4 * k;
                    q[0] = (uint32_t)e | (started ? 0u : 0x80000000u); q[1] = (uint32_t)rc;
                    q[2] = (uint32_t)(uint64_t)cc; q[3] = (uint32_t)((uint64_t)cc >> 32);
                }
            }
            continue;
        }
        Env1 en;
        en.hpx = hb; en.hpy = hb + 32; en.hgx = hb + 64; en.hgy = hb + 96; en.hr = hb + 128; en.hvp = hb + 160;
        en.hth = hb + 192;
        WRng m;
        m.w = mtw; m.off = 0; m.lane = lane; m.phx = PHX; m.edbg = -1;
        m.grid = pl.stride > CN_PEND_LDS ? base + CN_PEND_LDS : nullptr;
        m.sl = (double *)(base + 2 * CN_MT_N * 4 + 7 * 32 * 8);
        double rth = 0;
        uint32_t ovf = 0;
        int sc = 0, i0 = 0;
        if (PARK && started) {   // restore the parked spawn: stream at the park point, robot, the humans so far
            const PendPtrs P = pend_slot(pl.P, rc & 1, E, (int64_t)E * N);
            i0 = P.prog[e];
            const int nk = PHX ? 1 : CN_MT_N;
            for (int k = lane; k < nk; k += 64) mtw[k] = P.mt[e * CN_MT_N + k];
            if (lane < i0) {
                const int64_t h = e * N + lane, EN = (int64_t)E * N;
                en.hpx[lane] = P.h[h]; en.hpy[lane] = P.h[EN + h]; en.hgx[lane] = P.h[2 * EN + h];
                en.hgy[lane] = P.h[3 * EN + h]; en.hr[lane] = P.h[4 * EN + h]; en.hvp[lane] = P.h[5 * EN + h];
                en.hth[lane] = P.h[6 * EN + h];
            }
            en.rpx = P.r[e]; en.rpy = P.r[E + e]; en.rgx = P.r[2 * E + e]; en.rgy = P.r[3 * E + e];
            rth = P.r[4 * E + e];
            en.rr = c.robot_radius;
            ovf = P.ovf[e]; sc = P.sc[e];
            m.p = P.pos[e]; m.have1 = false; m.slid = false;
            m.key = mtw[0];
            if (lane == 0) atomicAdd(pl.stats + 2, 1u);
            wsync();
        }
#ifdef CN_STAMPS
        const unsigned long long ts0 = clock64();
#endif
        const int done = spawn_env<GRID>(c, c.env_offset + orow(pl.ov, e), cc, rc, pl.counter_offset, m, en, rth, ovf,
                                         sc, i0, deadline);
        worked = true;
        const bool in1 = !m.phx && m.p > CN_MT_N;
        write_pending<PARK && CN_SLOT_FENCE>(pl.P, c, E, e, en, rth, sc, ovf, m.blk(in1 ? 1 : 0), in1 ? m.p - CN_MT_N : m.p, cc, rc,
                      lane, done == N ? pl.launch_id : 0u, done);
        if (PARK && started && done == N && lane == 0) atomicAdd(pl.stats + 3, 1u);
        if (PARK && done < N && lane == 0) {   // parked mid-way
            atomicAdd(pl.stats + 1, 1u);
            const uint32_t k = atomicAdd(pl.rcount_w, 1u);
            if (k < (uint32_t)(2 * E)) {
                uint32_t *q = pl.rlist_w + 4 * k;
                q[0] = (uint32_t)e; q[1] = (uint32_t)rc;
                q[2] = (uint32_t)(uint64_t)cc; q[3] = (uint32_t)((uint64_t)cc >> 32);
            }
        }
#ifdef CN_STAMPS
        if (lane == 0 && e < 8192 && done == N) { cn_stamp_p[2 * e] = ts0; cn_stamp_p[2 * e + 1] = clock64(); }
#endif
        wsync();
    }
}

// ------------------------------------------------------------------------------------------------
// kernel A
// ------------------------------------------------------------------------------------------------
struct StepArgs {
    cn_state_ptrs s;
    const float *actions;
    float *robot_node, *temporal, *spatial;
    float *reward;
    uint8_t *done;
    int8_t *event;
    float *info;
    double *ep_return;
    int32_t *ep_len;
    // graph mode (cn_set_graph_mode, the DEVSEQ kernels): the launch's position in the step sequence lives on the device (ctl =
    // the engine's work_count words: [CN_CTL_NSTEP] launches so far, [CN_CTL_ALL] draw every env's next
    // spawn, [CN_CTL_DONE] finished workgroups; the last workgroup of a launch advances them), so a launch
    // has no per-call arguments and a sequence of cn_step calls can be captured in a hipGraph and replayed;
    // the pointers below are then derived at the top of the kernel. Otherwise the host passes them.
    uint32_t *ctl;
    uint32_t *plist_base;   // [3][E + 64][4] spawn lists: {env, reset_count, case_counter lo, hi} after the reset
    uint32_t *rlist_base;   // [3][2E + 64][4] parked-spawn lists
    uint32_t *plist_w;      // envs reset by this launch (their next spawn is drawn by the next launch)
    uint32_t *pcount_w;
    uint32_t *pcount_zero;  // the counter the NEXT launch appends to (triple-buffered), zeroed here
    uint32_t *rcount_zero;  // likewise for the parked-spawn list
    PendLaunch pend;        // spawn waves: the first or the last pend_blocks workgroups (pend.first)
    int64_t case_size;
    int E;
    OutView ov;             // output rows / human stride (mixed engines); also pend.ov
    double cth_h, cth_r;    // cos(human_fov / 2), cos(robot_fov / 2): in_fov's thresholds
};

// phase 5 reads cn_config from the kernarg segment right after StepArgs (cn_step_kernel's RNG loop): the
// by-value arguments are laid out in order at their natural alignment (AMDHSA metadata: 0 / 720 today)
static_assert(alignof(StepArgs) >= alignof(cn_config) || sizeof(StepArgs) % alignof(cn_config) == 0,
              "cn_step_kernel's kernarg layout: cn_config follows StepArgs");

// observed agent of slot k seen by lane (human i of env base eb): position/velocity float32,
// frozen RVO2 radius; `vis` = visible now, `dm` = dummy at simulator creation
__device__ inline void slot_agent(const SL &sl, const cn_config &c, int eb, int el, int EPB, int N, int i, int k,
                                  uint32_t vis, uint32_t dm, float rdummy, float &x, float &y, float &vx, float &vy,
                                  float &r)
{
    const bool v = (vis >> k) & 1u;
    if (k < N - 1) {
        const int j = eb + (k < i ? k : k + 1);
        if (v) {
            x = (float)HF(sl, H_PX, j); y = (float)HF(sl, H_PY, j);
            vx = (float)HF(sl, H_VX, j); vy = (float)HF(sl, H_VY, j);
        } else { x = (float)CN_DUMMY_POS; y = (float)CN_DUMMY_POS; vx = 0.0f; vy = 0.0f; }
        r = ((dm >> k) & 1u) ? rdummy : sl.orad[j];
    } else {  // robot slot (robot.visible)
        if (v) {
            x = (float)RF(sl, R_PX, el, EPB); y = (float)RF(sl, R_PY, el, EPB);
            vx = (float)RF(sl, R_VX, el, EPB); vy = (float)RF(sl, R_VY, el, EPB);
        } else { x = (float)CN_DUMMY_POS; y = (float)CN_DUMMY_POS; vx = 0.0f; vy = 0.0f; }
        r = ((dm >> k) & 1u) ? (float)(c.robot_radius + 0.01 + c.orca_safety_space)
                             : (float)(RF(sl, R_RAD, el, EPB) + 0.01 + c.orca_safety_space);
    }
}

__device__ inline float bbox_dist(float x, float y, float mnx, float mxx, float mny, float mxy)
{
    const float a = (0.0f < mnx - x) ? mnx - x : 0.0f, b = (0.0f < x - mxx) ? x - mxx : 0.0f;
    const float cc = (0.0f < mny - y) ? mny - y : 0.0f, d = (0.0f < y - mxy) ? y - mxy : 0.0f;
    return a * a + b * b + cc * cc + d * d;
}

// KD: RVO2 kd-tree neighbour order (> 10 agents per simulator); PHX: c.rng_mode == CN_RNG_PHILOX, a
// template argument so that the MT19937 build carries no Philox registers
// MIX: a group of a mixed engine (outputs through g.ov); a plain engine's identity view is then a
// compile-time constant and costs no registers
// DEVSEQ: graph mode (StepArgs::devseq), a variant of its own so the default launches carry none of it
template <bool KD, bool PHX, bool MIX, bool DEVSEQ = false>
__global__ void __launch_bounds__(CN_BLK, 3) cn_step_kernel(StepArgs g, cn_config c)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const OutView ov = MIX ? g.ov : OutView{nullptr, c.human_num};
    // this launch's spawn / parked-spawn lists (triple-buffered: launch t appends to t % 3, reads (t - 1) % 3,
    // zeroes (t + 1) % 3) and id, from the device-side step counter
    const uint32_t ns = DEVSEQ ? g.ctl[CN_CTL_NSTEP] : 0u;
    if (DEVSEQ) {
        const int64_t kw = ns % 3u, kr = (ns + 2u) % 3u, kz = (ns + 1u) % 3u;
        const int64_t ls = 4 * ((int64_t)g.E + 64), rs = 4 * (2 * (int64_t)g.E + 64);
        g.plist_w = g.plist_base + kw * ls;
        g.pcount_w = g.ctl + 2 + kw;
        g.pcount_zero = g.ctl + 2 + kz;
        g.rcount_zero = g.ctl + 5 + kz;
        g.pend.list = g.plist_base + kr * ls;
        g.pend.count = g.ctl + 2 + kr;
        g.pend.rlist = g.rlist_base + kr * rs;
        g.pend.rcount = g.ctl + 5 + kr;
        g.pend.rlist_w = g.rlist_base + kw * rs;
        g.pend.rcount_w = g.ctl + 5 + kw;
        g.pend.launch_id = ((ns + 1u) % 0x7ffffffeu) + 1u;   // nonzero, differs from the neighbours'
        g.pend.all = (int)g.ctl[CN_CTL_ALL];
    }
    // the last workgroup to finish advances the sequence (every workgroup has read it by then)
    // (the atomic carries a register dependency on this workgroup's read of the counter, so the read has
    // completed before the count can reach the grid size)
    STAMP_R(0);
    auto finish = [&]() {
#ifdef CN_STAMPS
        __syncthreads();
        STAMP_R(1);
#endif
        if (!DEVSEQ) return;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t dep;
            asm volatile("v_mov_b32 %0, 0" : "=v"(dep) : "v"(ns));
            if (atomicAdd(g.ctl + CN_CTL_DONE, 1u + dep) == gridDim.x - 1) {
                g.ctl[CN_CTL_DONE] = 0u;
                g.ctl[CN_CTL_ALL] = 0u;
                g.ctl[CN_CTL_NSTEP] = ns + 1u;
            }
        }
    };
    // the spawn-list counter the NEXT launch appends to (neither read nor appended to by this launch)
    if (blockIdx.x == 0 && threadIdx.x == 0) { *g.pcount_zero = 0u; *g.rcount_zero = 0u; }
    const int sb = (int)blockIdx.x - (g.pend.first ? g.pend.pend_blocks : 0);   // step workgroup index
    if (sb < 0 || sb >= g.pend.step_blocks) {  // spare workgroups: draw upcoming episodes' spawns
        PendLaunch pl = g.pend;
        pl.ov = ov;
        pend_waves<PHX, KD, KD || CN_QUAD_PARK>(pl, g.s, c, g.E, smem);
        finish();
        return;
    }
    const int N = c.human_num;
    const StepPlan P = cn_step_plan(N, c.robot_visible);
    const int EPB = P.EPB, M = P.M, A = P.A;
    SL sl;
    sl.T = P.H;
    sl.r = (double *)(smem + P.o_renv);
    sl.act = (float *)(smem + P.o_racts);
    sl.rflag = (uint32_t *)(smem + P.o_rflag);
    sl.rvr = (double *)(smem + P.o_rvr);
    sl.hvr = (double *)(smem + P.o_hvr);
    sl.hst = (double *)(smem + P.o_hst);
    sl.h = (double *)(smem + P.o_hum);
    sl.cd = (double *)(smem + P.o_lane);
    sl.lf = (uint32_t *)(smem + P.o_lane + P.H * 8);
    sl.orad = (float *)(smem + P.o_orad);
    sl.vis = (uint32_t *)(smem + P.o_vis);
    sl.dm = sl.vis + P.H;
    sl.vmax = (float *)(sl.vis + 2 * P.H);
    sl.npx = (double *)(smem + P.o_nv);
    sl.npy = sl.npx + P.H;
    sl.eg = (uint32_t *)(smem + P.o_eg);
    sl.lines = (float4 *)(smem + P.o_lines);
    sl.proj = (float4 *)(smem + P.o_proj);
    sl.nd = (float *)(smem + P.o_nd);
    sl.ns = (uint8_t *)(smem + P.o_ns);
    sl.perm = (uint8_t *)(smem + P.o_perm);
    const cn_state_ptrs &S = g.s;
    // human hh's velocity-rectangle corner k (x0..x3, y0..y3) and human_post's staged value f: [8][H] / [7][H]
    // arrays on the quad path, the human's own projected-line block on the kd-tree path (StepPlan)
    auto hvr_ref = [&](int hh, int k) -> double & {
        return KD ? ((double *)(sl.proj + hh * M))[k] : sl.hvr[k * 64 + hh];
    };
    auto hst_ref = [&](int hh, int f) -> double & {
        return KD ? ((double *)(sl.proj + hh * M))[f] : sl.hst[f * 64 + hh];
    };

    const int tid = threadIdx.x;
    // XCD-aware env placement: workgroup i runs on XCD i % 8 (round-robin dispatch; for speed only), so
    // give each XCD a contiguous run of env blocks. Neighbouring workgroups share the 128-B lines at the
    // ends of their SoA segments (a per-env field of one workgroup is only 48 B); on one XCD the second
    // reader hits in that XCD's L2 instead of fetching the line again.
    // (a leading pend_blocks is a multiple of 8, so step workgroup sb runs on XCD sb % 8 as well)
    const int nbk = g.pend.step_blocks, xq = nbk >> 3, xr = nbk & 7, xi = sb & 7;
    const int blk = xi * xq + min(xi, xr) + (sb >> 3);
    const int e0 = blk * EPB;
    const int nenv_here = min(EPB, g.E - e0);
    const int el = tid / N, i = tid - el * N;
    const bool hl = el < nenv_here;               // human lane
    const int gh = (e0 + el) * N + i;                 // global human index (E*N < 2^31, cn_config_validate)
    // env lanes (robot / reward / bookkeeping): wave 1 on the quad path, so they run beside the human
    // lanes of wave 0 in phases 0, 3 and 4; the first lanes on the kd-tree path
    const int re = tid - 64;
    const bool rl = re >= 0 && re < nenv_here;
    const int ge = e0 + re;
    const bool holo = c.kinematics == CN_HOLONOMIC;
    const double dt = c.time_step;

    STAMP_A(0);
    // ---- phase 0: load state into LDS -----------------------------------------------------------
    // values needed in later phases are loaded here, so their latency overlaps phase 0 (doubles parked
    // in LDS rather than registers across the ORCA phase)
    float pre_or = 0.0f, pre_vmax = 0.0f;
    uint32_t pre_dm = 0u;
    int32_t pre_epl = 0, pre_sc = 0;
    uint32_t pre_ovf = 0;
    // With a 360-degree robot FOV every human the robot can see is visible (only coincident agents are
    // not), so the previous belief is read only in that rare case, straight from the state in phase 4
    const bool rfull = c.robot_fov >= 2.0 * CN_PI;
    if (hl) {
        // every load issued before the first LDS store (the compiler otherwise waits on each load in turn)
        double hv[CN_HUM_F];
        pre_or = S.o_r[gh]; pre_vmax = S.o_vmax[gh]; pre_dm = S.o_dmask[gh];
        hv[H_PX] = S.h_px[gh]; hv[H_PY] = S.h_py[gh]; hv[H_GX] = S.h_gx[gh]; hv[H_GY] = S.h_gy[gh];
        hv[H_VX] = S.h_vx[gh]; hv[H_VY] = S.h_vy[gh]; hv[H_R] = S.h_r[gh]; hv[H_VP] = S.h_vpref[gh];
        hv[H_TH] = S.h_theta[gh];
        if (!rfull) {
            hv[H_BPX] = S.b_px[gh]; hv[H_BPY] = S.b_py[gh]; hv[H_BVX] = S.b_vx[gh]; hv[H_BVY] = S.b_vy[gh];
            hv[H_BR] = S.b_r[gh];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int f = 0; f < H_BPX; ++f) HF(sl, f, tid) = hv[f];
        if (!rfull) {
#pragma unroll
            for (int f = H_BPX; f < CN_HUM_F; ++f) HF(sl, f, tid) = hv[f];
        }
    }
    STAMP_A(12);
    if (rl) {
        double rv[CN_RENV_F];
        rv[R_PX] = S.r_px[ge]; rv[R_PY] = S.r_py[ge]; rv[R_GX] = S.r_gx[ge]; rv[R_GY] = S.r_gy[ge];
        rv[R_VX] = S.r_vx[ge]; rv[R_VY] = S.r_vy[ge]; rv[R_TH] = S.r_theta[ge]; rv[R_RAD] = S.r_radius[ge];
        rv[R_VP] = S.r_vpref[ge]; rv[R_POT] = S.potential[ge]; rv[R_GT] = S.gtime[ge]; rv[R_DV] = S.r_dv[ge];
        rv[R_LAX] = S.last_ax[ge]; rv[R_LAY] = S.last_ay[ge]; rv[R_EPR] = S.ep_return[ge];
        const uint32_t fl = S.flags[ge];
        pre_epl = S.ep_len[ge]; pre_sc = S.scenario[ge]; pre_ovf = S.overflow[ge];
        const int64_t oa = orow(ov, ge);   // the env's row in the caller's buffers
        float a0 = g.actions[oa * 2], a1 = g.actions[oa * 2 + 1];
        asm volatile("" ::: "memory");
        RF(sl, R_PX, re, EPB) = rv[R_PX]; RF(sl, R_PY, re, EPB) = rv[R_PY];
        RF(sl, R_GX, re, EPB) = rv[R_GX]; RF(sl, R_GY, re, EPB) = rv[R_GY];
        RF(sl, R_VX, re, EPB) = rv[R_VX]; RF(sl, R_VY, re, EPB) = rv[R_VY];
        RF(sl, R_TH, re, EPB) = rv[R_TH]; RF(sl, R_RAD, re, EPB) = rv[R_RAD];
        RF(sl, R_VP, re, EPB) = rv[R_VP]; RF(sl, R_POT, re, EPB) = rv[R_POT];
        RF(sl, R_GT, re, EPB) = rv[R_GT]; RF(sl, R_DV, re, EPB) = rv[R_DV];
        RF(sl, R_LAX, re, EPB) = rv[R_LAX]; RF(sl, R_LAY, re, EPB) = rv[R_LAY]; RF(sl, R_EPR, re, EPB) = rv[R_EPR];
        sl.rflag[re] = fl;
        STAMP_A(13);
        // ---- SRNN.clip_action (srnn.py:18-48) + unicycle integrator (crowd_sim_dict.py:211-217)
        if (holo) {
            const float n = np_norm2f(a0, a1);
            if ((double)n > RF(sl, R_VP, re, EPB)) {
                const float vp = (float)RF(sl, R_VP, re, EPB);
                a0 = fdiv(a0, n) * vp; a1 = fdiv(a1, n) * vp;
            }
        } else {
            a0 = np_clipf(a0, -0.1f, 0.1f);
            a1 = np_clipf(a1, -0.1f, 0.1f);
            const float vp = (float)RF(sl, R_VP, re, EPB);
            const float dv = np_clipf((float)RF(sl, R_DV, re, EPB) + a0, -vp, vp);
            RF(sl, R_DV, re, EPB) = dv;
            a0 = dv;
        }
        sl.act[re] = a0; sl.act[EPB + re] = a1;
        STAMP_A(10);
        STAMP_T(16, 64);
    }
    __syncthreads();
    STAMP_A(1);

    // per-human terms of calc_reward (crowd_sim.py:934-969), PRE-move, for human lane hh
    auto reward_terms = [&](int hh) {
        const int elh = hh / N;
        const double px = HF(sl, H_PX, hh), py = HF(sl, H_PY, hh);
        const double vx0 = HF(sl, H_VX, hh), vy0 = HF(sl, H_VY, hh), rad = HF(sl, H_R, hh);
        const double rdx = px - RF(sl, R_PX, elh, EPB), rdy = py - RF(sl, R_PY, elh, EPB);
        sl.cd[hh] = dsqrt(rdx * rdx + rdy * rdy) - rad - RF(sl, R_RAD, elh, EPB);
        double hcx[4], hcy[4];
        vel_rect(px, py, vx0, vy0, rad, false, hcx, hcy);
        for (int k = 0; k < 4; ++k) { hvr_ref(hh, k) = hcx[k]; hvr_ref(hh, 4 + k) = hcy[k]; }
        // (the path-violation test of this rectangle against the robot's runs in human_post, phase 2: the
        // robot's rectangle is computed beside this one, on wave 3)
        uint32_t f = 0u;
        if (!(np_norm2(px - HF(sl, H_GX, hh), py - HF(sl, H_GY, hh)) < rad)) f |= LF_NOTREACHED;
        sl.lf[hh] = f;
    };
    // robot VelocityRectangle (pre-move), phase 1 on wave 3
    auto robot_vr = [&](int q) {
        double cx[4], cy[4];
        vel_rect(RF(sl, R_PX, q, EPB), RF(sl, R_PY, q, EPB), RF(sl, R_VX, q, EPB), RF(sl, R_VY, q, EPB),
                 RF(sl, R_RAD, q, EPB), (sl.rflag[q] & CN_FLAG_ROBOT_F32) != 0, cx, cy);
        for (int k = 0; k < 4; ++k) { sl.rvr[k * EPB + q] = cx[k]; sl.rvr[(4 + k) * EPB + q] = cy[k]; }
    };
    // robot-only terms of calc_reward (crowd_sim.py:973-1030) and the robot's move (agent.py:172-212);
    // independent of the humans, so the quad path computes them in phase 1 on wave 2
    auto robot_terms = [&](int q) {
        const int64_t gq = e0 + q;
        const double rpx = RF(sl, R_PX, q, EPB), rpy = RF(sl, R_PY, q, EPB), rr = RF(sl, R_RAD, q, EPB);
        const double rgx = RF(sl, R_GX, q, EPB), rgy = RF(sl, R_GY, q, EPB);
        const bool rf32 = (sl.rflag[q] & CN_FLAG_ROBOT_F32) != 0;
        const float a0 = sl.act[q], a1 = sl.act[EPB + q];
        const bool reaching_goal = np_norm2(rpx - rgx, rpy - rgy) < rr;
        // commanded world-frame velocity; unicycle: theta + r is float32 (NEP 50)
        const float tr = (float)RF(sl, R_TH, q, EPB) + a1;
        const float th_new = np_modf(tr, (float)(2 * CN_PI));
        double cvx, cvy;
        if (holo) { cvx = a0; cvy = a1; }
        else { cvx = (double)(a0 * np_cosf(th_new)); cvy = (double)(a0 * np_sinf(th_new)); }
        // unicycle differential drive (agent.py:185-194)
        double upx = rpx, upy = rpy;
        if (!holo && !(fabsf(a1) < 0.0001f)) {
            const float w = fdiv(a1, (float)dt);
            const float R = fdiv(a0, w);
            const double th = RF(sl, R_TH, q, EPB);
            double t1x, t1y;
            if (rf32) { t1x = (double)(R * np_sinf((float)th)); t1y = (double)(R * np_cosf((float)th)); }
            else { t1x = (double)R * sin(th); t1y = (double)R * cos(th); }
            upx = rpx - t1x + (double)(R * np_sinf(tr));
            upy = rpy + t1y - (double)(R * np_cosf(tr));
        }
        double side_l = 0, side_r = 0, sep = 0;
        if (c.side_preference) {
            const int eb = q * N;
            double ex, ey;
            if (holo) { ex = rpx + (double)(a0 * (float)dt); ey = rpy + (double)(a1 * (float)dt); }
            else { ex = upx; ey = upy; }
            const double hy = HF(sl, H_PY, eb), hr = HF(sl, H_R, eb);
            if (ey <= hy + hr && ey >= hy - hr) { if (ex < HF(sl, H_PX, eb)) side_l = 1; else side_r = 1; }
            sep = np_norm2(HF(sl, H_PX, eb) - rpx, HF(sl, H_PY, eb) - rpy);
        }
        {   // jerk (crowd_sim.py:1002-1009), float32 like the reference's np.float32 action
            const float ax = (float)cvx - (float)RF(sl, R_VX, q, EPB), ay = (float)cvy - (float)RF(sl, R_VY, q, EPB);
            const float dax = ax - (float)RF(sl, R_LAX, q, EPB), day = ay - (float)RF(sl, R_LAY, q, EPB);
            RF(sl, R_JERK, q, EPB) = (double)(dax * dax + day * day);
            S.last_ax[gq] = ax; S.last_ay[gq] = ay;
        }
        RF(sl, R_D2G, q, EPB) = np_norm2(rpx - rgx, rpy - rgy);
        const bool inside = inside_world(rpx, rpy, rr, c.square_width / 2);
        { const float fx = (float)cvx, fy = (float)cvy; RF(sl, R_SPD, q, EPB) = (double)fsqrt(fx * fx + fy * fy); }
        RF(sl, R_SL, q, EPB) = side_l; RF(sl, R_SR, q, EPB) = side_r; RF(sl, R_SEP, q, EPB) = sep;
        RF(sl, R_BITS, q, EPB) = (double)((reaching_goal ? 1u : 0u) | (inside ? 2u : 0u));
        RF(sl, R_CVX, q, EPB) = cvx; RF(sl, R_CVY, q, EPB) = cvy; RF(sl, R_NTH, q, EPB) = th_new;
        if (holo) {
            RF(sl, R_NX, q, EPB) = rpx + (double)(a0 * (float)dt);
            RF(sl, R_NY, q, EPB) = rpy + (double)(a1 * (float)dt);
        } else { RF(sl, R_NX, q, EPB) = upx; RF(sl, R_NY, q, EPB) = upy; }
    };
    // ---- phase 1: visibility of the other agents to human i, frozen simulator parameters --------
    // (quad path: wave 1 computes the per-human reward terms, wave 2 the robot terms meanwhile)
    if (tid >= 64 && tid - 64 < nenv_here * N) reward_terms(tid - 64);
    STAMP_T(17, 64);
    if (tid >= 128 && tid - 128 < nenv_here) robot_terms(tid - 128);
    STAMP_T(18, 128);
    if (tid >= 192 && tid - 192 < nenv_here) robot_vr(tid - 192);
    const bool orca = c.human_policy == CN_POLICY_ORCA;
    uint32_t vis = 0, dm = 0;
    float my_vmax = 0.0f;
    bool frozen = true;
    if (hl) {
        const int eb = el * N;
        double fx = 0, fy = 0;
        bool have_dir = false;
        auto dir = [&]() {
            if (!have_dir) {
                if (holo) fov_dir64(atan2(HF(sl, H_VY, tid), HF(sl, H_VX, tid)), fx, fy);
                else fov_dir64(HF(sl, H_TH, tid), fx, fy);
                have_dir = true;
            }
        };
        const bool full = c.human_fov >= 2.0 * CN_PI;
        const bool hfin = holo ? (HF(sl, H_VX, tid) == HF(sl, H_VX, tid) && HF(sl, H_VY, tid) == HF(sl, H_VY, tid))
                               : isfinite(HF(sl, H_TH, tid));
        const double px = HF(sl, H_PX, tid), py = HF(sl, H_PY, tid);
        uint32_t undecided = 0;   // 360-degree FOV: decided without the heading except at |v|^2 extremes
        if (full) {
#pragma unroll 4
            for (int k = 0; k < N - 1; ++k) {
                const int j = eb + (k < i ? k : k + 1);
                const int v = vis360(hfin, px, py, HF(sl, H_PX, j), HF(sl, H_PY, j));
                if (v > 0) vis |= 1u << k;
                if (v < 0) undecided |= 1u << k;
            }
        } else undecided = (N - 1 >= 32) ? 0xffffffffu : ((1u << (N - 1)) - 1u);
        for (uint32_t um = undecided; um; um &= um - 1) {
            const int k = __ffs(um) - 1;
            const int j = eb + (k < i ? k : k + 1);
            dir();
            if (in_fov_fast(fx, fy, px, py, HF(sl, H_PX, j), HF(sl, H_PY, j), c.human_fov, g.cth_h)) vis |= 1u << k;
        }
        if (c.robot_visible) {
            int v = full ? vis360(hfin, px, py, RF(sl, R_PX, el, EPB), RF(sl, R_PY, el, EPB)) : -1;
            if (v < 0) {
                dir();
                v = in_fov_fast(fx, fy, px, py, RF(sl, R_PX, el, EPB), RF(sl, R_PY, el, EPB), c.human_fov, g.cth_h) ? 1 : 0;
            }
            if (v) vis |= 1u << (N - 1);
        }
        if (orca) {
            frozen = (sl.rflag[el] & CN_FLAG_ORCA_FROZEN) != 0;
            if (frozen) {
                sl.orad[tid] = pre_or;
                my_vmax = pre_vmax;
                dm = pre_dm;
            } else {  // first ORCA.predict of the episode creates the simulator (orca.py:85-109)
                sl.orad[tid] = (float)(HF(sl, H_R, tid) + 0.01 + c.orca_safety_space);
                my_vmax = (float)HF(sl, H_VP, tid);
                dm = ~vis & ((M >= 32) ? 0xffffffffu : ((1u << M) - 1u));
                S.o_r[gh] = sl.orad[tid];
                S.o_vmax[gh] = my_vmax;
                S.o_dmask[gh] = dm;
            }
        }
        sl.vis[tid] = vis; sl.dm[tid] = dm; sl.vmax[tid] = my_vmax;
    }
    STAMP_T(19, 0);
    __syncthreads();
    STAMP_A(2);

    // calc_reward ladder + Monitor (crowd_sim.py:907-1094) for env lane re: reads only phase-1 results (pre-move
    // distances / flags and the robot-only terms), so it runs inside phase 2 on the env lanes (wave 1, after
    // its own ORCA quads), in the slack while the slowest humans finish their linear programs. The robot's
    // kinematics update (which the ORCA simulators must not see yet) is applied after phase 2.
    bool ladder_done = false;   // the quad ORCA path runs it inside phase 2 (before the linearProgram3 tasks)
    auto ladder = [&]() {
        const double rr = RF(sl, R_RAD, re, EPB);
        const uint32_t flags = sl.rflag[re];
        const float a0 = sl.act[re], a1 = sl.act[EPB + re];
        const int eb = re * N;
        double dmin = INFINITY;
        bool collision = false, nz_viol = false;
        int agg = 0, kv = N;
        for (int k = 0; k < N; ++k) {
            const double cd = sl.cd[eb + k];
            if (cd < 0) { collision = true; kv = k; break; }
            else if (cd < dmin) dmin = cd;
            const uint32_t f = sl.lf[eb + k];
            agg += (f & LF_NOTREACHED) ? 1 : 0;
        }
        sl.rflag[2 * EPB + re] = (uint32_t)kv;   // the path violations of humans k < kv are counted after phase 2
        // the reference tests the norm zones inside the loop once human 0 is not a collision; the penalty
        // is read only on the no-collision branch of the ladder, where the loop ran past human 0, so
        // testing it here (outside the loop: the call's register saves only run when it is taken) is
        // the same
        if (c.norm_zones && !collision)
            nz_viol = robot_norm_zone_violation(RF(sl, R_PX, re, EPB), RF(sl, R_PY, re, EPB), RF(sl, R_VX, re, EPB),
                                                RF(sl, R_VY, re, EPB), rr, (flags & CN_FLAG_ROBOT_F32) != 0,
                                                c.norm_zone_lhs);
        const uint32_t bits = (uint32_t)RF(sl, R_BITS, re, EPB);
        const bool reaching_goal = (bits & 1u) != 0, inside = (bits & 2u) != 0;
        if (!reaching_goal) ++agg;
        const double dist_to_goal = RF(sl, R_D2G, re, EPB);
        const double gt = RF(sl, R_GT, re, EPB);
        double reward;
        int done, event;
        if (gt >= c.time_limit - 1) { reward = 0; done = 1; event = CN_EV_TIMEOUT; }
        else if (collision || !inside) { reward = c.collision_penalty; done = 1; event = CN_EV_COLLISION; }
        else if (reaching_goal) {
            reward = c.success_reward;
            if (c.time_factor) reward *= ddiv(c.time_limit - gt, c.time_limit);
            done = 1; event = CN_EV_REACHGOAL;
        } else if (dmin < c.discomfort_dist) {
            reward = (dmin - c.discomfort_dist) * c.discomfort_penalty_factor;
            done = 0; event = CN_EV_DANGER;
        } else {
            reward = c.potential_factor * (-fabs(dist_to_goal) - RF(sl, R_POT, re, EPB));
            RF(sl, R_POT, re, EPB) = -fabs(dist_to_goal);
            if (c.norm_zones && nz_viol) reward += c.norm_zone_penalty;
            done = 0; event = CN_EV_NOTHING;
        }
        if (!holo) {
            const float r_spin = -2.0f * (a1 * a1);
            const float r_back = a0 < 0 ? -2.0f * fabsf(a0) : 0.0f;
            if (event == CN_EV_DANGER || event == CN_EV_NOTHING) reward = reward + (double)r_spin + (double)r_back;
            else reward = (double)(((float)reward + r_spin) + r_back);
        }
        if (g.info) {
            float *info = g.info + orow(ov, ge) * CN_INFO_K;
            info[CN_INFO_AGG_NAV_TIME] = (float)agg;
            info[CN_INFO_PERSONAL_VIOLATION] = dmin < c.min_personal_space ? 1.0f : 0.0f;
            info[CN_INFO_JERK_COST] = (float)RF(sl, R_JERK, re, EPB);
            info[CN_INFO_DIST_TO_GOAL] = (float)dist_to_goal;
            info[CN_INFO_SPEED_VIOLATION] = RF(sl, R_SPD, re, EPB) > c.max_walking_speed ? 1.0f : 0.0f;
            info[CN_INFO_MIN_DIST] = (float)dmin;
            info[CN_INFO_SCENARIO] = (float)pre_sc;
            info[CN_INFO_SIDE_LEFT] = (float)RF(sl, R_SL, re, EPB);
            info[CN_INFO_SIDE_RIGHT] = (float)RF(sl, R_SR, re, EPB);
            info[CN_INFO_SEPARATION] = (float)RF(sl, R_SEP, re, EPB);
            info[CN_INFO_OVERFLOW] = (float)pre_ovf;
        }
        RF(sl, R_GT, re, EPB) = gt + dt;
        const double epr = RF(sl, R_EPR, re, EPB) + reward;
        const int32_t epl = pre_epl + 1;
        S.ep_return[ge] = epr; S.ep_len[ge] = epl;
        const int64_t oe = orow(ov, ge);
        if (g.reward) g.reward[oe] = (float)reward;
        if (g.done) g.done[oe] = (uint8_t)done;
        if (g.event) g.event[oe] = (int8_t)event;
        if (g.ep_return) g.ep_return[oe] = epr;
        if (g.ep_len) g.ep_len[oe] = epl;
        sl.rflag[EPB + re] = (uint32_t)done;   // aux word: done
    };
    // human kinematics, robot-FOV belief, observation and goal-reached detection of human hh from its new
    // velocity (agent.py:172-212 step, crowd_sim_dict.py:72-103 generate_ob): called by the lane that
    // produced the velocity as soon as it has it (ORCA: the quad's lane 0 after its linear programs)
    // path violation of human hh (crowd_sim.py:951-957): the robot's and the human's pre-move
    // VelocityRectangles intersect; quad version (4 lanes of the human's quad together) and a lane version
    auto path_vr_q = [&](int hh, int s4) -> bool {
        const int elh = hh / N;
        double rcx[4], rcy[4], hcx[4], hcy[4];
        for (int k = 0; k < 4; ++k) {
            rcx[k] = sl.rvr[k * EPB + elh]; rcy[k] = sl.rvr[(4 + k) * EPB + elh];
            hcx[k] = hvr_ref(hh, k); hcy[k] = hvr_ref(hh, 4 + k);
        }
        return quads_intersect_q(rcx, rcy, hcx, hcy, s4);
    };
    auto path_vr = [&](int hh) -> bool {
        const int elh = hh / N;
        double rcx[4], rcy[4], hcx[4], hcy[4];
        for (int k = 0; k < 4; ++k) {
            rcx[k] = sl.rvr[k * EPB + elh]; rcy[k] = sl.rvr[(4 + k) * EPB + elh];
            hcx[k] = hvr_ref(hh, k); hcy[k] = hvr_ref(hh, 4 + k);
        }
        return quads_intersect(rcx, rcy, hcx, hcy);
    };
    auto human_post = [&](int hh, double nvx, double nvy, bool vr) {
        const int elh = hh / N, ih = hh - elh * N;
        const int ghh = (e0 + elh) * N + ih;
        const double npx = HF(sl, H_PX, hh) + nvx * dt, npy = HF(sl, H_PY, hh) + nvy * dt;
        // detect_visible(robot, human, robot1=True) on the POST-move state (robot velocity now float32)
        const double rnx = RF(sl, R_NX, elh, EPB), rny = RF(sl, R_NY, elh, EPB);
        // the robot's post-move velocity / heading (agent.py:198-212, applied to the state after phase 2):
        // holonomic = the clipped action, unicycle = the commanded velocity and new heading of phase 1
        const float rvx = holo ? sl.act[elh] : (float)RF(sl, R_CVX, elh, EPB);
        const float rvy = holo ? sl.act[EPB + elh] : (float)RF(sl, R_CVY, elh, EPB);
        const float rth = holo ? 0.0f : (float)RF(sl, R_NTH, elh, EPB);
        const bool rfin = holo ? (rvx == rvx && rvy == rvy) : isfinite(rth);
        int rv = c.robot_fov >= 2.0 * CN_PI ? vis360(rfin, rnx, rny, npx, npy) : -1;
        if (rv < 0) {
            double fx, fy;
            if (holo) fov_dir32(atan2f(rvy, rvx), fx, fy);
            else fov_dir32(rth, fx, fy);
            rv = in_fov_fast(fx, fy, rnx, rny, npx, npy, c.robot_fov, g.cth_r) ? 1 : 0;
        }
        double bpx, bpy, bvx, bvy, br;
        if (rv) {
            bpx = npx; bpy = npy; bvx = nvx; bvy = nvy; br = HF(sl, H_R, hh);
        } else {
            if (rfull) {   // coincident with the robot (or a NaN state): the stored belief, extrapolated
                bvx = S.b_vx[ghh]; bvy = S.b_vy[ghh]; br = S.b_r[ghh];
                bpx = S.b_px[ghh] + bvx * dt; bpy = S.b_py[ghh] + bvy * dt;
            } else {
                bvx = HF(sl, H_BVX, hh); bvy = HF(sl, H_BVY, hh); br = HF(sl, H_BR, hh);
                bpx = HF(sl, H_BPX, hh) + bvx * dt; bpy = HF(sl, H_BPY, hh) + bvy * dt;
            }
        }
        // staged in LDS: the state / observation stores go out after phase 2 from consecutive lanes (one
        // lane per quad here would split every 128-B line of a field over several waves' partial writes:
        // +4 MB of HBM writes per C2 launch, measured)
        hst_ref(hh, 0) = nvx; hst_ref(hh, 1) = nvy;
        hst_ref(hh, 2) = bpx; hst_ref(hh, 3) = bpy; hst_ref(hh, 4) = bvx; hst_ref(hh, 5) = bvy;
        hst_ref(hh, 6) = br;
        uint32_t f = vr ? LF_VR : 0u;
        if (np_norm2(HF(sl, H_GX, hh) - npx, HF(sl, H_GY, hh) - npy) < HF(sl, H_R, hh)) f |= LF_ENDGOAL;
        if (!(npx == npx) || !(npy == npy)) f |= 0x80000000u;
        sl.eg[hh] = f;
        sl.npx[hh] = npx; sl.npy[hh] = npy;   // post-move positions for the goal changes (HF keeps the pre-move
                                              // ones: other humans' simulators may still be reading them)
    };
    // ---- phase 2: human policy (PRE-move state) -------------------------------------------------
    double nvx = 0.0, nvy = 0.0;
    {
        const int nh = nenv_here * N;
        if (orca) {
            // ORCA.predict for every human (orca.py:64-139), a quad of lanes per human. The neighbour list
            // (Agent::insertAgentNeighbor with maxNeighbors = M: every agent within neighborDist) is the
            // in-range slots stably sorted by distSq in the order RVO2's KdTree visits them. <= 10 agents:
            // one leaf, so that order is the simulator's agents_ order = slot order, and lane sq builds the
            // lines of slots sq, sq+4, sq+8 and ranks them itself. > 10 agents: lane 0 of the quad runs the
            // KdTree build (which also re-permutes the persisted agents_ order) and query, the quad then
            // builds the lines in neighbour order.
            const int h = tid >> 2, sq = tid & 3;
            {
                // lanes of quads past the last human (h >= nh) stay in step for the KdTree walk (whole
                // waves) and skip the per-human work; their LDS reads stay inside the [H] arrays
                const bool hq = h < nh;
                const int elq = h / N, iq = h - elq * N, eb = elq * N;
                const uint32_t visq = sl.vis[h], dmq = sl.dm[h];
                const double px = HF(sl, H_PX, h), py = HF(sl, H_PY, h);
                const float rdummy = (float)(c.human_radius + 0.01 + c.orca_safety_space);
                const float X0 = (float)px, Y0 = (float)py;
                const float VX0 = (float)HF(sl, H_VX, h), VY0 = (float)HF(sl, H_VY, h);
                const float R0 = sl.orad[h];
                const float rangeSq = (float)c.orca_neighbor_dist * (float)c.orca_neighbor_dist;
                const float invTH = fdiv(1.0f, (float)c.orca_time_horizon);
                const float invTS = fdiv(1.0f, (float)dt);
                // preferred velocity: unit vector to the goal only if farther than 1 (orca.py:118-122)
                double gdx = HF(sl, H_GX, h) - px, gdy = HF(sl, H_GY, h) - py;
                const double speed = np_norm2(gdx, gdy);
                if (speed > 1.0) { gdx = ddiv(gdx, speed); gdy = ddiv(gdy, speed); }
                float4 *Lb = sl.lines + h * M, *Pb = sl.proj + h * M;
                bool vr_kd = false;   // kd-tree path: path violation, tested before Pb is reused
                int cnt = 0;
                uint32_t inm = 0;
                if constexpr (!KD) {
                  if (hq)
                    cnt = orca_lines_quad(
                        [&](int k, float &x, float &y, float &vx, float &vy, float &r) {
                            slot_agent(sl, c, eb, elq, EPB, N, iq, k, visq, dmq, rdummy, x, y, vx, vy, r);
                        },
                        M, sq, X0, Y0, VX0, VY0, R0, rangeSq, invTH, invTS, Lb);
                } else {
                    // (1) the quad loads the persisted KdTree order and fills, in that order, the agents'
                    //     positions (XYP[q] = agent perm[q]: self = 0, slot k = k + 1; kept in the projected-
                    //     lines space, unused until linearProgram3) and each slot's distSq
                    // (0) the path-violation test reads this human's velocity rectangle from Pb, which the
                    //     KdTree exchange reuses below
                    if (hq) vr_kd = path_vr_q(h, sq);   // the whole quad
                    wsync();
                    const int HS = P.NH;   // LDS stride of the per-human slot / KdTree order arrays
                    float2 *XYP = (float2 *)Pb;          // [A] (x, y) in KdTree order, then the exchange space
                    float *D = (float *)Pb + 2 * A;      // [M] distSq of each slot (beside XYP in Pb)
                    uint8_t *perm = sl.perm, *tpos = sl.ns;
                    const bool frz = (sl.rflag[elq] & CN_FLAG_ORCA_FROZEN) != 0;
                    const int gq = (e0 + elq) * N + iq;
                    for (int q = sq; q < A && hq; q += 4) {
                        const int a = frz ? S.o_perm[gq * A + q] : q;
                        perm[q * HS + h] = (uint8_t)a;
                        if (a == 0) { XYP[q] = make_float2(X0, Y0); continue; }
                        float x, y, vx, vy, r;
                        slot_agent(sl, c, eb, elq, EPB, N, iq, a - 1, visq, dmq, rdummy, x, y, vx, vy, r);
                        XYP[q] = make_float2(x, y);
                        const float dx = X0 - x, dy = Y0 - y;
                        D[a - 1] = dx * dx + dy * dy;
                        if (D[a - 1] < rangeSq) inm |= 1u << (a - 1);
                    }
                    inm = (uint32_t)quad_or((int)inm);
                    wsync();
                    STAMP_A(15);
                    // (2) KdTree build (buildAgentTreeRecursive, which re-permutes the persisted agents_ order)
                    //     fused with the query's depth-first walk (queryAgentTreeRecursive: closer child first,
                    //     ties -> right). 4 lanes per human (lane sub holds positions sub, sub+4, ..., sub+28
                    //     of the agent order), all 16 humans of a wave at once (8 lanes and two rounds of 8
                    //     humans before: the walk's critical path was twice as long). Every node is partitioned
                    //     once: Hoare's two-pointer loop swaps the i-th element >= split left of the cut with the
                    //     i-th element < split counted from the right end, which ballots and popcounts give
                    //     directly (exchange through the human's projected-lines space). The children's
                    //     bounding boxes (exact min / max over the quad) give both the visiting order and
                    //     their own split. Pruned subtrees hold no agent within range, so walking them inserts
                    //     nothing: the in-range agents' visiting order tpos is the order
                    //     Agent::insertAgentNeighbor sees. The explicit stack (<= A - 9 entries) lives in the
                    //     sorted-lines space, written only after the walk.
                    //     The body is predicated rather than branched per element: every element's LDS write goes
                    //     to its slot or to a dummy slot of the human (tpos row M, perm row A, the exchange entry
                    //     XD past the distances), every read comes from a valid address and is selected, and the
                    //     group masks are quad ORs of per-lane bit sets (lane sub holds positions sub + 4u).
                    {
                        const int lane = tid & 63, grp = lane >> 2, sub = lane & 3;
                        const int wbase = (tid >> 6) * 16;
                        const uint32_t sbit = 1u << sub;
                        auto gmask = [&](const bool (&pr)[8]) -> uint32_t {
                            uint32_t m = 0;
#pragma unroll
                            for (int u = 0; u < 8; ++u) m |= pr[u] ? (sbit << (4 * u)) : 0u;
                            return (uint32_t)quad_or((int)m);
                        };
                        if (wbase + grp < nh) {   // 16 humans per wave, 4 lanes each, all at once
                            const int hw = wbase + grp;
                            const int elw = hw / N, iw = hw - elw * N;
                            const int gw = (e0 + elw) * N + iw;
                            int4 *stk = (int4 *)(sl.lines + hw * M);
                            // exchange: (x, y) of 2 x (A / 2) entries in Pb, their agent ids in perm (read once
                            // above); a slot's in-range test is bit (agent - 1) of the quad's inm
                            float2 *xch = (float2 *)(sl.proj + hw * M);
                            const int XD = (2 * A + M + 1) / 2;   // dummy exchange entry (floats [2A + M, 4M) are free)
                            uint8_t *permw = perm + hw, *tposw = tpos + hw;
                            const float SX = (float)HF(sl, H_PX, hw), SY = (float)HF(sl, H_PY, hw);
                            float px[8], py[8];
                            int pa[8];
                            bool inr[8];   // element u is an agent within range (bit pa - 1 of inm)
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int q = sub + 4 * u;
                                const bool v = q < A;
                                const float2 t = xch[v ? q : XD];
                                px[u] = v ? t.x : 0.0f; py[u] = v ? t.y : 0.0f;
                                const int a = permw[(v ? q : A) * HS];
                                pa[u] = v ? a : 0;
                                inr[u] = pa[u] != 0 && ((inm >> ((pa[u] - 1) & 31)) & 1u);
                            }
                            auto red = [&](int b0, int e1, float &mnx, float &mxx, float &mny, float &mxy) {
                                float a0 = INFINITY, a1 = -INFINITY, c0 = INFINITY, c1 = -INFINITY;
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int q = sub + 4 * u;
                                    const bool in = q >= b0 && q < e1;
                                    a1 = in && a1 < px[u] ? px[u] : a1; a0 = in && px[u] < a0 ? px[u] : a0;
                                    c1 = in && c1 < py[u] ? py[u] : c1; c0 = in && py[u] < c0 ? py[u] : c0;
                                }
                                mnx = quad_min(a0); mxx = quad_max(a1); mny = quad_min(c0); mxy = quad_max(c1);
                            };
                            // z: bit 0 = split on x, bit 1 = all points coincide (zero-extent box)
                            auto entry = [&](int b0, int e1, float mnx, float mxx, float mny, float mxy) {
                                const bool vert = (mxx - mnx > mxy - mny);
                                const float split = vert ? 0.5f * (mxx + mnx) : 0.5f * (mxy + mny);
                                const int deg = (mnx == mxx && mny == mxy) ? 2 : 0;
                                return make_int4(b0, e1, (vert ? 1 : 0) | deg, __float_as_int(split));
                            };
                            int sp = 0, tc = 0;
#ifdef CN_STAMPS
                            int dbg_it = 0;
#endif
                            {
                                float mnx, mxx, mny, mxy;
                                red(0, A, mnx, mxx, mny, mxy);
                                stk[0] = entry(0, A, mnx, mxx, mny, mxy);
                                sp = 1;
                            }
                            while (sp > 0) {
#ifdef CN_STAMPS
                                ++dbg_it;
#endif
                                const int4 en = stk[--sp];
                                const int b0 = en.x, e1 = en.y;
                                const bool leaf = e1 - b0 <= 10;           // RVO_MAX_LEAF_SIZE
                                const bool deg = !leaf && (en.z & 2) != 0;
                                // insertions of a leaf (positions [b0, e1) in order) or of a node whose points all
                                // coincide (e.g. the dummies of unseen humans, all at (7, 7)): no split separates
                                // them, so each level peels its first element into a one-agent leaf, nothing moves,
                                // and the equal-distance children are visited right first: positions [e1-10, e1) in
                                // order (set 1), then e1-11 down to b0 (set 2). Internal nodes insert nothing.
                                const int lo1 = leaf ? b0 : (deg ? e1 - 10 : e1), hi2 = deg ? e1 - 10 : b0;
                                bool s1[8], s2[8];
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int q = sub + 4 * u;
                                    s1[u] = q >= lo1 && q < e1 && inr[u];
                                    s2[u] = q >= b0 && q < hi2 && inr[u];
                                }
                                const uint32_t b1 = gmask(s1), b2 = gmask(s2);
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int q = sub + 4 * u;
                                    const int r1 = tc + __popc(b1 & ((1u << q) - 1u));
                                    const int r2 = tc + __popc(b1) + __popc(b2 >> q >> 1);
                                    const bool w = s1[u] || s2[u];
                                    tposw[(w ? pa[u] - 1 : M) * HS] = (uint8_t)(s1[u] ? r1 : r2);
                                }
                                tc += __popc(b1) + __popc(b2);
                                if (leaf || deg) continue;
                                const float split = __int_as_float(en.w);
                                bool lt[8], pr[8], pL[8], pR[8];
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int q = sub + 4 * u;
                                    lt[u] = ((en.z & 1) ? px[u] : py[u]) < split;
                                    pr[u] = q >= b0 && q < e1 && lt[u];
                                }
                                const int mid = b0 + __popc(gmask(pr));
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    const int q = sub + 4 * u;
                                    const bool in = q >= b0 && q < e1;
                                    pL[u] = in && q < mid && !lt[u];
                                    pR[u] = in && q >= mid && lt[u];
                                }
                                const uint32_t Lm = gmask(pL), Rm = gmask(pR);
                                if (Lm) {   // Hoare's swaps: the i-th misplaced left element with the i-th right one
                                    const int nsw = __popc(Lm);
                                    int src[8];
#pragma unroll
                                    for (int u = 0; u < 8; ++u) {
                                        const int q = sub + 4 * u;
                                        const bool mv = pL[u] || pR[u];
                                        const int slot = pL[u] ? __popc(Lm & ((1u << q) - 1u)) : nsw + __popc(Rm >> q >> 1);
                                        const int ws = mv ? slot : XD;
                                        xch[ws] = make_float2(px[u], py[u]);
                                        permw[(mv ? slot : A) * HS] = (uint8_t)pa[u];
                                        src[u] = mv ? (pL[u] ? slot + nsw : slot - nsw) : -1;
                                    }
                                    wsync();
#pragma unroll
                                    for (int u = 0; u < 8; ++u) {
                                        const bool mv = src[u] >= 0;
                                        const float2 t = xch[mv ? src[u] : XD];
                                        const int a = permw[(mv ? src[u] : A) * HS];
                                        px[u] = mv ? t.x : px[u]; py[u] = mv ? t.y : py[u];
                                        pa[u] = mv ? a : pa[u];
                                        inr[u] = pa[u] != 0 && ((inm >> ((pa[u] - 1) & 31)) & 1u);
                                    }
                                    wsync();
                                }
                                const int left = mid == b0 ? mid + 1 : mid;
                                float l0, l1, l2, l3, r0, r1, r2, r3;
                                red(b0, left, l0, l1, l2, l3);
                                red(left, e1, r0, r1, r2, r3);
                                const int4 cl = entry(b0, left, l0, l1, l2, l3), cr = entry(left, e1, r0, r1, r2, r3);
                                const float dl = bbox_dist(SX, SY, l0, l1, l2, l3);
                                const float dr = bbox_dist(SX, SY, r0, r1, r2, r3);
                                // (all 4 lanes store the same entries) left visited first when strictly closer
                                stk[sp] = dl < dr ? cr : cl;
                                stk[sp + 1] = dl < dr ? cl : cr;
                                sp += 2;
                                wsync();
                            }
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int q = sub + 4 * u;
                                if (q < A) S.o_perm[gw * A + q] = (uint8_t)pa[u];
                            }
#ifdef CN_STAMPS
                            if (threadIdx.x == 0 && blockIdx.x < 4096) cn_stamp_a[blockIdx.x * CN_NSTAMP + 13] = dbg_it;
#endif
                        }
                    }
                    wsync();
                    STAMP_A(14);
                    if (hq) {
                    // (3) neighbour rank = stable order of (distSq, visiting order): each lane ranks its slots
                    //     sq, sq+4, ... in one pass over the in-range slots, then writes their lines
                    float myD[8];
                    int myT[8], rk[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int k = sq + 4 * u;
                        const bool in = k < M && ((inm >> k) & 1u);
                        myD[u] = in ? D[k] : 0.0f;
                        myT[u] = in ? tpos[k * HS + h] : 0;
                        rk[u] = 0;
                    }
                    for (uint32_t mq = inm; mq; mq &= mq - 1) {
                        const int q = __ffs(mq) - 1;
                        const float dq = D[q];
                        const int tq = tpos[q * HS + h];
#pragma unroll
                        for (int u = 0; u < 8; ++u) rk[u] += (dq < myD[u] || (dq == myD[u] && tq < myT[u])) ? 1 : 0;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int k = sq + 4 * u;
                        if (k < M && ((inm >> k) & 1u)) {
                            float ox, oy, ovx, ovy, orr;
                            slot_agent(sl, c, eb, elq, EPB, N, iq, k, visq, dmq, rdummy, ox, oy, ovx, ovy, orr);
                            Lb[rk[u]] = orca_line(X0, Y0, VX0, VY0, R0, ox, oy, ovx, ovy, orr, invTH, invTS);
                        }
                    }
                    }
                    cnt = __popc(inm);
                }
                wsync();
                STAMP_A(7);
                if constexpr (!KD) {   // <= 12 lines: register-resident linear programs
                    uint32_t *l3b = (uint32_t *)(smem + P.o_l3b);
                    float2 *l3r = (float2 *)(smem + P.o_l3r);
                    uint8_t *l3k = (uint8_t *)(smem + P.o_l3k);
                    float rx = 0.0f, ry = 0.0f;
                    int fail_at = 0;
                    float4 R[3];
#pragma unroll
                    for (int u = 0; u < 3; ++u)
                        R[u] = hq && sq + 4 * u < cnt ? Lb[sq + 4 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
                    if (hq) {
                        fail_at = lp2_r<3>(R, cnt, sl.vmax[h], (float)gdx, (float)gdy, sq, rx, ry);
                    }
                    STAMP_A(8);
                    // linearProgram3 of the workgroup's infeasible humans: every sub-problem their loops may
                    // visit, solved by all quads (lp3_tasks), then each human's quad replays its loop
                    const bool l3 = hq && fail_at < cnt;
                    const int l3e = min(cnt, fail_at + CN_LP3_W);
                    if (sq == 0) l3b[h] = l3 ? (uint32_t)(fail_at | (l3e << 8)) : 0u;
                    // the calc_reward ladder here, while the waves wait for the slowest linearProgram2 at this
                    // barrier (after the linear programs it was the last item of its wave's phase 2: stamps of the
                    // driver's window put it at ~5 k of the slowest workgroups' ~63 k phase-2 cycles). It reads only
                    // phase-1 results and writes no value the linear programs or human_post read. Not with norm
                    // zones: their separating-axis tests make the ladder longer than that slack (C5 -1 %, A/B)
                    if (!c.norm_zones) {
                        if (rl) ladder();
                        ladder_done = true;
                    }
                    __syncthreads();
#ifdef CN_STAMPS
                    const unsigned long long tl3 = clock64();
#endif
                    lp3_tasks<3>(sl.lines, M, sl.vmax, l3b, l3r, l3k, tid);
                    __syncthreads();
                    int l3vis = 0;
                    if (l3) l3vis = lp3_replay<3>(R, Lb, cnt, fail_at, l3e, sl.vmax[h], sq, l3r + h * 12, l3k + h * 12, rx, ry);
#ifdef CN_STAMPS
                    if (tid == 0 && (unsigned)sb < 4096) cn_stamp_a[sb * CN_NSTAMP + 23] = clock64() - tl3;
#ifdef CN_STAMPS_LP3   // (two device-wide atomics per infeasible human: they slowed the stamps build by ~60 %)
                    if (l3 && sq == 0) {   // sub-problems solved / visited by RVO2's loop
                        atomicAdd(&cn_lp3_cnt[0], (unsigned long long)(l3e - fail_at));
                        atomicAdd(&cn_lp3_cnt[1], (unsigned long long)l3vis);
                    }
#endif
#else
                    (void)l3vis;
#endif
                    STAMP_A(9);
                    if (hq) {
                        const bool vr = path_vr_q(h, sq);   // the whole quad
                        if (sq == 0) human_post(h, (double)rx, (double)ry, vr);
                    }
                } else if (hq) {
                    float rx, ry;
                    const float vmq = sl.vmax[h];
                    const int fail_at = lp2_q(Lb, cnt, vmq, (float)gdx, (float)gdy, sq, rx, ry);
                    STAMP_A(8);
                    if (fail_at < cnt) lp3_q(Lb, Pb, cnt, fail_at, vmq, sq, rx, ry);
                    STAMP_A(9);
                    wsync();   // the quad's last reads of Pb (linearProgram3) before human_post stages into it
                    if (sq == 0) human_post(h, (double)rx, (double)ry, vr_kd);
                }
            }
        } else if (hl) {
            const int eb = el * N;
            const double px = HF(sl, H_PX, tid), py = HF(sl, H_PY, tid);
            const double vx0 = HF(sl, H_VX, tid), vy0 = HF(sl, H_VY, tid);
            const double rad = HF(sl, H_R, tid), vpref = HF(sl, H_VP, tid);
            // SOCIAL_FORCE.predict (social_force.py:11-66)
            const double dx = HF(sl, H_GX, tid) - px, dy = HF(sl, H_GY, tid) - py;
            const double dist = dsqrt(dx * dx + dy * dy);
            const double dvx = ddiv(dx, dist) * vpref, dvy = ddiv(dy, dist) * vpref;
            const double cdx = c.sf_KI * (dvx - vx0), cdy = c.sf_KI * (dvy - vy0);
            double ix = 0.0, iy = 0.0;
            for (int k = 0; k < M; ++k) {
                double ox, oy, orr;
                const bool v = (vis >> k) & 1u;
                if (k < N - 1) {
                    const int j = eb + (k < i ? k : k + 1);
                    ox = v ? HF(sl, H_PX, j) : CN_DUMMY_POS; oy = v ? HF(sl, H_PY, j) : CN_DUMMY_POS;
                    orr = v ? HF(sl, H_R, j) : c.human_radius;
                } else {
                    ox = v ? RF(sl, R_PX, el, EPB) : CN_DUMMY_POS; oy = v ? RF(sl, R_PY, el, EPB) : CN_DUMMY_POS;
                    orr = v ? RF(sl, R_RAD, el, EPB) : c.robot_radius;
                }
                const double ddx = px - ox, ddy = py - oy;
                const double d = dsqrt(ddx * ddx + ddy * ddy);
                const double ex = exp(ddiv(rad + orr - d, c.sf_B));
                ix += c.sf_A * ex * ddiv(ddx, d);
                iy += c.sf_A * ex * ddiv(ddy, d);
            }
            const double tx = (cdx + ix) * dt, ty = (cdy + iy) * dt;
            const double nx = vx0 + tx, ny = vy0 + ty;
            const double n = np_norm2(nx, ny);
            if (n > vpref) { nvx = ddiv(nx, n) * vpref; nvy = ddiv(ny, n) * vpref; }
            else { nvx = nx; nvy = ny; }
            human_post(tid, nvx, nvy, path_vr(tid));
        }
        STAMP_T(21, 64);
        if (rl && !ladder_done) ladder();
        STAMP_T(20, 64);
    }
    __syncthreads();
    STAMP_A(3);

    // ---- human state / observation stores (human lanes, consecutive) beside the robot kinematics, state
    //      and observation stores and RNG needs (env lanes) ---------------------------------------------
    if (hl) {
        S.h_px[gh] = sl.npx[tid]; S.h_py[gh] = sl.npy[tid];
        S.h_vx[gh] = hst_ref(tid, 0); S.h_vy[gh] = hst_ref(tid, 1);
        const double bpx = hst_ref(tid, 2), bpy = hst_ref(tid, 3);
        S.b_px[gh] = bpx; S.b_py[gh] = bpy; S.b_vx[gh] = hst_ref(tid, 4); S.b_vy[gh] = hst_ref(tid, 5);
        S.b_r[gh] = hst_ref(tid, 6);
        const int64_t oh = orow(ov, e0 + el) * ov.NS + i;
        g.spatial[oh * 2] = (float)(bpx - RF(sl, R_NX, el, EPB));
        g.spatial[oh * 2 + 1] = (float)(bpy - RF(sl, R_NY, el, EPB));
    }
    if (rl) {
        // robot kinematics (agent.py:198-212): the post-move state computed in phase 1
        const uint32_t flags = sl.rflag[re];
        const float a0 = sl.act[re], a1 = sl.act[EPB + re];
        if (holo) { RF(sl, R_VX, re, EPB) = a0; RF(sl, R_VY, re, EPB) = a1; }
        else {
            RF(sl, R_TH, re, EPB) = RF(sl, R_NTH, re, EPB);
            RF(sl, R_VX, re, EPB) = RF(sl, R_CVX, re, EPB); RF(sl, R_VY, re, EPB) = RF(sl, R_CVY, re, EPB);
        }
        sl.rflag[re] = flags | CN_FLAG_ROBOT_F32;
        const double nx = RF(sl, R_NX, re, EPB), ny = RF(sl, R_NY, re, EPB);
        S.r_px[ge] = nx; S.r_py[ge] = ny;
        S.r_vx[ge] = RF(sl, R_VX, re, EPB); S.r_vy[ge] = RF(sl, R_VY, re, EPB);
        S.r_theta[ge] = RF(sl, R_TH, re, EPB);
        S.r_dv[ge] = RF(sl, R_DV, re, EPB);
        S.potential[ge] = RF(sl, R_POT, re, EPB);
        const double gt = RF(sl, R_GT, re, EPB);
        S.gtime[ge] = gt;
        uint32_t flags2 = sl.rflag[re];
        if (orca) flags2 |= CN_FLAG_ORCA_FROZEN;
        bool endg = false, nan = false;
        int vr_viol = 0;
        const int kv = (int)sl.rflag[2 * EPB + re];
        for (int k = 0; k < N; ++k) {
            const uint32_t f = sl.eg[re * N + k];
            endg |= (f & LF_ENDGOAL) != 0;
            nan |= (f & 0x80000000u) != 0;
            vr_viol += (k < kv && (f & LF_VR)) ? 1 : 0;
        }
        if (g.info) g.info[orow(ov, ge) * CN_INFO_K + CN_INFO_PATH_VIOLATION] = (float)vr_viol;
        if (nan) flags2 |= CN_FLAG_NAN;
        S.flags[ge] = flags2;
        const int64_t oe = orow(ov, ge);
        float *rn = g.robot_node + oe * 7;
        rn[0] = (float)nx; rn[1] = (float)ny; rn[2] = (float)RF(sl, R_RAD, re, EPB);
        rn[3] = (float)RF(sl, R_GX, re, EPB); rn[4] = (float)RF(sl, R_GY, re, EPB);
        rn[5] = (float)RF(sl, R_VP, re, EPB); rn[6] = (float)RF(sl, R_TH, re, EPB);
        g.temporal[oe * 2] = (float)RF(sl, R_VX, re, EPB);
        g.temporal[oe * 2 + 1] = (float)RF(sl, R_VY, re, EPB);
        for (int k = N; k < ov.NS; ++k) {   // padding slots of a mixed engine (never-seen humans)
            g.spatial[(oe * ov.NS + k) * 2] = (float)(CN_PAD_POS - nx);
            g.spatial[(oe * ov.NS + k) * 2 + 1] = (float)(CN_PAD_POS - ny);
        }
        // random numbers needed? (crowd_sim_dict.py:260-269, shmem_vec_env.py:166-167)
        const bool done = sl.rflag[EPB + re] != 0;
        const bool rgoal = c.random_goal_changing && np_mod(gt, 5.0) == 0.0;
        const bool egoal = c.end_goal_changing && endg;
        sl.rflag[EPB + re] = (done ? 1u : 0u) | (rgoal ? 2u : 0u) | (egoal ? 4u : 0u);
    }
    if ((tid >> 6) == 1) {   // the env lanes' wave: one mask of the envs with RNG work, for phase 5's item split
        const uint64_t bm = __ballot(rl && (sl.rflag[EPB + re] & 7u) != 0u);
        if (tid == 64) { sl.rflag[3 * EPB] = (uint32_t)bm; sl.rflag[3 * EPB + 1] = (uint32_t)(bm >> 32); }
    }
    __syncthreads();
    STAMP_A(4);
    STAMP_A(5);

    // ---- phase 5: this workgroup's RNG work, one wave per env needing it --------------------------
    // Done envs auto-reset (VecEnv worker, shmem_vec_env.py:164-168) from the pending spawn drawn by an
    // earlier launch (reset_env: two slots per env, consumed only when an earlier launch completed the entry);
    // after cn_reset / cn_set_state, while this launch's spawn waves draw every env's entries, they draw inline.
    {
        // the wave index is wave-uniform: readfirstlane keeps it (and every LDS pointer derived from it) in
        // SGPRs -- as a VGPR value the RNG block's preheader spilled it to scratch (HBM writes every launch)
        const int nw = P.rng_waves, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        char *wb = smem + P.o_lines + (w < nw ? w : 0) * P.rng_stride;   // over the ORCA scratch, dead after phase 2
        WRng m;
        m.w = (uint32_t *)wb; m.off = 0; m.lane = lane; m.phx = PHX; m.edbg = -1;
        m.grid = P.rng_stride > CN_PEND_LDS ? wb + CN_PEND_LDS : nullptr;
        m.sl = (double *)(wb + 2 * CN_MT_N * 4 + 7 * 32 * 8);
        double *hb = (double *)(wb + 2 * CN_MT_N * 4);
        // the RNG waves' goal loops end most of the slowest workgroups (kd-tree path): issue priority over
        // the other workgroups' waves on their SIMD (C3 460.3 / 461.6 -> 456.8 / 456.4 us per launch, A/B)
        if ((KD || CN_RNG_PRIO_ALL) && w < nw) __builtin_amdgcn_s_setprio(3);
        // waves without an env to serve skip the block entirely: the loop's preheader (values the
        // compiler hoists out of the RNG work, and their spill stores) then runs only where it is needed.
        // The envs with work, in env order, go round-robin to the RNG waves: this wave's share from the mask
        // wave 1 wrote (scalar bit loop, one LDS read instead of a dependent chain over the envs' flags)
        const uint64_t rm = ((uint64_t)__builtin_amdgcn_readfirstlane(sl.rflag[3 * EPB + 1]) << 32) |
                            (uint64_t)__builtin_amdgcn_readfirstlane(sl.rflag[3 * EPB]);
        uint64_t mym = 0;
        {
            int jj = 0;
            for (uint64_t mm = rm; mm; mm &= mm - 1, ++jj)
                if (jj % nw == w) mym |= mm & (~mm + 1);
        }
        STAMP_T(22, 0);
        if (mym) {
        for (uint64_t mm = mym; mm; mm &= mm - 1) {
            const int q = __builtin_ctzll(mm);
            // the kernel arguments through pointers the compiler cannot see across iterations: their loads stay at
            // the uses in this body instead of a preheader that reloaded ~30 of them one by one and parked ~250
            // SGPR values in VGPR lanes before the first item (~4 k cycles on the slowest workgroups)
            // (read from the kernarg segment itself: taking the parameters' addresses would copy them to scratch;
            // by-value arguments in order at their natural alignment, StepArgs at 0, cn_config after it)
            typedef const __attribute__((address_space(4))) char *KArgs;
            typedef const __attribute__((address_space(4))) StepArgs *GArgs;
            typedef const __attribute__((address_space(4))) cn_config *CArgs;
            KArgs ks = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
            asm volatile("" : "+s"(ks));
            GArgs gq = (GArgs)ks;
            CArgs cq = (CArgs)(ks + ((sizeof(StepArgs) + alignof(cn_config) - 1) & ~(alignof(cn_config) - 1)));
            const StepArgs &G = *(const StepArgs *)gq;
            const cn_config &C = *(const cn_config *)cq;
            ResetOut o;
            o.s = G.s; o.robot_node = G.robot_node; o.temporal = G.temporal; o.spatial = G.spatial;
            o.case_size = G.case_size; o.ov = ov;
            const uint32_t need = sl.rflag[EPB + q] & 7u;
            const int64_t e = e0 + q;
            STAMP_B(e, 0);
            Env1 en;
            if (need & 1u) {
                en.hpx = hb; en.hpy = hb + 32; en.hgx = hb + 64; en.hgy = hb + 96; en.hr = hb + 128; en.hvp = hb + 160;
                en.hth = hb + 192;
                // (pend.all, pend.launch_id, pcount_w and plist_w from the kernel's own copy g: graph mode (DEVSEQ)
                // rewrote them at the top from the device-side step counter; the kernarg segment holds the values of
                // the captured launch)
                const bool may = g.pend.all != PEND_BOTH;   // ready unless this launch redraws both
                reset_env<KD, (KD || CN_QUAD_PARK) && CN_SLOT_FENCE>(o, G.pend.P, C, G.E, e, G.pend.counter_offset, may,
                                                                     g.pend.launch_id, m, en, G.pend.stats + 7);
                if (lane == 0) {   // each env resets at most once per launch: k < E (guarded all the same)
                    // the entry carries the counters this reset just wrote (its own stores, read back), so the
                    // next launch's spawn wave keys the spawn after next from them, never from a state that a
                    // later reset of the same env may be rewriting while it reads
                    const int64_t ccn = G.s.case_counter[e];
                    const int32_t rcn = G.s.reset_count[e];
                    const uint32_t k = atomicAdd(g.pcount_w, 1u);
                    if (k < (uint32_t)G.E) {
                        uint32_t *q = g.plist_w + 4 * k;
                        q[0] = (uint32_t)e; q[1] = (uint32_t)rcn;
                        q[2] = (uint32_t)(uint64_t)ccn; q[3] = (uint32_t)((uint64_t)ccn >> 32);
                    }
                }
                STAMP_B(e, 5);
            } else {
                const int b = q * N;
                en.hpx = sl.npx + b; en.hpy = sl.npy + b; en.hgx = &HF(sl, H_GX, b);
                en.hgy = &HF(sl, H_GY, b); en.hr = &HF(sl, H_R, b); en.hvp = &HF(sl, H_VP, b); en.hth = &HF(sl, H_TH, b);
                en.rpx = RF(sl, R_NX, q, EPB); en.rpy = RF(sl, R_NY, q, EPB);
                en.rgx = RF(sl, R_GX, q, EPB); en.rgy = RF(sl, R_GY, q, EPB); en.rr = RF(sl, R_RAD, q, EPB);
                // update_human_goal checks every human AFTER the random changes (a new random goal may
                // land within reach of its own human), so it runs whenever end goal changing is on
                m.edbg = e;
                goal_changes<KD>(C, G.s, e, en, m, (need & 2u) != 0, C.end_goal_changing != 0, hb);
            }
        }
        }
        // back to normal priority for the epilogue (graph mode's finish barrier, stamps)
        if ((KD || CN_RNG_PRIO_ALL) && w < nw) __builtin_amdgcn_s_setprio(0);
    }
#ifdef CN_STAMPS
    __syncthreads();
    STAMP_A(6);
#endif
    finish();
}

// cn_reset: CrowdSimDict.reset of every env, one wave (single-wave workgroup) per env
__global__ void __launch_bounds__(64) cn_reset_kernel(RngArgs g, cn_config c)
{
    __shared__ uint32_t mtw[2 * CN_MT_N];
    __shared__ double hbuf[7][32];
    __shared__ double slots[6 * 64];
    __shared__ __attribute__((aligned(16))) char gridbuf[CN_GRID_LDS];
    const int lane = threadIdx.x;
    for (int64_t e = blockIdx.x; e < g.E; e += gridDim.x) {
        Env1 en;
        en.hpx = hbuf[0]; en.hpy = hbuf[1]; en.hgx = hbuf[2]; en.hgy = hbuf[3]; en.hr = hbuf[4]; en.hvp = hbuf[5];
        en.hth = hbuf[6];
        WRng m;
        m.w = mtw; m.off = 0; m.lane = lane; m.sl = slots; m.phx = c.rng_mode == CN_RNG_PHILOX; m.edbg = -1;
        m.grid = gridbuf;
        reset_env<true>(g.o, g.pend, c, g.E, e, g.counter_offset, true, 0u, m, en);
        // and the spawns of the env's next two resets (both pending slots), so that the first step launches
        // find every spawn they need drawn (PEND_FRESH): keys = the counters the reset just wrote, advanced
        int64_t cc1 = g.o.s.case_counter[e];
        int32_t rc1 = g.o.s.reset_count[e];
        for (int k = 0; k < (g.draw_next ? 2 : 0); ++k) {
            double rth;
            uint32_t ovf;
            int sc;
            spawn_env<true>(c, c.env_offset + orow(g.o.ov, e), cc1, rc1, g.counter_offset, m, en, rth, ovf, sc);
            const bool in1 = !m.phx && m.p > CN_MT_N;
            write_pending<true>(g.pend, c, g.E, e, en, rth, sc, ovf, m.blk(in1 ? 1 : 0), in1 ? m.p - CN_MT_N : m.p, cc1,
                                rc1, lane, CN_OK_RESET, c.human_num);
            wsync();
            cc1 = (cc1 + c.nenv) % g.o.case_size;   // write_reset's counter update
            rc1 += 1;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// fused DSRNN edge-feature assembly (srnn_model.py:160-161, 210-211, 466)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cn_edge_features_kernel(int64_t E, int N, const float *__restrict__ robot_node,
                                                               const float *__restrict__ temporal,
                                                               const float *__restrict__ spatial,
                                                               const float *__restrict__ Wt, const float *__restrict__ bt,
                                                               const float *__restrict__ Ws, const float *__restrict__ bs,
                                                               const float *__restrict__ Wr, const float *__restrict__ br,
                                                               const float *__restrict__ Wn, const float *__restrict__ bn,
                                                               float *__restrict__ t_out, float *__restrict__ s_out,
                                                               float *__restrict__ n_out)
{
    // one thread per (row, 4 output features); rows = E temporal + E*N spatial + E node
    const int64_t rows = E * (N + 2);
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t row = idx >> 4;
    const int q = (int)(idx & 15) * 4;
    if (row >= rows) return;
    float o[4];
    if (row < E) {  // temporal edge: relu(Wt x + bt), x = robot velocity
        const float x0 = temporal[row * 2], x1 = temporal[row * 2 + 1];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = fmaxf(__fmaf_rn(Wt[(q + k) * 2 + 1], x1, __fmaf_rn(Wt[(q + k) * 2], x0, bt[q + k])), 0.0f);
        *(float4 *)(t_out + row * 64 + q) = make_float4(o[0], o[1], o[2], o[3]);
    } else if (row < E + E * N) {  // spatial edges
        const int64_t r = row - E;
        const float x0 = spatial[r * 2], x1 = spatial[r * 2 + 1];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = fmaxf(__fmaf_rn(Ws[(q + k) * 2 + 1], x1, __fmaf_rn(Ws[(q + k) * 2], x0, bs[q + k])), 0.0f);
        *(float4 *)(s_out + r * 64 + q) = make_float4(o[0], o[1], o[2], o[3]);
    } else {  // robot node: relu(Wn (Wr x + br) + bn)
        const int64_t r = row - E - E * N;
        float h[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float a = br[j];
#pragma unroll
            for (int k = 0; k < 7; ++k) a = __fmaf_rn(Wr[j * 7 + k], robot_node[r * 7 + k], a);
            h[j] = a;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float a = bn[q + k];
#pragma unroll
            for (int j = 0; j < 3; ++j) a = __fmaf_rn(Wn[(q + k) * 3 + j], h[j], a);
            o[k] = fmaxf(a, 0.0f);
        }
        *(float4 *)(n_out + r * 64 + q) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// LiDAR observation of the ConvGRU policy: CrowdSimDict.generate_ob's 'convgru' branch
// (crowd_sim_dict.py:96-101) over LidarSensor.sensor_spin (crowd_sim/envs/utils/lidarv2.py:398-427).
// As shipped, the reference computes the scan only inside reset() (crowd_sim_dict.py:174-191, robot
// heading atan2(0, 0) = 0, and only the LAST human is parsed: the append sits outside the loop), AFTER the
// reset observation was built (:166), and step() never refreshes lidar_rel_dist. So the observation that
// reset() returns carries the previous scan (zeros before the first), and every step of the episode
// carries the scan taken at its reset. One 64-lane wave per env, three beams per lane, float64 as the
// reference; the observation row is
//   [clip(robot (px, py, r, gx, gy, v_pref, theta) / max_range, 0, 1), |1 - clip(dist / max_range, 0, 1)|].
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double np_rem(double a, double b)   // numpy float remainder (sign of divisor)
{
    double m = fmod(a, b);
    if (m != 0.0) { if ((b < 0) != (m < 0)) m += b; }
    else m = copysign(0.0, b);
    return m;
}
__device__ __forceinline__ double rescale_angle(double t) { return np_rem(t + 2.0 * CN_PI, 2.0 * CN_PI); }

__device__ __forceinline__ int seg_orient(double px, double py, double qx, double qy, double rx, double ry)
{   // get_intersect.py:25-37
    const double v = ((qy - py) * (rx - qx)) - ((qx - px) * (ry - qy));
    return v > 0 ? 1 : (v < 0 ? 2 : 0);
}
__device__ __forceinline__ bool on_seg(double px, double py, double qx, double qy, double rx, double ry)
{   // get_intersect.py:12-21
    return qx <= fmax(px, rx) && qx >= fmin(px, rx) && qy <= fmax(py, ry) && qy >= fmin(py, ry);
}

__global__ void __launch_bounds__(256) cn_lidar_obs_kernel(cn_state_ptrs S, int E, int N, double half_world,
                                                           const uint8_t *__restrict__ reset_mask, int enable,
                                                           int beams, double max_range, double robot_r,
                                                           float *__restrict__ lidar, float *__restrict__ obs)
{
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= E) return;
    const int D = 7 + beams;
    float *o = obs + (int64_t)e * D;
    if (lane < 7) {
        double v;
        switch (lane) {
        case 0: v = S.r_px[e]; break;
        case 1: v = S.r_py[e]; break;
        case 2: v = S.r_radius[e]; break;
        case 3: v = S.r_gx[e]; break;
        case 4: v = S.r_gy[e]; break;
        case 5: v = S.r_vpref[e]; break;
        default: v = S.r_theta[e]; break;
        }
        v = v / max_range;
        v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);   // np.clip
        o[lane] = (float)v;
    }
    float *L = lidar + (int64_t)e * beams;
    const bool fresh = reset_mask == nullptr || reset_mask[e] != 0;
    if (fresh) {
        if (enable) {
            const double sx = S.r_px[e], sy = S.r_py[e];
            const int hl = e * N + (N - 1);                 // the last human only (see above)
            const double hx = S.h_px[hl], hy = S.h_py[hl], hr = S.h_r[hl];
            // get_valid_angles (lidarv2.py:17-52) for the one obstacle, sorted (min, max)
            const double rlx = hx - sx, rly = hy - sy;
            const double hd = rescale_angle(atan2(rly, rlx));
            const double ddx = hr * sin(hd), ddy = hr * cos(hd);
            const double m0 = rescale_angle(atan2(rly - ddy, rlx + ddx));
            const double m1 = rescale_angle(atan2(rly + ddy, rlx - ddx));
            const double lo0 = m0 < m1 ? m0 : m1, up0 = m0 < m1 ? m1 : m0;
            const double bstep = (2.0 * CN_PI) / (double)(beams - 1);   // np.linspace(0, 2 pi, beams)
            const int npts = 500;                                         // max_range / 0.01 samples (+ endpoint)
            const double sstep = max_range / (double)(npts - 1);
            for (int b = lane; b < beams; b += 64) {
                const double th0 = (b == beams - 1) ? 2.0 * CN_PI : (double)b * bstep;
                const double th = rescale_angle(th0 + 0.0);
                // get_valid_angle_idx (lidarv2.py:55-75) mutates the caller's (min, max) arrays in place and
                // they are reused for every beam: replay the mutation sequence up to this beam
                double lo = lo0, up = up0, tt = th;
                for (int q = 0; q <= b; ++q) {
                    const bool wide = up - lo >= CN_PI;
                    double tq = th;
                    if (wide) { const double nu = up - 2.0 * CN_PI; up = lo; lo = nu; tq -= 2.0 * CN_PI; }
                    if (q == b) tt = tq;
                }
                const bool valid = np_rem(tt - lo, 2.0 * CN_PI) < np_rem(up - lo, 2.0 * CN_PI);
                const double c = cos(th), sn = sin(th);
                double ex = c * max_range + sx, ey = sn * max_range + sy;   // beam_end
                bool hit = false;
                if (valid) {   // check_dist_collision_polygon (lidarv2.py:164-198): first sample inside the disc
                    const double wx = hx - sx, wy = hy - sy;
                    const double proj = wx * c + wy * sn, perp2 = wx * wx + wy * wy - proj * proj;
                    const double r2 = hr * hr;
                    if (perp2 <= r2 * (1.0 + 1e-9) + 1e-12) {
                        const double hw = sqrt(fmax(r2 - perp2, 0.0));
                        const double s_in = proj - hw, s_out = proj + hw;
                        int k0 = (int)floor(s_in / sstep) - 2, k1 = (int)ceil(s_out / sstep) + 2;
                        k0 = k0 < 0 ? 0 : k0;
                        k1 = k1 > npts - 1 ? npts - 1 : k1;
                        for (int k = k0; k <= k1 && !hit; ++k) {
                            const double sk = (k == npts - 1) ? max_range : (double)k * sstep;
                            const double bx = c * sk + sx, by = sn * sk + sy;
                            const double ax = hx - bx, ay = hy - by;
                            if (sqrt(ax * ax + ay * ay) < hr) { ex = bx; ey = by; hit = true; }
                        }
                    }
                }
                if (!hit) {    // walls (lidarv2.py:261-275): first intersecting wall, kept if within range
                    const double t = half_world;
                    const double wxs[5] = {-t, t, t, -t, -t}, wys[5] = {-t, -t, t, t, -t};
                    const double p1x = sx, p1y = sy, q1x = ex, q1y = ey;
                    for (int j = 0; j < 4; ++j) {
                        const double p2x = wxs[j], p2y = wys[j], q2x = wxs[j + 1], q2y = wys[j + 1];
                        const int o1 = seg_orient(p1x, p1y, q1x, q1y, p2x, p2y);
                        const int o2 = seg_orient(p1x, p1y, q1x, q1y, q2x, q2y);
                        const int o3 = seg_orient(p2x, p2y, q2x, q2y, p1x, p1y);
                        const int o4 = seg_orient(p2x, p2y, q2x, q2y, q1x, q1y);
                        const bool inter = (o1 != o2 && o3 != o4) || (o1 == 0 && on_seg(p1x, p1y, p2x, p2y, q1x, q1y)) ||
                                           (o2 == 0 && on_seg(p1x, p1y, q2x, q2y, q1x, q1y)) ||
                                           (o3 == 0 && on_seg(p2x, p2y, p1x, p1y, q2x, q2y)) ||
                                           (o4 == 0 && on_seg(p2x, p2y, q1x, q1y, q2x, q2y));
                        if (!inter) continue;
                        // line_intersection (get_intersect.py:72-89)
                        const double xd0 = p1x - q1x, xd1 = p2x - q2x, yd0 = p1y - q1y, yd1 = p2y - q2y;
                        const double div = xd0 * yd1 - xd1 * yd0;
                        if (div != 0.0) {
                            const double d0 = p1x * q1y - p1y * q1x, d1 = p2x * q2y - p2y * q2x;
                            const double ix = (d0 * xd1 - d1 * xd0) / div, iy = (d0 * yd1 - d1 * yd0) / div;
                            if (np_norm2(ix - sx, iy - sy) <= max_range) { ex = ix; ey = iy; }
                        }
                        break;
                    }
                }
                if (np_norm2(ex - sx, ey - sy) < robot_r) {   // beams cannot end inside the robot
                    ex = sx + robot_r * cos(th);
                    ey = sy + robot_r * sin(th);
                }
                const double rx = ex - sx, ry = ey - sy;
                double rd = sqrt(rx * rx + ry * ry) / max_range;
                rd = rd < 0.0 ? 0.0 : (rd > 1.0 ? 1.0 : rd);
                o[7 + b] = L[b];                 // the reset observation keeps the previous scan
                L[b] = (float)fabs(1.0 - rd);
            }
            return;
        }
        for (int b = lane; b < beams; b += 64) { o[7 + b] = L[b]; L[b] = 0.0f; }
        return;
    }
    for (int b = lane; b < beams; b += 64) o[7 + b] = L[b];
}

struct cn_engine {
    cn_config c;
    int device;
    int E, N, A;
    StepPlan plan;
    void *state;
    int64_t state_bytes;
    cn_state_ptrs s;
    uint32_t *work;       // [E]
    uint32_t *work_count; // [16]: [2..4] spawn-list counters (triple buffered), [5..7] parked-spawn counters,
                          // [8..11] spawn statistics (PendLaunch::stats), [15] inline reset draws
    uint32_t *plist;      // [3][E + 64][4] envs whose spawn after next kernel A draws, with their counters
    uint32_t *rlist;      // [3][2E][4] spawns parked by a launch (resumed by the next); counters work_count[5..7]
    int devseq;           // graph mode (cn_set_graph_mode): the step sequence lives in work_count[12..14]
    uint32_t ctl_host[4];
    int pend_all;         // next kernel A's pending mode: PEND_BOTH (after cn_set_state) or PEND_FRESH (after cn_reset)
    uint64_t nstep;
    long long spawn_budget;   // clock cycles a spawning wave works per launch before parking (0: never)
    void *pend_mem;       // pending next-episode spawns (PendPtrs)
    PendPtrs pend;
    int pend_blocks;      // spare workgroups of kernel A running spawn waves
    int pend_waves;       // spawning waves per spare workgroup
    int a_lds;            // kernel A dynamic LDS: max(step plan, spawn waves)
    int64_t case_size, counter_offset;
    int rng_grid;
    // kernel timing (cn_profile)
    int prof_on, prof_cap, prof_n;
    hipEvent_t *ev;  // [2]: before the first, after the last launch of the window
    // output view (a group of a mixed engine: its envs' rows in the caller's buffers and the padded human
    // stride; identity / N for a plain engine)
    int32_t *rows;   // device [E] or nullptr
    int NS;
    // mixed engine (cn_create_mixed): the groups, each a plain engine over its envs; E = all envs,
    // N = NS = the largest human count
    int ngroups;
    cn_engine **grp;
    hipStream_t *gstream;   // [ngroups]: group k > 0 steps on gstream[k] (forked from / joined to the caller's)
    hipEvent_t *gev;        // [ngroups + 1]: fork, then one join event per forked group
};

// unit-circle table of GEOS's 64-gon point buffer (norm zones), per device; every entry point whose
// kernels read it (cn_create, cn_debug_disc_quad) uploads it first
static hipError_t circ_table_init()
{
    double cs[64], sn[64];
    for (int k = 0; k < 64; ++k) { const double a = -(k * (CN_PI / 2 / 16)); cs[k] = cos(a); sn[k] = sin(a); }
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_circ_cos), cs, sizeof cs);
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_circ_sin), sn, sizeof sn);
    return e;
}

static thread_local char g_err[512];
static int set_err(int code, const char *fmt, const char *a = "")
{
    snprintf(g_err, sizeof g_err, fmt, a);
    return code;
}
int cn_set_error(int code, const char *msg) { return set_err(code, "%s", msg); }   // for cn_gru.hip
#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t _e = (x);                                                            \
        if (_e != hipSuccess) return set_err(CN_EHIP, "HIP error: %s", hipGetErrorString(_e)); \
    } while (0)

__global__ void __launch_bounds__(64) cn_disc_quad_kernel(int64_t n, int mode, const double *px, const double *py,
                                                          const double *r, const double *qx, const double *qy,
                                                          int32_t *out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 2)   // the robot's norm-zone penalty predicate: qx[i] = {vx, f32, ...}, qy[i] = {vy, lhs, ...}
        out[i] = robot_norm_zone_violation(px[i], py[i], qx[4 * i], qy[4 * i], r[i], qx[4 * i + 1] != 0.0,
                                           (int)qy[4 * i + 1]);
    else
        out[i] = mode ? disc_quad_sat(px[i], py[i], r[i], qx + 4 * i, qy + 4 * i)
                      : disc_quad_intersect(px[i], py[i], r[i], qx + 4 * i, qy + 4 * i);
}

// cn_debug_copy64: one wave per segment of `seg` doubles
__global__ void __launch_bounds__(64) cn_copy64_kernel(int64_t n, int seg, const double *__restrict__ src,
                                                       double *__restrict__ dst)
{
    const int64_t k = (int64_t)blockIdx.x * seg + threadIdx.x;
    if ((int)threadIdx.x < seg && k < n) dst[k] = src[k];
}

// cn_debug_orca: one quad per simulator (16 per 64-lane workgroup), the step kernel's quad-path functions
__global__ void __launch_bounds__(64) cn_orca_kernel(int64_t n, int A, const float *__restrict__ ag,
                                                     const float *__restrict__ self, float nd, float th, float ts,
                                                     float *__restrict__ out)
{
    __shared__ float4 Ls[16][9];
    const int q = threadIdx.x >> 2, sq = threadIdx.x & 3;
    const int64_t i = (int64_t)blockIdx.x * 16 + q;
    const bool act = i < n;
    const float *a = ag + (act ? i : 0) * A * 5;
    const int M = A - 1;
    int cnt = 0;
    if (act)
        cnt = orca_lines_quad(
            [&](int k, float &x, float &y, float &vx, float &vy, float &r) {
                const float *o = a + (k + 1) * 5;
                x = o[0]; y = o[1]; vx = o[2]; vy = o[3]; r = o[4];
            },
            M, sq, a[0], a[1], a[2], a[3], a[4], nd * nd, fdiv(1.0f, th), fdiv(1.0f, ts), Ls[q]);
    wsync();
    if (act) {
        const float vmax = self[3 * i], ox = self[3 * i + 1], oy = self[3 * i + 2];
        float rx, ry;
        float4 R[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) R[u] = sq + 4 * u < cnt ? Ls[q][sq + 4 * u] : make_float4(0.f, 0.f, 0.f, 0.f);
        const int fail_at = lp2_r<3>(R, cnt, vmax, ox, oy, sq, rx, ry);
        if (fail_at < cnt) lp3_r<3>(R, Ls[q], cnt, fail_at, vmax, sq, rx, ry);
        if (sq == 0) {
            out[4 * i] = rx; out[4 * i + 1] = ry; out[4 * i + 2] = (float)fail_at; out[4 * i + 3] = (float)cnt;
        }
    }
}

// cn_orca_predict_kd: ORCA.predict of simulators of any size up to CN_ORCA_MAXA agents, with RVO2's KdTree
// (MAX_LEAF_SIZE 10) and its persisted agents_ order. One quad per simulator (16 per 64-lane workgroup):
// lane 0 of the quad builds the tree (buildAgentTreeRecursive, which re-permutes agents_ in place) and runs
// the query (queryAgentTreeRecursive + insertAgentNeighbor with maxNeighbors = A - 1), both sequential as
// in RVO2 -- the plugin serves one predict per agent per env step, off the batched step path, which has its
// own ballot-partitioned walk; then the quad builds the ORCA lines in neighbour order and runs the quad
// linear programs of the step kernel. Oracle: cpu_ref.c:kd_build / kd_query / rvo2_agent0.
#define CN_ORCA_MAXA 64
// 20 B per node: ranges and child indices fit bytes (A <= 64 agents, < 2A nodes); the build / query stacks
// below are bytes too -- the per-lane private arrays were 5.7 KB of scratch per lane with ints, 3.3 KB now
struct KdNodeS { uint8_t begin, end, left, right; float minX, maxX, minY, maxY; };

__device__ __forceinline__ float kd_bdist(const KdNodeS &t, float x, float y)
{
    const float a = (0.0f < t.minX - x) ? t.minX - x : 0.0f, b = (0.0f < x - t.maxX) ? x - t.maxX : 0.0f;
    const float cc = (0.0f < t.minY - y) ? t.minY - y : 0.0f, d = (0.0f < y - t.maxY) ? y - t.maxY : 0.0f;
    return a * a + b * b + cc * cc + d * d;
}

// lane-sequential KdTree build + query over X / Y [A] (LDS), perm [A] (LDS, updated in place); writes the
// neighbours of agent 0 in insertion-sorted order to nb [A - 1] (agent ids) and returns their count
__device__ int kd_neighbors_seq(int A, const float *X, const float *Y, uint8_t *perm, float rangeSq, uint8_t *nb)
{
    KdNodeS T[2 * CN_ORCA_MAXA];
    uint8_t stk[CN_ORCA_MAXA + 2][3];
    int sp = 0;
    stk[sp][0] = 0; stk[sp][1] = (uint8_t)A; stk[sp][2] = 0; ++sp;
    while (sp > 0) {   // any order of the recursive calls gives the same tree: children own disjoint ranges
        --sp;
        const int begin = stk[sp][0], end = stk[sp][1], node = stk[sp][2];
        KdNodeS t;
        t.begin = (uint8_t)begin; t.end = (uint8_t)end; t.left = t.right = 0;
        t.minX = t.maxX = X[perm[begin]];
        t.minY = t.maxY = Y[perm[begin]];
        for (int i = begin + 1; i < end; ++i) {
            const float x = X[perm[i]], y = Y[perm[i]];
            t.maxX = t.maxX < x ? x : t.maxX; t.minX = x < t.minX ? x : t.minX;
            t.maxY = t.maxY < y ? y : t.maxY; t.minY = y < t.minY ? y : t.minY;
        }
        if (end - begin > 10) {
            const bool vert = t.maxX - t.minX > t.maxY - t.minY;
            const float split = vert ? 0.5f * (t.maxX + t.minX) : 0.5f * (t.maxY + t.minY);
            int left = begin, right = end;
            while (left < right) {
                while (left < right && (vert ? X[perm[left]] : Y[perm[left]]) < split) ++left;
                while (right > left && (vert ? X[perm[right - 1]] : Y[perm[right - 1]]) >= split) --right;
                if (left < right) {
                    const uint8_t s = perm[left]; perm[left] = perm[right - 1]; perm[right - 1] = s;
                    ++left; --right;
                }
            }
            if (left == begin) { ++left; ++right; }
            t.left = (uint8_t)(node + 1);
            t.right = (uint8_t)(node + 2 * (left - begin));
            stk[sp][0] = (uint8_t)left; stk[sp][1] = (uint8_t)end; stk[sp][2] = t.right; ++sp;
            stk[sp][0] = (uint8_t)begin; stk[sp][1] = (uint8_t)left; stk[sp][2] = t.left; ++sp;
        }
        T[node] = t;
    }
    // query: a node popped with distance d is walked only if d < rangeSq at that moment (the recursion tests
    // the nearer child at once and the farther one after the nearer subtree; ties visit the right first)
    const int maxN = A - 1;
    float nd[CN_ORCA_MAXA];
    int cnt = 0;
    float dst[CN_ORCA_MAXA + 2];
    uint8_t nst[CN_ORCA_MAXA + 2];
    sp = 0;
    nst[0] = 0; dst[0] = -1.0f; sp = 1;
    const float x0 = X[0], y0 = Y[0];
    while (sp > 0) {
        --sp;
        const int node = nst[sp];
        if (!(dst[sp] < rangeSq)) continue;
        const KdNodeS &t = T[node];
        if (t.end - t.begin <= 10) {
            for (int i = t.begin; i < t.end; ++i) {   // Agent::insertAgentNeighbor
                const int a = perm[i];
                if (a == 0) continue;
                const float dx = x0 - X[a], dy = y0 - Y[a];
                const float distSq = dx * dx + dy * dy;
                if (distSq < rangeSq) {
                    if (cnt < maxN) { nd[cnt] = distSq; nb[cnt] = (uint8_t)a; ++cnt; }
                    int k = cnt - 1;
                    while (k != 0 && distSq < nd[k - 1]) { nd[k] = nd[k - 1]; nb[k] = nb[k - 1]; --k; }
                    nd[k] = distSq; nb[k] = (uint8_t)a;
                    if (cnt == maxN) rangeSq = nd[cnt - 1];
                }
            }
            continue;
        }
        const float dl = kd_bdist(T[t.left], x0, y0), dr = kd_bdist(T[t.right], x0, y0);
        if (dl < dr) { nst[sp] = t.right; dst[sp] = dr; nst[sp + 1] = t.left; dst[sp + 1] = dl; }
        else { nst[sp] = t.left; dst[sp] = dl; nst[sp + 1] = t.right; dst[sp + 1] = dr; }
        sp += 2;
    }
    return cnt;
}

// LDS of one cn_orca_kd_kernel workgroup, sized by the simulators' agent count A (dynamic): 16 quads' lines
// and projected lines [A - 1] float4 each, positions [A] float x 2, agents_ order and neighbours [A] bytes, counts.
// (Sized for CN_ORCA_MAXA it was 42.5 KB, 3 one-wave workgroups per CU; at A = 26, 17 KB: 9.)
__host__ __device__ inline int orca_kd_lds(int A)
{
    return 16 * (2 * 16 * (A - 1) + 2 * 4 * A) + ((2 * 16 * A + 15) & ~15) + 16 * 4;
}

__global__ void __launch_bounds__(64) cn_orca_kd_kernel(int64_t n, int A, const float *__restrict__ ag,
                                                        const float *__restrict__ self, float nd, float th, float ts,
                                                        uint8_t *__restrict__ perm_io, float *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) char kd_smem[];
    const int q = threadIdx.x >> 2, sq = threadIdx.x & 3;
    float4 *Lq = (float4 *)kd_smem + q * (A - 1);                 // [16][A - 1]
    float4 *Pq = (float4 *)kd_smem + 16 * (A - 1) + q * (A - 1);  // [16][A - 1]
    float *Xq = (float *)(kd_smem + 16 * 2 * 16 * (A - 1)) + q * A;
    float *Yq = (float *)(kd_smem + 16 * 2 * 16 * (A - 1)) + 16 * A + q * A;
    uint8_t *Pmq = (uint8_t *)(kd_smem + 16 * (2 * 16 * (A - 1) + 2 * 4 * A)) + q * A;
    uint8_t *Nbq = (uint8_t *)(kd_smem + 16 * (2 * 16 * (A - 1) + 2 * 4 * A)) + 16 * A + q * A;
    int *Cn = (int *)(kd_smem + orca_kd_lds(A) - 16 * 4);
    const int64_t i = (int64_t)blockIdx.x * 16 + q;
    const bool act = i < n;
    const float *a = ag + (act ? i : 0) * A * 5;
    if (act)
        for (int k = sq; k < A; k += 4) {
            Xq[k] = a[k * 5]; Yq[k] = a[k * 5 + 1];
            Pmq[k] = perm_io ? perm_io[i * A + k] : (uint8_t)k;
        }
    wsync();
    if (act && sq == 0) Cn[q] = A > 1 ? kd_neighbors_seq(A, Xq, Yq, Pmq, nd * nd, Nbq) : 0;
    wsync();
    if (act) {
        const int cnt = Cn[q];
        const float invTH = fdiv(1.0f, th), invTS = fdiv(1.0f, ts);
        for (int k = sq; k < cnt; k += 4) {
            const float *o = a + Nbq[k] * 5;
            Lq[k] = orca_line(a[0], a[1], a[2], a[3], a[4], o[0], o[1], o[2], o[3], o[4], invTH, invTS);
        }
        if (perm_io)
            for (int k = sq; k < A; k += 4) perm_io[i * A + k] = Pmq[k];
    }
    wsync();
    if (act) {
        const int cnt = Cn[q];
        const float vmax = self[3 * i], ox = self[3 * i + 1], oy = self[3 * i + 2];
        float rx, ry;
        const int fail_at = lp2_q<uint64_t>(Lq, cnt, vmax, ox, oy, sq, rx, ry);
        if (fail_at < cnt) lp3_q<uint64_t>(Lq, Pq, cnt, fail_at, vmax, sq, rx, ry);
        if (sq == 0) {
            out[4 * i] = rx; out[4 * i + 1] = ry; out[4 * i + 2] = (float)fail_at; out[4 * i + 3] = (float)cnt;
        }
    }
}

// cn_social_force_predict: SOCIAL_FORCE.predict (social_force.py:11-66) for n agents, one lane each, f64 in
// the reference's operation order (the step kernel's phase 2 on caller-given states)
__global__ void __launch_bounds__(64) cn_sf_predict_kernel(int64_t n, int M, const double *__restrict__ self,
                                                           const double *__restrict__ others, double A, double B,
                                                           double KI, double dt, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *s = self + 9 * i;   // px, py, vx, vy, radius, gx, gy, v_pref, theta
    const double px = s[0], py = s[1], vx0 = s[2], vy0 = s[3], rad = s[4], vpref = s[7];
    const double gdx = s[5] - px, gdy = s[6] - py;
    const double dg = dsqrt(gdx * gdx + gdy * gdy);
    const double dvx = ddiv(gdx, dg) * vpref, dvy = ddiv(gdy, dg) * vpref;
    const double cdx = KI * (dvx - vx0), cdy = KI * (dvy - vy0);
    double ix = 0.0, iy = 0.0;
    for (int k = 0; k < M; ++k) {
        const double *o = others + (i * M + k) * 5;   // px, py, vx, vy, radius
        const double ddx = px - o[0], ddy = py - o[1];
        const double d = dsqrt(ddx * ddx + ddy * ddy);
        const double ex = exp(ddiv(rad + o[4] - d, B));
        ix += A * ex * ddiv(ddx, d);
        iy += A * ex * ddiv(ddy, d);
    }
    const double nx = vx0 + (cdx + ix) * dt, ny = vy0 + (cdy + iy) * dt;
    const double nn = np_norm2(nx, ny);
    if (nn > vpref) { out[2 * i] = ddiv(nx, nn) * vpref; out[2 * i + 1] = ddiv(ny, nn) * vpref; }
    else { out[2 * i] = nx; out[2 * i + 1] = ny; }
}

// One control word of the engine set from the stream (graph mode's draw-all flag after cn_reset /
// cn_set_state). A kernel, not hipMemsetAsync: captured into a hipGraph it is a kernel node, and this
// runtime replays memset nodes with stale bytes (cn_graph_node_counts).
__global__ void cn_ctl_set_kernel(uint32_t *w, uint32_t v)
{
    if (threadIdx.x == 0) *w = v;
}

static int ctl_set(uint32_t *w, uint32_t v, hipStream_t st)
{
    (void)hipGetLastError();
    hipLaunchKernelGGL(cn_ctl_set_kernel, dim3(1), dim3(64), 0, st, w, v);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : set_err(CN_EHIP, hipGetErrorString(e));
}

// Key snapshot for a PEND_BOTH launch (after cn_set_state, and the quad path's cn_reset): every env's
// {e, reset_count, case_counter lo, hi} into the spawn list the next step launch reads (kr = (t + 2) % 3 for
// launch t: the host's sequence number, or graph mode's device word). That launch's spawn waves key both of an
// env's pending spawns from this entry, not from the state its own step workgroups rewrite when a terminal env
// resets inline (crowd_sim_dict.py:147-164: the seed of the k-th reset is offset + case_counter + thisSeed).
__global__ void cn_keysnap_kernel(const int32_t *__restrict__ reset_count, const int64_t *__restrict__ case_counter,
                                  uint32_t *plist_base, const uint32_t *ctl, int host_kr, int E)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int64_t kr = host_kr >= 0 ? host_kr : (int64_t)((ctl[CN_CTL_NSTEP] + 2u) % 3u);
    uint32_t *q = plist_base + kr * 4 * ((int64_t)E + 64) + 4 * (int64_t)e;
    const uint64_t cc = (uint64_t)case_counter[e];
    const uint4 v = make_uint4((uint32_t)e, (uint32_t)reset_count[e], (uint32_t)cc, (uint32_t)(cc >> 32));
    *(uint4 *)q = v;
}

// the snapshot for the engine's next step launch (g->nstep: the host sequence; graph mode reads the device's)
static int keysnap(const cn_engine *g, hipStream_t st)
{
    const int host_kr = g->devseq ? -1 : (int)((g->nstep + 2) % 3);
    (void)hipGetLastError();
    hipLaunchKernelGGL(cn_keysnap_kernel, dim3((g->E + 255) / 256), dim3(256), 0, st, g->s.reset_count, g->s.case_counter,
                       g->plist, (const uint32_t *)g->work_count, host_kr, (int)g->E);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : set_err(CN_EHIP, hipGetErrorString(e));
}

extern "C" {

int cn_graph_node_counts(void *graph, int64_t *counts, int n, int64_t *total)
{
    if (!graph || (n > 0 && !counts) || n < 0 || n > 32) return set_err(CN_EINVAL, "cn_graph_node_counts: graph, 0 <= n <= 32");
    for (int k = 0; k < n; ++k) counts[k] = 0;
    size_t num = 0;
    HIPCHK(hipGraphGetNodes((hipGraph_t)graph, nullptr, &num));
    std::vector<hipGraphNode_t> nodes(num);
    if (num) HIPCHK(hipGraphGetNodes((hipGraph_t)graph, nodes.data(), &num));
    for (size_t i = 0; i < num; ++i) {
        hipGraphNodeType t;
        HIPCHK(hipGraphNodeGetType(nodes[i], &t));
        if ((int)t >= 0 && (int)t < n) ++counts[(int)t];
    }
    if (total) *total = (int64_t)num;
    return CN_OK;
}

const char *cn_last_error(void) { return g_err; }
#ifndef CN_SRC_HASH
#define CN_SRC_HASH "unversioned"
#endif
// build.py passes the sha256 of the flags + sources; _lib.lib() compares it with the sources on disk
const char *cn_version(void) { return "crowdnav_dsrnn_amd 0.2 (gfx950) CN_SRC_HASH=" CN_SRC_HASH; }

int cn_config_validate(const cn_config *c)
{
    if (!c) return set_err(CN_EINVAL, "null config");
    if (c->num_envs <= 0) return set_err(CN_EINVAL, "num_envs must be > 0");
    if ((int64_t)c->num_envs * (c->human_num + 1) >= (1LL << 31) / 8)
        return set_err(CN_EUNSUPPORTED, "num_envs * human_num too large for one engine (shard over engines)");
    if (c->human_num < 1 || c->human_num > 31) return set_err(CN_EUNSUPPORTED, "human_num must be in [1, 31]");
    if (c->human_num + (c->robot_visible ? 1 : 0) > CN_MAX_A) return set_err(CN_EUNSUPPORTED, "too many agents");
    if (c->num_scenarios < 1 || c->num_scenarios > CN_MAX_SCENARIOS) return set_err(CN_EINVAL, "num_scenarios");
    for (int k = 0; k < c->num_scenarios; ++k)
        if (c->scenarios[k] < 0 || c->scenarios[k] > CN_SC_SIDE_PREF_CROSSING) return set_err(CN_EINVAL, "scenario id");
    if (c->kinematics != CN_HOLONOMIC && c->kinematics != CN_UNICYCLE) return set_err(CN_EINVAL, "kinematics");
    if (c->rng_mode != CN_RNG_MT19937 && c->rng_mode != CN_RNG_PHILOX) return set_err(CN_EINVAL, "rng_mode");
    if (c->human_policy != CN_POLICY_ORCA && c->human_policy != CN_POLICY_SOCIAL_FORCE)
        return set_err(CN_EUNSUPPORTED, "human policy");
    if (!c->potential_based) return set_err(CN_EUNSUPPORTED, "only potential-based reward shaping is supported");
    if (!(c->time_step > 0)) return set_err(CN_EINVAL, "time_step must be > 0");
    if (c->phase < 0 || c->phase > 2) return set_err(CN_EINVAL, "phase");
    if (c->nenv <= 0) return set_err(CN_EINVAL, "nenv must be > 0");
    if (c->max_tries <= 0) return set_err(CN_EINVAL, "max_tries must be > 0");
    return CN_OK;
}

int cn_state_field_info(int field, const char **name, int *type_code, int *count_kind)
{
    static const char *names[] = {
#define X(n, ct, tc, ck) #n,
        CN_STATE_FIELDS(X)
#undef X
    };
    static const int tcs[] = {
#define X(n, ct, tc, ck) tc,
        CN_STATE_FIELDS(X)
#undef X
    };
    static const int cks[] = {
#define X(n, ct, tc, ck) ck,
        CN_STATE_FIELDS(X)
#undef X
    };
    if (field < 0 || field >= CN_NUM_FIELDS) return set_err(CN_EINVAL, "field index");
    if (name) *name = names[field];
    if (type_code) *type_code = tcs[field];
    if (count_kind) *count_kind = cks[field];
    return CN_OK;
}

int cn_state_layout_offsets(const cn_config *cfg, int64_t *offsets, int64_t *total)
{
    if (!cfg) return set_err(CN_EINVAL, "null config");
    const int64_t t = cn_state_layout(cfg->num_envs, cfg->human_num, cfg->robot_visible, offsets);
    if (total) *total = t;
    return CN_OK;
}

int cn_create(const cn_config *cfg, int device, cn_engine **out)
{
    if (!out) return set_err(CN_EINVAL, "null out");
    *out = nullptr;
    int rc = cn_config_validate(cfg);
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    cn_engine *g = new cn_engine();
    g->c = *cfg;
    g->device = device;
    g->E = cfg->num_envs;
    g->N = cfg->human_num;
    g->NS = g->N;
    g->A = cn_sim_agents(g->N, cfg->robot_visible);
    g->plan = cn_step_plan(g->N, cfg->robot_visible);
    g->state_bytes = cn_state_layout(g->E, g->N, cfg->robot_visible, nullptr);
    switch (cfg->phase) {
    case CN_PHASE_TRAIN: g->case_size = 4294967295LL - 2000; g->counter_offset = 2000; break;
    case CN_PHASE_VAL: g->case_size = cfg->val_size; g->counter_offset = 0; break;
    default: g->case_size = cfg->test_size; g->counter_offset = 1000; break;
    }
    if (g->case_size <= 0) { delete g; return set_err(CN_EINVAL, "case size (val_size/test_size) must be > 0"); }
    const int64_t E = g->E, EN = (int64_t)g->E * g->N;
    auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
    // pending spawns: every array holds both slots ([2][...], pend_slot)
    const int64_t pb_mt = al(2 * E * CN_MT_N * 4), pb_i = al(2 * E * 4), pb_cc = al(2 * E * 8), pb_r = al(2 * 5 * E * 8),
                  pb_h = al(2 * 7 * EN * 8);
    const int64_t pend_bytes = pb_mt + 5 * pb_i + 2 * pb_cc + pb_r + pb_h;
    hipError_t e1 = hipMalloc(&g->state, g->state_bytes);
    hipError_t e2 = hipMalloc(&g->work, sizeof(uint32_t) * (g->E + 64));
    hipError_t e3 = hipMalloc(&g->work_count, 64);
    hipError_t e4 = hipMalloc(&g->plist, sizeof(uint32_t) * 3 * 4 * (g->E + 64));
    hipError_t e6 = hipMalloc(&g->rlist, sizeof(uint32_t) * 3 * 4 * (2 * (int64_t)g->E + 64));
    hipError_t e5 = hipMalloc(&g->pend_mem, pend_bytes);
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess || e5 != hipSuccess ||
        e6 != hipSuccess) {
        (void)hipFree(g->state); (void)hipFree(g->work); (void)hipFree(g->work_count); (void)hipFree(g->plist); (void)hipFree(g->pend_mem);
        (void)hipFree(g->rlist);
        delete g;
        return set_err(CN_ENOMEM, "hipMalloc failed");
    }
    if (hipMemset(g->state, 0, g->state_bytes) != hipSuccess || hipMemset(g->work_count, 0, 64) != hipSuccess ||
        hipMemset(g->pend_mem, 0, pend_bytes) != hipSuccess) {
        cn_destroy(g);
        return set_err(CN_EHIP, "hipMemset failed");
    }
    {
        char *b = (char *)g->pend_mem;
        g->pend.mt = (uint32_t *)b; b += pb_mt;
        g->pend.pos = (int32_t *)b; b += pb_i;
        g->pend.ovf = (uint32_t *)b; b += pb_i;
        g->pend.sc = (int32_t *)b; b += pb_i;
        g->pend.rc = (int32_t *)b; b += pb_i;
        g->pend.ok = (uint64_t *)b; b += pb_cc;
        g->pend.prog = (int32_t *)b; b += pb_i;
        g->pend.cc = (int64_t *)b; b += pb_cc;
        g->pend.r = (double *)b; b += pb_r;
        g->pend.h = (double *)b;
    }
    g->pend_all = PEND_BOTH;
    {
        // the plan holds phase 5's RNG regions (laid over the ORCA scratch); spare workgroups run as many
        // spawning waves as regions fit in the same allocation
        g->a_lds = g->plan.total;
        const int fit = g->a_lds / g->plan.rng_stride;
        g->pend_waves = fit < g->plan.T / 64 ? fit : g->plan.T / 64;
        const int nw = g->pend_waves;
        const int64_t need = (E + nw - 1) / nw;
        // ~128 spawning waves on the quad path; 256 on the kd-tree path, whose crowded spawns (~1M cycles
        // each at 25 humans in square_crossing, ~4 % of the envs per step) must not queue behind each other
        const int cap = (g->plan.kd ? 256 : CN_QUAD_SPAWN_WAVES) / nw;
        const int pb = (int)(need < cap ? need : cap);
        g->pend_blocks = g->plan.kd ? (pb + 7) & ~7 : pb;   // leading: a multiple of 8 (XCD placement)
        // kd-tree path: a crowded spawn may take longer than the launch's step rounds; each spawning wave parks
        // its spawn after ~0.6 M cycles and a later launch resumes it (the spawn is needed one whole episode
        // later). Round 5: spawn-list entries carry the counters of the reset that queued them (a spawn wave
        // that read them from the state could see a later reset of the same env and queue a key that the next
        // launch queued again: two writers of one pending slot, one of them resuming from it -- 5 of 149 C3 runs
        // departed; 0 of 149 with keyed entries). The quad path parks after CN_QUAD_BUDGET cycles (round 6).
        g->spawn_budget = g->plan.kd ? 600000 : (CN_QUAD_PARK ? CN_QUAD_BUDGET : 0);
    }
    cn_state_bind(&g->s, g->state, g->E, g->N, cfg->robot_visible);
    if (circ_table_init() != hipSuccess) {
        cn_destroy(g);
        return set_err(CN_EHIP, "hipMemcpyToSymbol failed");
    }
    if (g->a_lds > 160 * 1024) { cn_destroy(g); return set_err(CN_EUNSUPPORTED, "LDS plan exceeds 160 KiB"); }
    if (g->a_lds > 64 * 1024) {
        const void *ks[8] = {(const void *)cn_step_kernel<true, false, false>, (const void *)cn_step_kernel<false, false, false>,
                             (const void *)cn_step_kernel<true, true, false>, (const void *)cn_step_kernel<false, true, false>,
                             (const void *)cn_step_kernel<true, false, true>, (const void *)cn_step_kernel<false, false, true>,
                             (const void *)cn_step_kernel<true, true, true>, (const void *)cn_step_kernel<false, true, true>};
        for (const void *k : ks) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g->a_lds);
    }
    g->rng_grid = g->E < 2048 ? g->E : 2048;
    // the first launch draws every env's spawns (PEND_BOTH) from the key snapshot of the zeroed state
    if (keysnap(g, nullptr) != CN_OK) { cn_destroy(g); return CN_EHIP; }
    HIPCHK(hipDeviceSynchronize());
    *out = g;
    return CN_OK;
}

// Mixed engine (per-env scenario dispatch with per-env human counts). Env r of the engine
// (global index cfg.env_offset + r) belongs to group env_group[r]; each group is a plain engine over its
// envs with its own cn_config (human count, scenario set, circle radius, side preference, goal changing,
// ...), stepping them in the caller's (E, ...) buffers at their own rows (spatial_edges padded to the
// largest human count). Seeds and round-robin scenarios use the global index, so groups[g].scenarios
// must be the full scenario list and env r's scenario (scenarios[(env_offset + r) % num_scenarios]) must
// be one its group was configured for -- which the caller guarantees by assigning groups per scenario.
int cn_create_mixed(const cn_config *groups, int num_groups, const int32_t *env_group, int64_t num_envs, int device,
                    cn_engine **out)
{
    if (!out) return set_err(CN_EINVAL, "null out");
    *out = nullptr;
    if (!groups || !env_group || num_groups < 1 || num_groups > 64 || num_envs <= 0)
        return set_err(CN_EINVAL, "cn_create_mixed: 1..64 groups, env_group[num_envs] required");
    if (num_envs >= (1LL << 31) / 64) return set_err(CN_EUNSUPPORTED, "cn_create_mixed: too many envs");
    std::vector<std::vector<int32_t>> rows(num_groups);
    for (int64_t r = 0; r < num_envs; ++r) {
        if (env_group[r] < 0 || env_group[r] >= num_groups) return set_err(CN_EINVAL, "cn_create_mixed: env_group out of range");
        rows[env_group[r]].push_back((int32_t)r);
    }
    int NS = 0;
    for (int k = 0; k < num_groups; ++k) {
        const cn_config &c = groups[k];
        if ((int64_t)c.num_envs != (int64_t)rows[k].size())
            return set_err(CN_EINVAL, "cn_create_mixed: groups[g].num_envs must equal the envs assigned to group g");
        if (c.env_offset != groups[0].env_offset || c.nenv != groups[0].nenv || c.seed != groups[0].seed ||
            c.phase != groups[0].phase)
            return set_err(CN_EINVAL, "cn_create_mixed: env_offset / nenv / seed / phase must agree across groups");
        if (c.scenario_mode != CN_SCMODE_ROUND_ROBIN)
            return set_err(CN_EUNSUPPORTED, "cn_create_mixed: round-robin scenario mode only");
        NS = c.human_num > NS ? c.human_num : NS;
    }
    HIPCHK(hipSetDevice(device));
    cn_engine *m = new cn_engine();
    m->c = groups[0];
    m->c.num_envs = (int32_t)num_envs;
    m->c.human_num = NS;
    m->device = device;
    m->E = (int)num_envs;
    m->N = m->NS = NS;
    m->grp = new cn_engine *[num_groups]();
    for (int k = 0; k < num_groups; ++k) {
        if (groups[k].num_envs == 0) continue;
        int rc = cn_create(&groups[k], device, &m->grp[m->ngroups]);
        if (rc) { cn_destroy(m); return rc; }
        cn_engine *g = m->grp[m->ngroups++];
        g->NS = NS;
        if (hipMalloc(&g->rows, sizeof(int32_t) * rows[k].size()) != hipSuccess) {
            cn_destroy(m);
            return set_err(CN_ENOMEM, "hipMalloc failed");
        }
        if (hipMemcpy(g->rows, rows[k].data(), sizeof(int32_t) * rows[k].size(), hipMemcpyHostToDevice) != hipSuccess) {
            cn_destroy(m);
            return set_err(CN_EHIP, "hipMemcpy failed");
        }
        m->state_bytes += g->state_bytes;
    }
    // the groups' step launches are independent (disjoint envs and output rows): run them concurrently,
    // group 0 on the caller's stream, group k > 0 on its own stream forked after the caller's prior work
    // and joined back before the caller's next work (stream order is kept for the caller)
    m->gstream = new hipStream_t[m->ngroups]();
    m->gev = new hipEvent_t[m->ngroups + 1]();
    for (int k = 0; k <= m->ngroups; ++k)
        if (hipEventCreateWithFlags(&m->gev[k], hipEventDisableTiming) != hipSuccess) {
            cn_destroy(m);
            return set_err(CN_EHIP, "hipEventCreate failed");
        }
    for (int k = 1; k < m->ngroups; ++k)
        if (hipStreamCreateWithFlags(&m->gstream[k], hipStreamNonBlocking) != hipSuccess) {
            cn_destroy(m);
            return set_err(CN_EHIP, "hipStreamCreate failed");
        }
    *out = m;
    return CN_OK;
}

// per-env human count of an engine (plain: N everywhere), into host memory [E]
int cn_env_humans(const cn_engine *g, int32_t *dst)
{
    if (!g || !dst) return set_err(CN_EINVAL, "null argument");
    if (!g->ngroups) {
        for (int64_t r = 0; r < g->E; ++r) dst[r] = g->N;
        return CN_OK;
    }
    for (int k = 0; k < g->ngroups; ++k) {
        const cn_engine *q = g->grp[k];
        std::vector<int32_t> rows(q->E);
        HIPCHK(hipMemcpy(rows.data(), q->rows, sizeof(int32_t) * q->E, hipMemcpyDeviceToHost));
        for (int64_t e = 0; e < q->E; ++e) dst[rows[e]] = q->N;
    }
    return CN_OK;
}

static void prof_free(cn_engine *g)
{
    if (g->ev) {
        for (int k = 0; k < 2; ++k) (void)hipEventDestroy(g->ev[k]);
        delete[] g->ev;
    }
    g->ev = nullptr;
    g->prof_cap = g->prof_n = g->prof_on = 0;
}

// Two events bracket the whole window of `max_steps` launches (one before the first, one after the
// last): per-launch event pairs cost ~12 us of stream time each on this GPU, more than the launch gaps
// they would exclude (back-to-back step launches are separated by < 0.2 us).
int cn_profile(cn_engine *g, int enable, int max_steps)
{
    if (!g) return set_err(CN_EINVAL, "null engine");
    prof_free(g);
    if (!enable) return CN_OK;
    if (max_steps <= 0) return set_err(CN_EINVAL, "max_steps must be > 0");
    g->ev = new hipEvent_t[2];
    for (int k = 0; k < 2; ++k) HIPCHK(hipEventCreate(&g->ev[k]));
    g->prof_cap = max_steps;
    g->prof_on = 1;
    return CN_OK;
}

int cn_profile_read(cn_engine *g, double *a_ms, double *b_ms, int64_t *launches)
{
    if (!g) return set_err(CN_EINVAL, "null engine");
    float ta = 0;
    if (g->prof_n > 0) {
        if (g->prof_n < g->prof_cap) return set_err(CN_EINVAL, "profile window not complete (fewer launches than max_steps)");
        HIPCHK(hipEventSynchronize(g->ev[1]));
        HIPCHK(hipEventElapsedTime(&ta, g->ev[0], g->ev[1]));
    }
    if (a_ms) *a_ms = ta;
    if (b_ms) *b_ms = 0;
    if (launches) *launches = g->prof_n;
    return CN_OK;
}

void cn_destroy(cn_engine *g)
{
    if (!g) return;
    (void)hipSetDevice(g->device);
    prof_free(g);
    if (g->grp) {
        for (int k = 0; k < g->ngroups; ++k) cn_destroy(g->grp[k]);
        if (g->gstream)
            for (int k = 1; k < g->ngroups; ++k) (void)hipStreamDestroy(g->gstream[k]);
        if (g->gev)
            for (int k = 0; k <= g->ngroups; ++k) (void)hipEventDestroy(g->gev[k]);
        delete[] g->grp;
        delete[] g->gstream;
        delete[] g->gev;
        delete g;
        return;
    }
    (void)hipFree(g->rows);
    (void)hipFree(g->state);
    (void)hipFree(g->work);
    (void)hipFree(g->work_count);
    (void)hipFree(g->plist);
    (void)hipFree(g->rlist);
    (void)hipFree(g->pend_mem);
    delete g;
}

int cn_reset(cn_engine *g, void *stream, float *robot_node, float *temporal, float *spatial)
{
    if (!g || !robot_node || !temporal || !spatial) return set_err(CN_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    if (g->ngroups) {
        for (int k = 0; k < g->ngroups; ++k) {
            const int rc = cn_reset(g->grp[k], stream, robot_node, temporal, spatial);
            if (rc) return rc;
        }
        return CN_OK;
    }
    RngArgs a;
    a.o.s = g->s; a.o.robot_node = robot_node; a.o.temporal = temporal; a.o.spatial = spatial;
    a.o.case_size = g->case_size;
    a.o.ov.row = g->rows; a.o.ov.NS = g->NS;
    a.pend = g->pend; a.E = g->E; a.counter_offset = g->counter_offset;
    // the reset kernel draws the next two spawns too, so the first step launches (whose spawns would otherwise
    // run inline in step workgroups until the budgeted spawn waves catch up) find them drawn (PEND_FRESH);
    // without quad-path parking the quad path's first launch draws them (PEND_BOTH, as after cn_set_state)
    a.draw_next = (g->plan.kd || CN_QUAD_PARK) ? 1 : 0;
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_reset_kernel, dim3(g->rng_grid), dim3(64), 0, st, a, g->c);
    HIPCHK(hipGetLastError());
    // every env starts a new episode (kd-tree path: with its next two spawns drawn): the next step launch
    // draws them (none) and ignores the earlier launches' lists (host flag; graph mode: the device flag,
    // stream-ordered)
    g->pend_all = a.draw_next ? PEND_FRESH : PEND_BOTH;
    if (!a.draw_next) {   // PEND_BOTH keys its items from a snapshot of the counters the reset kernel wrote
        const int rk = keysnap(g, st);
        if (rk) return rk;
    }
    if (g->devseq) return ctl_set(g->work_count + CN_CTL_ALL, (uint32_t)g->pend_all, st);
    return CN_OK;
}

int cn_step(cn_engine *g, void *stream, const float *actions, float *robot_node, float *temporal, float *spatial,
            float *reward, uint8_t *done, int8_t *event, float *info, double *ep_return, int32_t *ep_len)
{
    if (!g || !actions || !robot_node || !temporal || !spatial) return set_err(CN_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    // spawn lists, triple-buffered: launch t appends to t%3, reads (t-1)%3, zeroes (t+1)%3 (host sequence;
    // graph mode keeps it on the device, StepArgs::devseq)
    const int kw = (int)(g->nstep % 3), kr = (int)((g->nstep + 2) % 3), kz = (int)((g->nstep + 1) % 3);
    ++g->nstep;
    const bool prof = g->prof_on && g->prof_n < g->prof_cap;
    if (prof && g->prof_n == 0) HIPCHK(hipEventRecord(g->ev[0], st));
    if (g->ngroups) {   // one step launch per group, concurrently (fork / join around the caller's stream)
        if (g->ngroups > 1) HIPCHK(hipEventRecord(g->gev[0], st));
        for (int k = 0; k < g->ngroups; ++k) {
            hipStream_t sk = st;
            if (k > 0) { sk = g->gstream[k]; HIPCHK(hipStreamWaitEvent(sk, g->gev[0], 0)); }
            const int rc = cn_step(g->grp[k], (void *)sk, actions, robot_node, temporal, spatial, reward, done, event,
                                   info, ep_return, ep_len);
            if (rc) {   // join the groups already forked, so no side-stream work outlives the caller's order
                for (int j = 1; j < k; ++j) (void)hipStreamWaitEvent(st, g->gev[j], 0);
                return rc;
            }
            if (k > 0) HIPCHK(hipEventRecord(g->gev[k], sk));
        }
        for (int k = 1; k < g->ngroups; ++k) HIPCHK(hipStreamWaitEvent(st, g->gev[k], 0));
        if (prof && ++g->prof_n == g->prof_cap) HIPCHK(hipEventRecord(g->ev[1], st));
        return CN_OK;
    }
    StepArgs a;
    a.s = g->s; a.actions = actions; a.robot_node = robot_node; a.temporal = temporal; a.spatial = spatial;
    a.reward = reward; a.done = done; a.event = event; a.info = info; a.ep_return = ep_return; a.ep_len = ep_len;
    a.E = g->E;
    a.case_size = g->case_size;
    a.ctl = g->work_count; a.plist_base = g->plist; a.rlist_base = g->rlist;
    a.plist_w = g->plist + (int64_t)kw * 4 * (g->E + 64);
    a.pcount_w = g->work_count + 2 + kw;
    a.pcount_zero = g->work_count + 2 + kz;
    a.rcount_zero = g->work_count + 5 + kz;
    a.pend.rlist = g->rlist + (int64_t)kr * 4 * (2 * (int64_t)g->E + 64); a.pend.rcount = g->work_count + 5 + kr;
    a.pend.rlist_w = g->rlist + (int64_t)kw * 4 * (2 * (int64_t)g->E + 64); a.pend.rcount_w = g->work_count + 5 + kw;
    a.pend.budget = g->spawn_budget;
    a.pend.stats = g->work_count + 8;
    a.pend.launch_id = (uint32_t)(g->nstep % 0x7ffffffeu) + 1u;   // nonzero, differs from the neighbours'
    const int blocks = (g->E + g->plan.EPB - 1) / g->plan.EPB;
    a.pend.P = g->pend; a.pend.list = g->plist + (int64_t)kr * 4 * (g->E + 64); a.pend.count = g->work_count + 2 + kr;
    a.pend.all = g->pend_all;
    a.pend.step_blocks = blocks; a.pend.pend_blocks = g->pend_blocks; a.pend.counter_offset = g->counter_offset;
    a.pend.first = g->plan.kd ? 1 : 0;
    a.pend.waves = g->pend_waves;
    a.pend.stride = g->plan.rng_stride;
    a.pend.case_size = g->case_size;
    a.ov.row = g->rows; a.ov.NS = g->NS;
    a.pend.ov = a.ov;
    a.cth_h = cos(g->c.human_fov / 2); a.cth_r = cos(g->c.robot_fov / 2);
    g->pend_all = 0;
    const int grid = blocks + g->pend_blocks;
    const bool phx = g->c.rng_mode == CN_RNG_PHILOX;
    const int variant = (g->plan.kd ? 4 : 0) | (phx ? 2 : 0) | (g->rows ? 1 : 0);
    void (*const kern[8])(StepArgs, cn_config) = {
        cn_step_kernel<false, false, false>, cn_step_kernel<false, false, true>, cn_step_kernel<false, true, false>,
        cn_step_kernel<false, true, true>,   cn_step_kernel<true, false, false>,  cn_step_kernel<true, false, true>,
        cn_step_kernel<true, true, false>,   cn_step_kernel<true, true, true>};
    void (*const kern_dev[4])(StepArgs, cn_config) = {   // graph mode (plain engines)
        cn_step_kernel<false, false, false, true>, cn_step_kernel<false, true, false, true>,
        cn_step_kernel<true, false, false, true>, cn_step_kernel<true, true, false, true>};
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    if (g->devseq)
        hipLaunchKernelGGL(kern_dev[variant >> 1], dim3(grid), dim3(g->plan.T), g->a_lds, st, a, g->c);
    else
        hipLaunchKernelGGL(kern[variant], dim3(grid), dim3(g->plan.T), g->a_lds, st, a, g->c);
    HIPCHK(hipGetLastError());
    if (prof && ++g->prof_n == g->prof_cap) HIPCHK(hipEventRecord(g->ev[1], st));
    return CN_OK;
}

int cn_step_seq(cn_engine *g, void *stream, int T, const float *actions, int64_t action_stride, float *robot_node,
                float *temporal, float *spatial, float *reward, uint8_t *done, int8_t *event, float *info,
                double *ep_return, int32_t *ep_len)
{
    if (!g || !actions) return set_err(CN_EINVAL, "null argument");
    if (T < 0 || (T > 1 && action_stride < 2 * g->E))
        return set_err(CN_EINVAL, "cn_step_seq: T >= 0 and action_stride >= 2 * E required");
    for (int t = 0; t < T; ++t) {
        const int rc = cn_step(g, stream, actions + (int64_t)t * action_stride, robot_node, temporal, spatial, reward,
                               done, event, info, ep_return, ep_len);
        if (rc) return rc;
    }
    return CN_OK;
}

int cn_set_graph_mode(cn_engine *g, void *stream, int on)
{
    if (!g) return set_err(CN_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    if (g->ngroups || g->rows) return set_err(CN_EUNSUPPORTED, "graph mode: plain engines only (not cn_create_mixed)");
    if (on && !g->devseq) {   // hand the host sequence to the device
        g->ctl_host[0] = (uint32_t)g->nstep; g->ctl_host[1] = (uint32_t)g->pend_all; g->ctl_host[2] = 0u;
        HIPCHK(hipMemcpyAsync(g->work_count + CN_CTL_NSTEP, g->ctl_host, 3 * sizeof(uint32_t), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));   // ctl_host may be rewritten by the next call
    } else if (!on && g->devseq) {   // and back
        HIPCHK(hipMemcpyAsync(g->ctl_host, g->work_count + CN_CTL_NSTEP, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        g->nstep = g->ctl_host[0]; g->pend_all = (int)g->ctl_host[1];
    }
    g->devseq = on ? 1 : 0;
    return CN_OK;
}

int cn_state_bytes(const cn_engine *g, int64_t *bytes)
{
    if (!g || !bytes) return set_err(CN_EINVAL, "null argument");
    *bytes = g->state_bytes;
    return CN_OK;
}

const void *cn_state_device_ptr(const cn_engine *g) { return g && !g->ngroups ? g->state : nullptr; }

int cn_get_state(cn_engine *g, void *stream, void *dst, int dst_on_host)
{
    if (!g || !dst) return set_err(CN_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    if (g->ngroups) {   // the groups' blobs, concatenated in group order
        char *d = (char *)dst;
        for (int k = 0; k < g->ngroups; ++k) {
            const int rc = cn_get_state(g->grp[k], stream, d, dst_on_host);
            if (rc) return rc;
            d += g->grp[k]->state_bytes;
        }
        return CN_OK;
    }
    if (dst_on_host) {
        HIPCHK(hipMemcpyAsync(dst, g->state, g->state_bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    } else {
        HIPCHK(hipMemcpyAsync(dst, g->state, g->state_bytes, hipMemcpyDeviceToDevice, st));
    }
    return CN_OK;
}

int cn_set_state(cn_engine *g, void *stream, const void *src, int src_on_host)
{
    if (!g || !src) return set_err(CN_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    if (g->ngroups) {
        const char *d = (const char *)src;
        for (int k = 0; k < g->ngroups; ++k) {
            const int rc = cn_set_state(g->grp[k], stream, d, src_on_host);
            if (rc) return rc;
            d += g->grp[k]->state_bytes;
        }
        return CN_OK;
    }
    if (src_on_host) {
        HIPCHK(hipMemcpyAsync(g->state, src, g->state_bytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
    } else {
        HIPCHK(hipMemcpyAsync(g->state, src, g->state_bytes, hipMemcpyDeviceToDevice, st));
    }
    // pending spawns are keyed by (case_counter, reset_count); redraw them for the new state, keyed from a
    // snapshot of its counters (the next launch's own resets rewrite the state's while its spawn waves run)
    g->pend_all = PEND_BOTH;
    const int rk = keysnap(g, st);
    if (rk) return rk;
    if (g->devseq) return ctl_set(g->work_count + CN_CTL_ALL, PEND_BOTH, st);
    return CN_OK;
}

#ifdef CN_STAMPS
int cn_debug_stamps_c(unsigned long long *c, unsigned long long *p)
{
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(c, HIP_SYMBOL(cn_stamp_c), sizeof(unsigned long long) * 8192 * 4));
    HIPCHK(hipMemcpyFromSymbol(p, HIP_SYMBOL(cn_stamp_p), sizeof(unsigned long long) * 8192 * 2));
    return CN_OK;
}

// per-workgroup start / end on the device-wide 100 MHz realtime clock; spawn_env's segment stamps
int cn_debug_stamps_r(unsigned long long *r, unsigned long long *sp)
{
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(r, HIP_SYMBOL(cn_stamp_r), sizeof(unsigned long long) * 8192 * 2));
    if (sp) HIPCHK(hipMemcpyFromSymbol(sp, HIP_SYMBOL(cn_stamp_s), sizeof(unsigned long long) * 8192 * 16));
    unsigned long long l3[14];
    HIPCHK(hipMemcpyFromSymbol(l3, HIP_SYMBOL(cn_lp3_cnt), sizeof(l3)));
    for (int k = 0; k < 14; ++k) r[8192 * 2 - 14 + k] = l3[k];   // (the last workgroup slots: never a real grid here)
    return CN_OK;
}

int cn_debug_stamps(unsigned long long *a, unsigned long long *b)
{
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(a, HIP_SYMBOL(cn_stamp_a), sizeof(unsigned long long) * 4096 * CN_NSTAMP));
    HIPCHK(hipMemcpyFromSymbol(b, HIP_SYMBOL(cn_stamp_b), sizeof(unsigned long long) * 8192 * CN_NSTAMP));
    return CN_OK;
}
#endif

int cn_debug_set_spawn_budget(cn_engine *g, long long cycles)
{
    if (!g || cycles < 0) return set_err(CN_EINVAL, "cn_debug_set_spawn_budget: engine and cycles >= 0 required");
    for (int k = 0; k < g->ngroups; ++k) cn_debug_set_spawn_budget(g->grp[k], cycles);
    if (!g->ngroups && (g->plan.kd || CN_QUAD_PARK)) g->spawn_budget = cycles;   // (parking paths only)
    return CN_OK;
}

int cn_debug_spawn_stats(cn_engine *g, uint32_t *out)
{
    if (!g || !out) return set_err(CN_EINVAL, "null argument");
    for (int j = 0; j < 5; ++j) out[j] = 0;
    if (g->ngroups) {
        for (int k = 0; k < g->ngroups; ++k) {
            uint32_t v[5];
            const int rc = cn_debug_spawn_stats(g->grp[k], v);
            if (rc) return rc;
            for (int j = 0; j < 5; ++j) out[j] += v[j];
        }
        return CN_OK;
    }
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, g->work_count + 8, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out + 4, g->work_count + 15, sizeof(uint32_t), hipMemcpyDeviceToHost));
    return CN_OK;
}

int cn_lidar_obs(cn_engine *g, void *stream, const uint8_t *reset_mask, int enable, int beams, double max_range,
                 double robot_radius, float *lidar, float *obs)
{
    if (!g) return set_err(CN_EINVAL, "null engine");
    if (g->ngroups) return set_err(CN_EUNSUPPORTED, "cn_lidar_obs: not on a mixed engine");
    if (beams < 2 || beams > 4096 || !(max_range > 0) || !lidar || !obs)
        return set_err(CN_EINVAL, "cn_lidar_obs: beams in [2, 4096], max_range > 0 and buffers required");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_lidar_obs_kernel, dim3((unsigned)((g->E + 3) / 4)), dim3(256), 0, (hipStream_t)stream, g->s,
                       g->E, g->N, 0.5 * g->c.square_width, reset_mask, enable, beams, max_range, robot_radius,
                       lidar, obs);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_debug_disc_quad(void *stream, int64_t n, int mode, const double *px, const double *py, const double *r,
                       const double *qx, const double *qy, int32_t *out)
{
    if (n <= 0 || !px || !py || !r || !qx || !qy || !out) return set_err(CN_EINVAL, "cn_debug_disc_quad: n > 0 and buffers required");
    HIPCHK(circ_table_init());
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_disc_quad_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, n, mode,
                       px, py, r, qx, qy, out);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_debug_copy64(void *stream, int64_t n, int seg, const double *src, double *dst)
{
    if (n <= 0 || seg < 1 || seg > 64 || !src || !dst) return set_err(CN_EINVAL, "cn_debug_copy64: n > 0, 1 <= seg <= 64");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_copy64_kernel, dim3((unsigned)((n + seg - 1) / seg)), dim3(64), 0, (hipStream_t)stream, n, seg,
                       src, dst);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_debug_orca(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                  float time_horizon, float time_step, float *out)
{
    if (n <= 0 || !agents || !self || !out) return set_err(CN_EINVAL, "cn_debug_orca: n > 0 and buffers required");
    if (A < 1 || A > 10) return set_err(CN_EUNSUPPORTED, "cn_debug_orca: 1 <= A <= 10 (the quad path)");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_orca_kernel, dim3((unsigned)((n + 15) / 16)), dim3(64), 0, (hipStream_t)stream, n, A,
                       agents, self, neighbor_dist, time_horizon, time_step, out);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_orca_predict_kd(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                       float time_horizon, float time_step, uint8_t *perm, float *out)
{
    if (n <= 0 || !agents || !self || !out) return set_err(CN_EINVAL, "cn_orca_predict_kd: n > 0 and buffers required");
    if (A < 1 || A > CN_ORCA_MAXA) return set_err(CN_EUNSUPPORTED, "cn_orca_predict_kd: 1 <= A <= 64");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_orca_kd_kernel, dim3((unsigned)((n + 15) / 16)), dim3(64), orca_kd_lds(A), (hipStream_t)stream,
                       n, A, agents, self, neighbor_dist, time_horizon, time_step, perm, out);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_orca_predict(void *stream, int64_t n, int A, const float *agents, const float *self, float neighbor_dist,
                    float time_horizon, float time_step, float *out)
{
    if (A > 10)   // a fresh simulator per call: identity KdTree order
        return cn_orca_predict_kd(stream, n, A, agents, self, neighbor_dist, time_horizon, time_step, nullptr, out);
    return cn_debug_orca(stream, n, A, agents, self, neighbor_dist, time_horizon, time_step, out);
}

int cn_social_force_predict(void *stream, int64_t n, int M, const double *self, const double *others, double A,
                            double B, double KI, double time_step, double *out)
{
    if (n <= 0 || M < 0 || M > 64 || !self || (M && !others) || !out)
        return set_err(CN_EINVAL, "cn_social_force_predict: n > 0, 0 <= M <= 64 and buffers required");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_sf_predict_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, n, M,
                       self, others, A, B, KI, time_step, out);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

int cn_edge_features(void *stream, int64_t E, int N, const float *robot_node, const float *temporal_edges,
                     const float *spatial_edges, const float *Wt, const float *bt, const float *Ws, const float *bs,
                     const float *Wr, const float *br, const float *Wn, const float *bn, float *temporal_embed,
                     float *spatial_embed, float *node_embed)
{
    if (E <= 0 || N <= 0) return set_err(CN_EINVAL, "E, N must be > 0");
    const int64_t threads = E * (N + 2) * 16;
    const int64_t blocks = (threads + 255) / 256;
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_edge_features_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, E, N,
                       robot_node, temporal_edges, spatial_edges, Wt, bt, Ws, bs, Wr, br, Wn, bn, temporal_embed,
                       spatial_embed, node_embed);
    HIPCHK(hipGetLastError());
    return CN_OK;
}

}  // extern "C"
