/*
 * oracle/cpu_ref.c — CPU restatement of the reference CrowdSimDict hot path.
 *
 *   *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke() and bench.py's
 *   cpu_baseline leg may load this library, and only as the checker / the timed CPU baseline.
 *   The product path (crowdnav_dsrnn_amd/) never links, imports or falls back to it.
 *
 * What it restates (paths relative to the CrowdNav_DSRNN checkout, evan-tan/CrowdNav_DSRNN @ 2025-02-13):
 *   CrowdSimDict.reset / step            crowd_sim/envs/crowd_sim_dict.py:105-271
 *   CrowdSim spawn / goals / reward / FOV crowd_sim/envs/crowd_sim.py:296-393, 555-663, 724-865, 907-1161
 *   Agent kinematics                     crowd_sim/envs/utils/agent.py:44-64, 172-218
 *   SRNN.clip_action                     crowd_nav/policy/srnn.py:18-48
 *   ORCA.predict                         crowd_nav/policy/orca.py:64-139
 *   SOCIAL_FORCE.predict                 crowd_nav/policy/social_force.py:11-66
 *   numpy legacy RandomState (MT19937)   numpy 2.2 _legacy_seeding / mt19937_seed / mt19937_gen /
 *                                        mt19937_next_double / random_uniform (numpy is the reference's RNG)
 *   RVO2 v2.0 (third-party, NOT vendored in the reference; Python-RVO2 git master, unpinned per
 *   setup/full_setup.sh:40-44): RVOSimulator::doStep, KdTree::buildAgentTreeRecursive /
 *   queryAgentTreeRecursive, Agent::insertAgentNeighbor / computeNewVelocity, linearProgram1/2/3,
 *   restated from the published algorithm in float32. No RVO2 binary exists
 *   here, so the RVO2 arithmetic is PARITY UNPINNED; it is pinned by analytic known-answer tests.
 *   GEOS/shapely predicates (third-party, absent): restated analytically.
 *
 * Numerics mirror what numpy 2.2 does on the reference side (NEP 50 scalar promotion):
 *   - float64 state; np.linalg.norm of a float64 2-vector = sqrt(fma(b, b, a*a)) (OpenBLAS ddot,
 *     verified in this container), of a float32 2-vector = sqrtf(a*a + b*b) (no FMA, verified);
 *   - np.float32 (op) python-float stays float32; np.float32 (op) np.float64 goes float64;
 *   - everything else plain IEEE double, compiled with -ffp-contract=off.
 * Deviations (documented in DESIGN.md): bounded rejection sampling (max_tries);
 * the unicycle jerk/speed metrics use the commanded world-frame velocity.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/crowdnav.h"
#include "../include/crowdnav_state.h"

#define EXPORT __attribute__((visibility("default")))

static __thread char g_err[256];
static int fail(int code, const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); return code; }
EXPORT const char *cnref_last_error(void) { return g_err; }

typedef struct ref_engine {
    cn_config c;
    int E, N, A, M;      /* envs, humans, agents per RVO2 sim, observed slots per human (A-1) */
    int64_t bytes;
    void *blob;
    cn_state_ptrs s;
    int64_t case_size, counter_offset;
    int32_t *rows;       /* env e's row in a mixed engine (global index = env_offset + rows[e]); NULL: e */
} ref_engine;

/* ------------------------------------------------------------------------------------------------ */
/* numpy-compatible scalar helpers                                                                   */
/* ------------------------------------------------------------------------------------------------ */
static inline double np_norm2(double a, double b) { return sqrt(fma(b, b, a * a)); }
static inline float np_norm2f(float a, float b) { return sqrtf(a * a + b * b); }
static inline double np_dot2(double a0, double a1, double b0, double b1) { return fma(a1, b1, a0 * b0); }
static inline double np_mod(double a, double b)
{ /* numpy float64 remainder (npy_divmod) */
    double m = fmod(a, b);
    if (m != 0.0) { if ((b < 0) != (m < 0)) m += b; }
    else m = copysign(0.0, b);
    return m;
}
static inline float np_modf(float a, float b)
{ /* numpy float32 remainder */
    float m = fmodf(a, b);
    if (m != 0.0f) { if ((b < 0) != (m < 0)) m += b; }
    else m = copysignf(0.0f, b);
    return m;
}

/* numpy 2.x float32 sin/cos (umath loops_trigonometric: Cody-Waite reduction + minimax polynomials
 * with FMA, max 1.49 ulp); np.sin/np.cos on float32 scalars use it instead of libm. Verified
 * bit-exact against numpy in this container. Outside the Cody-Waite range numpy calls libm. */
static float np_sincosf(float x, int want_cos)
{
    const float max_cody = want_cos ? 71476.0625f : 117435.992f;
    if (!(fabsf(x) <= max_cody)) return want_cos ? cosf(x) : sinf(x);
    float q = x * 0x1.45f306p-1f;
    q = q + 0x1.800000p+23f;
    q = q - 0x1.800000p+23f;
    float r = fmaf(q, -0x1.921fb0p+00f, x);
    r = fmaf(q, -0x1.5110b4p-22f, r);
    r = fmaf(q, -0x1.846988p-48f, r);
    const float r2 = r * r;
    float c = fmaf(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = fmaf(c, r2, 0x1.55553cp-05f);
    c = fmaf(c, r2, -0x1.000000p-01f);
    c = fmaf(c, r2, 0x1.000000p+00f);
    float s = fmaf(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = fmaf(s, r2, 0x1.11119ap-07f);
    s = fmaf(s, r2, -0x1.555556p-03f);
    s = fmaf(s, r2, 0.0f);
    s = fmaf(s, r, r);
    int iq = (int)q + (want_cos ? 1 : 0);
    float out = (iq & 1) == 0 ? s : c;
    if ((iq & 2) == 2) out = 0.0f - out;
    return out;
}
static inline float np_sinf(float x) { return np_sincosf(x, 0); }
static inline float np_cosf(float x) { return np_sincosf(x, 1); }
static inline float np_clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ------------------------------------------------------------------------------------------------ */
/* numpy legacy MT19937                                                                              */
/* ------------------------------------------------------------------------------------------------ */
static void mt_seed(uint32_t *mt, int32_t *pos, uint32_t seed)
{
    for (int i = 0; i < CN_MT_N; ++i) {
        mt[i] = seed;
        seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
    }
    *pos = CN_MT_N;
}
static void mt_gen(uint32_t *mt)
{
    const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
    uint32_t y;
    int i;
    for (i = 0; i < CN_MT_N - 397; ++i) {
        y = (mt[i] & UP) | (mt[i + 1] & LO);
        mt[i] = mt[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & MA);
    }
    for (; i < CN_MT_N - 1; ++i) {
        y = (mt[i] & UP) | (mt[i + 1] & LO);
        mt[i] = mt[i + (397 - CN_MT_N)] ^ (y >> 1) ^ ((0u - (y & 1u)) & MA);
    }
    y = (mt[CN_MT_N - 1] & UP) | (mt[0] & LO);
    mt[CN_MT_N - 1] = mt[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & MA);
}
static uint32_t mt_next(uint32_t *mt, int32_t *pos)
{
    if (*pos >= CN_MT_N) { mt_gen(mt); *pos = 0; }
    uint32_t y = mt[(*pos)++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
static double mt_double(uint32_t *mt, int32_t *pos)
{
    int32_t a = (int32_t)(mt_next(mt, pos) >> 5), b = (int32_t)(mt_next(mt, pos) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* CN_RNG_PHILOX fast mode (include/crowdnav.h): Philox4x32-10 as published by Salmon, Moraes, Dror &
 * Shaw (SC'11) / Random123 (multipliers 0xD2511F53, 0xCD9E8D57; Weyl key bumps 0x9E3779B9, 0xBB67AE85),
 * key (episode seed, 0x43726f77), counter (word >> 2, 0, 0, 0); a double is two consecutive words with
 * numpy's random_sample conversion. Restated here independently of the HIP engine's copy. */
static void philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t x[4] = {ctr[0], ctr[1], ctr[2], ctr[3]}, k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * x[0], p1 = (uint64_t)0xCD9E8D57u * x[2];
        const uint32_t y0 = (uint32_t)(p1 >> 32) ^ x[1] ^ k0, y1 = (uint32_t)p1;
        const uint32_t y2 = (uint32_t)(p0 >> 32) ^ x[3] ^ k1, y3 = (uint32_t)p0;
        x[0] = y0; x[1] = y1; x[2] = y2; x[3] = y3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    memcpy(out, x, sizeof x);
}
EXPORT void cnref_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out)
{ /* test hook: Random123 known-answer vectors */
    philox4x32_10(ctr, key, out);
}
static double philox_double(uint32_t key, int32_t *pos)
{
    uint32_t w[4];
    const uint32_t ctr[4] = {(uint32_t)*pos >> 2, 0, 0, 0}, k[2] = {key, 0x43726f77u};
    philox4x32_10(ctr, k, w);
    const int o = *pos & 3;   /* 0 or 2: draws start at even words */
    *pos += 2;
    const int32_t a = (int32_t)(w[o] >> 5), b = (int32_t)(w[o + 1] >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* an env's stream: MT19937 key words + position, or (philox) the key in mt[0] + words drawn since reset */
typedef struct { uint32_t *mt; int32_t *pos; int philox; } rng_t;
static inline double rnd(rng_t r)                                                            /* np.random.random() */
{
    return r.philox ? philox_double(r.mt[0], r.pos) : mt_double(r.mt, r.pos);
}
static inline double unif(rng_t r, double lo, double hi) { return lo + (hi - lo) * rnd(r); } /* np.random.uniform */

EXPORT void cnref_philox_draw(uint32_t key, int n, double *out)
{ /* test hook: the first n doubles of the Philox stream of episode seed `key` */
    uint32_t mt[1] = {key};
    int32_t pos = 0;
    rng_t r = {mt, &pos, 1};
    for (int i = 0; i < n; ++i) out[i] = rnd(r);
}

EXPORT void cnref_mt_draw(uint32_t seed, int n, double *out)
{ /* test hook: np.random.seed(seed); [np.random.random() for _ in range(n)] */
    uint32_t mt[CN_MT_N];
    int32_t pos;
    mt_seed(mt, &pos, seed);
    rng_t r = {mt, &pos, 0};
    for (int i = 0; i < n; ++i) out[i] = rnd(r);
}

/* ------------------------------------------------------------------------------------------------ */
/* RVO2 v2.0 restated (float32) — agent 0 of one simulator                                           */
/* ------------------------------------------------------------------------------------------------ */
#define RVO_EPSILON 0.00001f
#define MAX_LINES 64
typedef struct { float px, py, dx, dy; } rline;

static inline float det2(float ax, float ay, float bx, float by) { return ax * by - ay * bx; }

/* linearProgram1 */
static int lp1(const rline *L, int no, float radius, float ox, float oy, int dirOpt, float *rx, float *ry)
{
    const float dot = L[no].px * L[no].dx + L[no].py * L[no].dy;
    const float disc = dot * dot + radius * radius - (L[no].px * L[no].px + L[no].py * L[no].py);
    if (disc < 0.0f) return 0;
    const float sd = sqrtf(disc);
    float tL = -dot - sd, tR = -dot + sd;
    for (int i = 0; i < no; ++i) {
        const float den = det2(L[no].dx, L[no].dy, L[i].dx, L[i].dy);
        const float num = det2(L[i].dx, L[i].dy, L[no].px - L[i].px, L[no].py - L[i].py);
        if (fabsf(den) <= RVO_EPSILON) {
            if (num < 0.0f) return 0;
            continue;
        }
        const float t = num / den;
        if (den >= 0.0f) tR = (t < tR) ? t : tR;   /* std::min(tRight, t) */
        else tL = (tL < t) ? t : tL;               /* std::max(tLeft, t) */
        if (tL > tR) return 0;
    }
    if (dirOpt) {
        if (ox * L[no].dx + oy * L[no].dy > 0.0f) { *rx = L[no].px + tR * L[no].dx; *ry = L[no].py + tR * L[no].dy; }
        else { *rx = L[no].px + tL * L[no].dx; *ry = L[no].py + tL * L[no].dy; }
    } else {
        const float t = L[no].dx * (ox - L[no].px) + L[no].dy * (oy - L[no].py);
        if (t < tL) { *rx = L[no].px + tL * L[no].dx; *ry = L[no].py + tL * L[no].dy; }
        else if (t > tR) { *rx = L[no].px + tR * L[no].dx; *ry = L[no].py + tR * L[no].dy; }
        else { *rx = L[no].px + t * L[no].dx; *ry = L[no].py + t * L[no].dy; }
    }
    return 1;
}

/* linearProgram2: returns n on success, else the failing line index */
static int lp2(const rline *L, int n, float radius, float ox, float oy, int dirOpt, float *rx, float *ry)
{
    if (dirOpt) { *rx = ox * radius; *ry = oy * radius; }
    else if (ox * ox + oy * oy > radius * radius) {
        const float len = sqrtf(ox * ox + oy * oy);
        const float inv = 1.0f / len;
        *rx = (ox * inv) * radius; *ry = (oy * inv) * radius;
    } else { *rx = ox; *ry = oy; }
    for (int i = 0; i < n; ++i) {
        if (det2(L[i].dx, L[i].dy, L[i].px - *rx, L[i].py - *ry) > 0.0f) {
            const float tx = *rx, ty = *ry;
            if (!lp1(L, i, radius, ox, oy, dirOpt, rx, ry)) { *rx = tx; *ry = ty; return i; }
        }
    }
    return n;
}

static long long g_cnt_lp2 = 0, g_cnt_lp3 = 0, g_cnt_lines = 0;
EXPORT void cnref_debug_counters(long long *out) { out[0] = g_cnt_lp2; out[1] = g_cnt_lp3; out[2] = g_cnt_lines; }

/* linearProgram3 (numObstLines = 0) */
static void lp3(const rline *L, int n, int begin, float radius, float *rx, float *ry)
{
    float distance = 0.0f;
    rline proj[MAX_LINES];
    for (int i = begin; i < n; ++i) {
        if (det2(L[i].dx, L[i].dy, L[i].px - *rx, L[i].py - *ry) > distance) {
            int np_ = 0;
            for (int j = 0; j < i; ++j) {
                rline ln;
                const float determinant = det2(L[i].dx, L[i].dy, L[j].dx, L[j].dy);
                if (fabsf(determinant) <= RVO_EPSILON) {
                    if (L[i].dx * L[j].dx + L[i].dy * L[j].dy > 0.0f) continue;
                    ln.px = 0.5f * (L[i].px + L[j].px);
                    ln.py = 0.5f * (L[i].py + L[j].py);
                } else {
                    const float s = det2(L[j].dx, L[j].dy, L[i].px - L[j].px, L[i].py - L[j].py) / determinant;
                    ln.px = L[i].px + s * L[i].dx;
                    ln.py = L[i].py + s * L[i].dy;
                }
                const float ddx = L[j].dx - L[i].dx, ddy = L[j].dy - L[i].dy;
                const float len = sqrtf(ddx * ddx + ddy * ddy);
                const float inv = 1.0f / len;
                ln.dx = ddx * inv; ln.dy = ddy * inv;
                proj[np_++] = ln;
            }
            const float tx = *rx, ty = *ry;
            if (lp2(proj, np_, radius, -L[i].dy, L[i].dx, 1, rx, ry) < np_) { *rx = tx; *ry = ty; }
            distance = det2(L[i].dx, L[i].dy, L[i].px - *rx, L[i].py - *ry);
        }
    }
}

/* KdTree (MAX_LEAF_SIZE 10) over the simulator's agents; `perm` is KdTree::agents_ (persists). */
#define KD_MAX_NODES 128
typedef struct { int begin, end, left, right; float minX, maxX, minY, maxY; } kdnode;

static void kd_build(kdnode *T, uint8_t *perm, const float *X, const float *Y, int begin, int end, int node)
{
    T[node].begin = begin; T[node].end = end;
    T[node].minX = T[node].maxX = X[perm[begin]];
    T[node].minY = T[node].maxY = Y[perm[begin]];
    for (int i = begin + 1; i < end; ++i) {
        const float x = X[perm[i]], y = Y[perm[i]];
        T[node].maxX = T[node].maxX < x ? x : T[node].maxX;  /* std::max(maxX, x) */
        T[node].minX = x < T[node].minX ? x : T[node].minX;  /* std::min(minX, x) */
        T[node].maxY = T[node].maxY < y ? y : T[node].maxY;
        T[node].minY = y < T[node].minY ? y : T[node].minY;
    }
    if (end - begin > 10) {
        const int vert = (T[node].maxX - T[node].minX > T[node].maxY - T[node].minY);
        const float split = vert ? 0.5f * (T[node].maxX + T[node].minX) : 0.5f * (T[node].maxY + T[node].minY);
        int left = begin, right = end;
        while (left < right) {
            while (left < right && (vert ? X[perm[left]] : Y[perm[left]]) < split) ++left;
            while (right > left && (vert ? X[perm[right - 1]] : Y[perm[right - 1]]) >= split) --right;
            if (left < right) {
                uint8_t t = perm[left]; perm[left] = perm[right - 1]; perm[right - 1] = t;
                ++left; --right;
            }
        }
        if (left == begin) { ++left; ++right; }
        T[node].left = node + 1;
        T[node].right = node + 2 * (left - begin);
        kd_build(T, perm, X, Y, begin, left, T[node].left);
        kd_build(T, perm, X, Y, left, end, T[node].right);
    }
}

typedef struct { float distSq; int agent; } nbr;

static void insert_nbr(nbr *nb, int *cnt, int maxN, int agent, const float *X, const float *Y, float *rangeSq)
{
    if (agent == 0) return;
    const float dx = X[0] - X[agent], dy = Y[0] - Y[agent];
    const float distSq = dx * dx + dy * dy;
    if (distSq < *rangeSq) {
        if (*cnt < maxN) nb[(*cnt)++] = (nbr){distSq, agent};
        int i = *cnt - 1;
        while (i != 0 && distSq < nb[i - 1].distSq) { nb[i] = nb[i - 1]; --i; }
        nb[i] = (nbr){distSq, agent};
        if (*cnt == maxN) *rangeSq = nb[*cnt - 1].distSq;
    }
}

static float sqrf(float x) { return x * x; }
static float pos0(float v) { return (0.0f < v) ? v : 0.0f; }   /* std::max(0.0f, v) */

static void kd_query(const kdnode *T, const uint8_t *perm, const float *X, const float *Y, int node,
                     nbr *nb, int *cnt, int maxN, float *rangeSq)
{
    if (T[node].end - T[node].begin <= 10) {
        for (int i = T[node].begin; i < T[node].end; ++i) insert_nbr(nb, cnt, maxN, perm[i], X, Y, rangeSq);
        return;
    }
    const kdnode *l = &T[T[node].left], *r = &T[T[node].right];
    const float x = X[0], y = Y[0];
    const float dl = sqrf(pos0(l->minX - x)) + sqrf(pos0(x - l->maxX)) +
                     sqrf(pos0(l->minY - y)) + sqrf(pos0(y - l->maxY));
    const float dr = sqrf(pos0(r->minX - x)) + sqrf(pos0(x - r->maxX)) +
                     sqrf(pos0(r->minY - y)) + sqrf(pos0(y - r->maxY));
    if (dl < dr) {
        if (dl < *rangeSq) {
            kd_query(T, perm, X, Y, T[node].left, nb, cnt, maxN, rangeSq);
            if (dr < *rangeSq) kd_query(T, perm, X, Y, T[node].right, nb, cnt, maxN, rangeSq);
        }
    } else {
        if (dr < *rangeSq) {
            kd_query(T, perm, X, Y, T[node].right, nb, cnt, maxN, rangeSq);
            if (dl < *rangeSq) kd_query(T, perm, X, Y, T[node].left, nb, cnt, maxN, rangeSq);
        }
    }
}

/*
 * One RVO2 doStep, agent 0's new velocity.  Agents 0..A-1 with float32 position/velocity/radius;
 * agent 0 has maxSpeed `vmax` and preferred velocity (prefx, prefy). `perm` (A entries) is the
 * persisted KdTree::agents_ order, used only when A > 10. neighborDist, maxNeighbors = A-1,
 * timeHorizon, timeStep as in orca.py:79-84.
 */
static void rvo2_agent0(int A, const float *X, const float *Y, const float *VX, const float *VY, const float *R,
                        float vmax, float prefx, float prefy, float neighborDist, float timeHorizon,
                        float timeStep, uint8_t *perm, float *outx, float *outy)
{
    nbr nb[MAX_LINES];
    int cnt = 0;
    float rangeSq = neighborDist * neighborDist;
    const int maxN = A - 1;
    if (maxN > 0) {
        if (A > 10) {
            kdnode T[KD_MAX_NODES];
            kd_build(T, perm, X, Y, 0, A, 0);
            kd_query(T, perm, X, Y, 0, nb, &cnt, maxN, &rangeSq);
        } else {
            for (int a = 0; a < A; ++a) insert_nbr(nb, &cnt, maxN, a, X, Y, &rangeSq);
        }
    }
    rline L[MAX_LINES];
    const float invTH = 1.0f / timeHorizon;
    for (int k = 0; k < cnt; ++k) {
        const int o = nb[k].agent;
        const float rpx = X[o] - X[0], rpy = Y[o] - Y[0];
        const float rvx = VX[0] - VX[o], rvy = VY[0] - VY[o];
        const float distSq = rpx * rpx + rpy * rpy;
        const float cr = R[0] + R[o];
        const float crSq = cr * cr;
        float ux, uy;
        rline ln;
        if (distSq > crSq) {
            const float wx = rvx - invTH * rpx, wy = rvy - invTH * rpy;
            const float wLenSq = wx * wx + wy * wy;
            const float dot1 = wx * rpx + wy * rpy;
            if (dot1 < 0.0f && dot1 * dot1 > crSq * wLenSq) {
                const float wLen = sqrtf(wLenSq);
                const float inv = 1.0f / wLen;
                const float uwx = wx * inv, uwy = wy * inv;
                ln.dx = uwy; ln.dy = -uwx;
                const float s = cr * invTH - wLen;
                ux = s * uwx; uy = s * uwy;
            } else {
                const float leg = sqrtf(distSq - crSq);
                const float inv = 1.0f / distSq;
                if (det2(rpx, rpy, wx, wy) > 0.0f) {
                    ln.dx = (rpx * leg - rpy * cr) * inv;
                    ln.dy = (rpx * cr + rpy * leg) * inv;
                } else {
                    ln.dx = -((rpx * leg + rpy * cr) * inv);
                    ln.dy = -((-rpx * cr + rpy * leg) * inv);
                }
                const float dot2 = rvx * ln.dx + rvy * ln.dy;
                ux = dot2 * ln.dx - rvx; uy = dot2 * ln.dy - rvy;
            }
        } else {
            const float invTS = 1.0f / timeStep;
            const float wx = rvx - invTS * rpx, wy = rvy - invTS * rpy;
            const float wLen = sqrtf(wx * wx + wy * wy);
            const float inv = 1.0f / wLen;
            const float uwx = wx * inv, uwy = wy * inv;
            ln.dx = uwy; ln.dy = -uwx;
            const float s = cr * invTS - wLen;
            ux = s * uwx; uy = s * uwy;
        }
        ln.px = VX[0] + 0.5f * ux;
        ln.py = VY[0] + 0.5f * uy;
        L[k] = ln;
    }
    float rx, ry;
    const int fail_at = lp2(L, cnt, vmax, prefx, prefy, 0, &rx, &ry);
    __atomic_add_fetch(&g_cnt_lp2, 1, __ATOMIC_RELAXED);
    __atomic_add_fetch(&g_cnt_lines, cnt, __ATOMIC_RELAXED);
    if (fail_at < cnt) { lp3(L, cnt, fail_at, vmax, &rx, &ry); __atomic_add_fetch(&g_cnt_lp3, 1, __ATOMIC_RELAXED); }
    *outx = rx; *outy = ry;
}

EXPORT void cnref_rvo2_agent0(int A, const float *X, const float *Y, const float *VX, const float *VY,
                              const float *R, float vmax, float prefx, float prefy, float neighborDist,
                              float timeHorizon, float timeStep, uint8_t *perm, float *out)
{ /* test hook for analytic known-answer tests */
    uint8_t id[64];
    if (!perm) { for (int a = 0; a < A; ++a) id[a] = (uint8_t)a; perm = id; }
    rvo2_agent0(A, X, Y, VX, VY, R, vmax, prefx, prefy, neighborDist, timeHorizon, timeStep, perm, &out[0], &out[1]);
}

/* ------------------------------------------------------------------------------------------------ */
/* env helpers                                                                                       */
/* ------------------------------------------------------------------------------------------------ */
#define H(f, e, i) (g->s.f[(int64_t)(e) * g->N + (i)])
#define R1(f, e) (g->s.f[(e)])

/* CrowdSim.detect_visible (crowd_sim.py:820-847): is agent 2 in agent 1's FOV. `holo` is
 * self.robot.kinematics == 'holonomic' (used even when agent 1 is a human). */
static int detect_visible(int holo, double vx1, double vy1, double th1, double px1, double py1,
                          double px2, double py2, double fov)
{
    const double real_theta = holo ? atan2(vy1, vx1) : th1;
    double fx = cos(real_theta), fy = sin(real_theta);
    double vx = px2 - px1, vy = py2 - py1;
    const double nf = np_norm2(fx, fy), nv = np_norm2(vx, vy);
    fx = fx / nf; fy = fy / nf;
    vx = vx / nv; vy = vy / nv;
    double d = np_dot2(fx, fy, vx, vy);
    if (d != d) return 0;                    /* np.clip(nan) -> nan, arccos(nan) -> nan: not visible */
    d = d < -1.0 ? -1.0 : (d > 1.0 ? 1.0 : d);
    const double offset = acos(d);
    return fabs(offset) <= fov / 2;
}

/* detect_visible(self.robot, human, robot1=True): once the robot's velocity/theta are np.float32
 * (CN_FLAG_ROBOT_F32) the FOV direction is computed in float32 (np.arctan2/np.cos on float32 scalars,
 * float32 norm), then promoted to float64 for the dot with the float64 offset vector. */
static int robot_sees(ref_engine *g, int e, double px2, double py2)
{
    const int holo = g->c.kinematics == CN_HOLONOMIC;
    if (!(R1(flags, e) & CN_FLAG_ROBOT_F32))
        return detect_visible(holo, R1(r_vx, e), R1(r_vy, e), R1(r_theta, e), R1(r_px, e), R1(r_py, e), px2, py2,
                              g->c.robot_fov);
    const float th = holo ? atan2f((float)R1(r_vy, e), (float)R1(r_vx, e)) : (float)R1(r_theta, e);
    float fx = np_cosf(th), fy = np_sinf(th);
    const float nf = np_norm2f(fx, fy);
    fx = fx / nf; fy = fy / nf;
    double vx = px2 - R1(r_px, e), vy = py2 - R1(r_py, e);
    const double nv = np_norm2(vx, vy);
    vx = vx / nv; vy = vy / nv;
    double d = np_dot2((double)fx, (double)fy, vx, vy);
    if (d != d) return 0;
    d = d < -1.0 ? -1.0 : (d > 1.0 ? 1.0 : d);
    return fabs(acos(d)) <= g->c.robot_fov / 2;
}

/* The robot/human observation seen by human i of slot k (index order, crowd_sim.py:1121-1161). */
typedef struct { double px, py, vx, vy, r; int dummy; } obs_t;

static void human_obs(ref_engine *g, int e, int i, obs_t *o /* [M] */)
{
    const int N = g->N, holo = g->c.kinematics == CN_HOLONOMIC;
    int k = 0;
    for (int j = 0; j < N; ++j) {
        if (j == i) continue;
        const int vis = detect_visible(holo, H(h_vx, e, i), H(h_vy, e, i), H(h_theta, e, i), H(h_px, e, i),
                                       H(h_py, e, i), H(h_px, e, j), H(h_py, e, j), g->c.human_fov);
        if (vis) o[k] = (obs_t){H(h_px, e, j), H(h_py, e, j), H(h_vx, e, j), H(h_vy, e, j), H(h_r, e, j), 0};
        else o[k] = (obs_t){7.0, 7.0, 0.0, 0.0, g->c.human_radius, 1};  /* dummy_human, crowd_sim.py:161-164 */
        ++k;
    }
    if (g->c.robot_visible) {
        const int vis = detect_visible(holo, H(h_vx, e, i), H(h_vy, e, i), H(h_theta, e, i), H(h_px, e, i),
                                       H(h_py, e, i), R1(r_px, e), R1(r_py, e), g->c.human_fov);
        if (vis) o[k] = (obs_t){R1(r_px, e), R1(r_py, e), R1(r_vx, e), R1(r_vy, e), R1(r_radius, e), 0};
        else o[k] = (obs_t){7.0, 7.0, 0.0, 0.0, g->c.robot_radius, 1};  /* dummy_robot, crowd_sim.py:166-170 */
    }
}

/* ORCA.predict (orca.py:64-139) for human i given its observation; returns the new velocity. */
static void orca_predict(ref_engine *g, int e, int i, const obs_t *o, double *nvx, double *nvy)
{
    const int A = g->A, M = g->M;
    float X[64], Y[64], VX[64], VY[64], R[64];
    X[0] = (float)H(h_px, e, i); Y[0] = (float)H(h_py, e, i);
    VX[0] = (float)H(h_vx, e, i); VY[0] = (float)H(h_vy, e, i);
    R[0] = g->s.o_r[(int64_t)e * g->N + i];
    const uint32_t dm = g->s.o_dmask[(int64_t)e * g->N + i];
    const float rdummy = (float)(g->c.human_radius + 0.01 + g->c.orca_safety_space);
    for (int k = 0; k < M; ++k) {
        X[k + 1] = (float)o[k].px; Y[k + 1] = (float)o[k].py;
        VX[k + 1] = (float)o[k].vx; VY[k + 1] = (float)o[k].vy;
        if (k < g->N - 1) {
            const int j = k < i ? k : k + 1;
            R[k + 1] = ((dm >> k) & 1u) ? rdummy : g->s.o_r[(int64_t)e * g->N + j];
        } else {
            R[k + 1] = ((dm >> k) & 1u) ? (float)(g->c.robot_radius + 0.01 + g->c.orca_safety_space)
                                        : (float)(R1(r_radius, e) + 0.01 + g->c.orca_safety_space);
        }
    }
    /* preferred velocity: unit vector towards goal only if farther than 1 (orca.py:118-122) */
    double dx = H(h_gx, e, i) - H(h_px, e, i), dy = H(h_gy, e, i) - H(h_py, e, i);
    const double speed = np_norm2(dx, dy);
    if (speed > 1.0) { dx = dx / speed; dy = dy / speed; }
    uint8_t *perm = A > 10 ? &g->s.o_perm[((int64_t)e * g->N + i) * A] : NULL;
    uint8_t id[64];
    if (!perm) { for (int a = 0; a < A; ++a) id[a] = (uint8_t)a; perm = id; }
    float rx, ry;
    rvo2_agent0(A, X, Y, VX, VY, R, g->s.o_vmax[(int64_t)e * g->N + i], (float)dx, (float)dy,
                (float)g->c.orca_neighbor_dist, (float)g->c.orca_time_horizon, (float)g->c.time_step, perm, &rx, &ry);
    *nvx = (double)rx; *nvy = (double)ry;
}

/* SOCIAL_FORCE.predict (social_force.py:11-66). */
static void sf_predict(ref_engine *g, int e, int i, const obs_t *o, double *nvx, double *nvy)
{
    const double px = H(h_px, e, i), py = H(h_py, e, i), vx = H(h_vx, e, i), vy = H(h_vy, e, i);
    const double vpref = H(h_vpref, e, i), r = H(h_r, e, i);
    double dx = H(h_gx, e, i) - px, dy = H(h_gy, e, i) - py;
    const double dist = sqrt(dx * dx + dy * dy);
    const double dvx = (dx / dist) * vpref, dvy = (dy / dist) * vpref;
    const double cdx = g->c.sf_KI * (dvx - vx), cdy = g->c.sf_KI * (dvy - vy);
    double ix = 0.0, iy = 0.0;
    for (int k = 0; k < g->M; ++k) {
        const double ddx = px - o[k].px, ddy = py - o[k].py;
        const double d = sqrt(ddx * ddx + ddy * ddy);
        ix += g->c.sf_A * exp((r + o[k].r - d) / g->c.sf_B) * (ddx / d);
        iy += g->c.sf_A * exp((r + o[k].r - d) / g->c.sf_B) * (ddy / d);
    }
    const double tx = (cdx + ix) * g->c.time_step, ty = (cdy + iy) * g->c.time_step;
    const double nx = vx + tx, ny = vy + ty;
    const double n = np_norm2(nx, ny);
    if (n > vpref) { *nvx = nx / n * vpref; *nvy = ny / n * vpref; }
    else { *nvx = nx; *nvy = ny; }
}

/* ---- shapely/GEOS predicates, restated analytically; parity unpinned ------------- */

/* VelocityRectangle (helper.py:199-231) corners: box(-w/2,-l/2,w/2,l/2) -> translate(0,l/2)
 * -> rotate(heading - pi/2 about origin) -> translate(front point). `f32`: the agent's velocity holds
 * np.float32 values, so heading / front offset are float32 (np.arctan2, np.cos on float32). */
static void vel_rect(double px, double py, double vx, double vy, double r, int f32, double *cx, double *cy)
{
    const double w = 2 * r * 1;
    double len, heading, dth, xos, yos;
    if (f32) {
        const float fvx = (float)vx, fvy = (float)vy;
        len = (double)(3.0f * sqrtf(fvx * fvx + fvy * fvy));
        const float h = atan2f(fvy, fvx);
        heading = h;
        dth = (double)(h - (float)(M_PI / 2));
        xos = px + (double)((float)r * np_cosf(h));
        yos = py + (double)((float)r * np_sinf(h));
    } else {
        len = 3 * sqrt(vx * vx + vy * vy);
        heading = atan2(vy, vx);
        dth = heading - M_PI / 2;
        xos = px + r * cos(heading);
        yos = py + r * sin(heading);
    }
    double c = cos(dth), s = sin(dth);
    if (fabs(c) < 2.5e-16) c = 0.0;   /* shapely.affinity.rotate snapping */
    if (fabs(s) < 2.5e-16) s = 0.0;
    const double bx[4] = {w / 2, w / 2, -w / 2, -w / 2};
    const double by0[4] = {-len / 2, len / 2, len / 2, -len / 2};
    for (int k = 0; k < 4; ++k) {
        const double x = bx[k], y = by0[k] + len / 2;
        cx[k] = (c * x - s * y) + xos;
        cy[k] = (s * x + c * y) + yos;
    }
}

/* closed-set intersection of two convex quads (possibly degenerate): separating-axis test over
 * the edge normals and edge directions of both. */
static int quads_intersect(const double *ax, const double *ay, const double *bx, const double *by)
{
    for (int p = 0; p < 2; ++p) {
        const double *qx = p ? bx : ax, *qy = p ? by : ay;
        for (int k = 0; k < 4; ++k) {
            const double ex = qx[(k + 1) & 3] - qx[k], ey = qy[(k + 1) & 3] - qy[k];
            if (ex == 0.0 && ey == 0.0) continue;
            for (int t = 0; t < 2; ++t) {
                const double nx = t ? ex : -ey, ny = t ? ey : ex;
                double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
                for (int v = 0; v < 4; ++v) {
                    const double pa = ax[v] * nx + ay[v] * ny, pb = bx[v] * nx + by[v] * ny;
                    amin = pa < amin ? pa : amin; amax = pa > amax ? pa : amax;
                    bmin = pb < bmin ? pb : bmin; bmax = pb > bmax ? pb : bmax;
                }
                if (amax < bmin || bmax < amin) return 0;
            }
        }
    }
    return 1;
}

/* check_inside_world (helper.py:42-55) with the robot disc as GEOS's 64-gon buffer: a wall segment
 * touches the polygon iff the disc's extreme vertex reaches the wall line (touching counts). */
static int inside_world(double px, double py, double r, double half)
{
    const int right = (px + r >= half) && (px - r <= half);
    const int left = (px - r <= -half) && (px + r >= -half);
    const int top = (py + r >= half) && (py - r <= half);
    const int bottom = (py - r <= -half) && (py + r >= -half);
    return !(right || left || top || bottom);
}

/* NormZoneRectangle (helper.py:234-280) for the robot; lhs/rhs, left/right side. */
static void norm_zone(double px, double py, double vx, double vy, double r, int f32, int lhs, int left, double *cx,
                      double *cy)
{
    const double w = 2 * r * 1.5, len = 1.5 * 1.2;
    double dth, xos, yos;
    if (f32) {
        const float h = atan2f((float)vy, (float)vx);
        dth = (double)(h - (float)(M_PI / 2));
        xos = px + (double)((float)r * np_cosf(h));
        yos = py + (double)((float)r * np_sinf(h));
    } else {
        const double heading = atan2(vy, vx);
        dth = heading - M_PI / 2;
        xos = px + r * cos(heading);
        yos = py + r * sin(heading);
    }
    double tx, ty;
    if (lhs) { if (left) { tx = -w / 2; ty = len / 2 + 0.6; } else { tx = w / 2; ty = len / 2; } }
    else { if (left) { tx = -w / 2; ty = len / 2; } else { tx = w / 2; ty = len / 2 + 0.6; } }
    double c = cos(dth), s = sin(dth);
    if (fabs(c) < 2.5e-16) c = 0.0;
    if (fabs(s) < 2.5e-16) s = 0.0;
    const double bx[4] = {w / 2, w / 2, -w / 2, -w / 2};
    const double by[4] = {-len / 2, len / 2, len / 2, -len / 2};
    for (int k = 0; k < 4; ++k) {
        const double x = bx[k] + tx, y = by[k] + ty;
        cx[k] = (c * x - s * y) + xos;
        cy[k] = (s * x + c * y) + yos;
    }
}

/* disc 64-gon (GEOS buffer, quad_segs 16) vs convex quad: SAT over quad edge normals and the
 * polygon's 64 edge normals. */
static int disc_quad_intersect(double px, double py, double r, const double *qx, const double *qy)
{
    double vx[64], vy[64];
    for (int k = 0; k < 64; ++k) {
        const double ang = -(k * (M_PI / 2 / 16));
        vx[k] = px + r * cos(ang);
        vy[k] = py + r * sin(ang);
    }
    vx[0] = px + r; vy[0] = py;
    for (int p = 0; p < 2; ++p) {
        const int nv = p ? 64 : 4;
        const double *ex_ = p ? vx : qx, *ey_ = p ? vy : qy;
        for (int k = 0; k < nv; ++k) {
            const double ex = ex_[(k + 1) % nv] - ex_[k], ey = ey_[(k + 1) % nv] - ey_[k];
            if (ex == 0.0 && ey == 0.0) continue;
            const double nx = -ey, ny = ex;
            double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
            for (int v = 0; v < 64; ++v) { const double t = vx[v] * nx + vy[v] * ny; amin = t < amin ? t : amin; amax = t > amax ? t : amax; }
            for (int v = 0; v < 4; ++v) { const double t = qx[v] * nx + qy[v] * ny; bmin = t < bmin ? t : bmin; bmax = t > bmax ? t : bmax; }
            if (amax < bmin || bmax < amin) return 0;
        }
    }
    return 1;
}

/* test hook: the predicate above on n cases (tests/test_norm_zone.py checks the GPU's against it) */
EXPORT void cnref_disc_quad(int64_t n, const double *px, const double *py, const double *r, const double *qx,
                            const double *qy, int32_t *out)
{
    for (int64_t i = 0; i < n; ++i) out[i] = disc_quad_intersect(px[i], py[i], r[i], qx + 4 * i, qy + 4 * i);
}

/* test hook: the robot's norm-zone penalty predicate (both zones, crowd_sim.py:918-926,957-960) on n cases */
EXPORT void cnref_norm_zone_violation(int64_t n, const double *px, const double *py, const double *vx, const double *vy,
                                      const double *r, const int32_t *f32, int32_t lhs, int32_t *out)
{
    for (int64_t i = 0; i < n; ++i) {
        int v = 0;
        for (int z = 0; z < 2 && !v; ++z) {
            double qx[4], qy[4];
            norm_zone(px[i], py[i], vx[i], vy[i], r[i], f32[i], lhs, z == 0, qx, qy);
            v = disc_quad_intersect(px[i], py[i], r[i], qx, qy);
        }
        out[i] = v;
    }
}

/* test hook: how far the robot's norm-zone predicate is from its decision boundary. For each of the two
 * zones (norm_zone, crowd_sim.py:918-926) the separating-axis gap between the robot's 64-gon and the zone
 * over all 68 unit edge normals (> 0 separated by that distance, <= 0 overlapping: max over axes of the
 * gap); returns the zone value closest to 0 in magnitude. A GPU/oracle disagreement on the penalty is
 * legitimate only when this is within rounding of 0 (the zone corner touches the disc). */
EXPORT double cnref_norm_zone_margin(double px, double py, double vx, double vy, double r, int f32, int lhs)
{
    double best = INFINITY;
    for (int z = 0; z < 2; ++z) {
        double qx[4], qy[4], vxs[64], vys[64];
        norm_zone(px, py, vx, vy, r, f32, lhs, z == 0, qx, qy);
        for (int k = 0; k < 64; ++k) {
            const double ang = -(k * (M_PI / 2 / 16));
            vxs[k] = px + r * cos(ang);
            vys[k] = py + r * sin(ang);
        }
        vxs[0] = px + r; vys[0] = py;
        double gap = -INFINITY;
        for (int p = 0; p < 2; ++p) {
            const int nv = p ? 64 : 4;
            const double *ex_ = p ? vxs : qx, *ey_ = p ? vys : qy;
            for (int k = 0; k < nv; ++k) {
                const double ex = ex_[(k + 1) % nv] - ex_[k], ey = ey_[(k + 1) % nv] - ey_[k];
                const double len = sqrt(ex * ex + ey * ey);
                if (len == 0.0) continue;
                const double nx = -ey / len, ny = ex / len;
                double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
                for (int v = 0; v < 64; ++v) { const double t = vxs[v] * nx + vys[v] * ny; amin = t < amin ? t : amin; amax = t > amax ? t : amax; }
                for (int v = 0; v < 4; ++v) { const double t = qx[v] * nx + qy[v] * ny; bmin = t < bmin ? t : bmin; bmax = t > bmax ? t : bmax; }
                const double g1 = bmin - amax, g2 = amin - bmax;
                const double gg = g1 > g2 ? g1 : g2;
                gap = gg > gap ? gg : gap;
            }
        }
        if (fabs(gap) < fabs(best)) best = gap;
    }
    return best;
}

/* ------------------------------------------------------------------------------------------------ */
/* spawn (crowd_sim.py:296-393, 555-663)                                                             */
/* ------------------------------------------------------------------------------------------------ */
static double rand_world_pt(ref_engine *g, rng_t r) { return (rnd(r) - 0.5) * g->c.square_width / 2; }

/* create_agent_attributes: returns px, py, gx, gy, heading, v_pref */
static void create_agent_attributes(ref_engine *g, int e, rng_t r, int scenario, double agent_vpref, double agent_radius,
                                    double *px, double *py, double *gx, double *gy, double *heading, double *vp)
{
    double v_pref = agent_vpref == 0 ? 1.0 : agent_vpref;
    const double pxn = (rnd(r) - 0.5) * v_pref;
    const double pyn = (rnd(r) - 0.5) * v_pref;
    const double R = g->c.circle_radius;
    *heading = 0;
    switch (scenario) {
    case CN_SC_CIRCLE_CROSSING: {
        const double angle = rnd(r) * M_PI * 2;
        *px = R * cos(angle) + pxn; *py = R * sin(angle) + pyn;
        *gx = -*px; *gy = -*py;
    } break;
    case CN_SC_SQUARE_CROSSING:
        *px = rand_world_pt(g, r) * 0.4 + pxn;
        *py = rand_world_pt(g, r) * 0.4 + pyn;
        *gx = rand_world_pt(g, r) * 0.4 + pxn;
        *gy = rand_world_pt(g, r) * 0.4 + pyn;
        break;
    case CN_SC_PARALLEL_TRAFFIC: {
        const double sign = rnd(r) >= 0.5 ? 1 : -1;
        *px = rand_world_pt(g, r) * 0.4 + pxn;
        *py = sign * (rnd(r) * 3 + 1 + pyn);
        *gx = *px; *gy = -*py;
    } break;
    case CN_SC_PERPENDICULAR_TRAFFIC: {
        const double sign = rnd(r) >= 0.5 ? 1 : -1;
        *px = sign * (rnd(r) * 3 + 1 + pxn);
        *gx = -*px;
        *py = rand_world_pt(g, r) * 0.4 + pyn;
        *gy = *py;
    } break;
    case CN_SC_SIDE_PREF_PASSING:
    case CN_SC_SIDE_PREF_OVERTAKING: {
        const double min_x = -(R1(r_radius, e) + agent_radius), max_x = -min_x;
        const double hx = (max_x - min_x) * rnd(r) + min_x;
        *px = hx; *gx = hx;
        if (scenario == CN_SC_SIDE_PREF_PASSING) { *py = R; *gy = -R; *heading = -M_PI / 2; }
        else { *py = -R + 2; *gy = R + 2; *heading = M_PI / 2; v_pref = 0.3; }
    } break;
    default: { /* side_pref_crossing */
        const double min_x = -(R + R1(r_radius, e) + agent_radius), max_x = -(R - R1(r_radius, e) - agent_radius);
        const double hx = (max_x - min_x) * rnd(r) + min_x;
        *px = hx; *gx = -hx; *py = 0; *gy = 0;
    } break;
    }
    *vp = v_pref;
}

/* update_last_human_states + generate_ob (crowd_sim_dict.py:72-103, crowd_sim.py:429-455, 851-865) */
static void gen_obs(ref_engine *g, int e, int reset, float *robot_node, float *temporal, float *spatial)
{
    const int N = g->N;
    for (int i = 0; i < N; ++i) {
        const int vis = robot_sees(g, e, H(h_px, e, i), H(h_py, e, i));
        if (vis) {
            H(b_px, e, i) = H(h_px, e, i); H(b_py, e, i) = H(h_py, e, i);
            H(b_vx, e, i) = H(h_vx, e, i); H(b_vy, e, i) = H(h_vy, e, i); H(b_r, e, i) = H(h_r, e, i);
        } else if (reset) {
            H(b_px, e, i) = 15.0; H(b_py, e, i) = 15.0; H(b_vx, e, i) = 0.0; H(b_vy, e, i) = 0.0; H(b_r, e, i) = 0.3;
        } else {
            H(b_px, e, i) = H(b_px, e, i) + H(b_vx, e, i) * g->c.time_step;
            H(b_py, e, i) = H(b_py, e, i) + H(b_vy, e, i) * g->c.time_step;
        }
    }
    if (robot_node) {
        float *rn = robot_node + (int64_t)e * 7;
        rn[0] = (float)R1(r_px, e); rn[1] = (float)R1(r_py, e); rn[2] = (float)R1(r_radius, e);
        rn[3] = (float)R1(r_gx, e); rn[4] = (float)R1(r_gy, e); rn[5] = (float)R1(r_vpref, e);
        rn[6] = (float)R1(r_theta, e);
        temporal[(int64_t)e * 2] = (float)R1(r_vx, e); temporal[(int64_t)e * 2 + 1] = (float)R1(r_vy, e);
        for (int i = 0; i < N; ++i) {
            spatial[((int64_t)e * N + i) * 2] = (float)(H(b_px, e, i) - R1(r_px, e));
            spatial[((int64_t)e * N + i) * 2 + 1] = (float)(H(b_py, e, i) - R1(r_py, e));
        }
    }
}

/* CrowdSimDict.reset (crowd_sim_dict.py:105-203) */
static void env_reset(ref_engine *g, int e, float *robot_node, float *temporal, float *spatial)
{
    const int N = g->N;
    const int64_t gidx = g->c.env_offset + (g->rows ? g->rows[e] : e);
    rng_t r = {&g->s.mt[(int64_t)e * CN_MT_N], &g->s.mt_pos[e], g->c.rng_mode == CN_RNG_PHILOX};
    /* scenario choice (crowd_sim_dict.py:110-125); the unseeded random.choices is replaced by a
     * deterministic assignment (identical to the reference when one scenario is configured) */
    int sc;
    if (g->c.scenario_mode == CN_SCMODE_SEQUENTIAL) sc = g->c.scenarios[R1(reset_count, e) % g->c.num_scenarios];
    else sc = g->c.scenarios[gidx % g->c.num_scenarios];
    R1(scenario, e) = sc;
    R1(gtime, e) = 0.0;
    R1(r_dv, e) = 0.0;
    const int64_t seed = g->counter_offset + R1(case_counter, e) + (g->c.seed + gidx);
    if (r.philox) { r.mt[0] = (uint32_t)seed; *r.pos = 0; }
    else mt_seed(r.mt, r.pos, (uint32_t)seed);
    uint32_t ovf = 0;
    const double R = g->c.circle_radius;
    /* robot (crowd_sim.py:626-660) */
    R1(r_radius, e) = g->c.robot_radius; R1(r_vpref, e) = g->c.robot_vpref;
    R1(r_vx, e) = 0.0; R1(r_vy, e) = 0.0;
    if (g->c.kinematics == CN_UNICYCLE) {
        const double angle = unif(r, 0, M_PI * 2);
        const double px = R * cos(angle), py = R * sin(angle);
        double gx = 0, gy = 0;
        for (int t = 0;; ++t) {
            gx = unif(r, -R, R); gy = unif(r, -R, R);
            if (np_norm2(px - gx, py - gy) >= 6) break;
            if (t + 1 >= g->c.max_tries) { ++ovf; break; }
        }
        R1(r_px, e) = px; R1(r_py, e) = py; R1(r_gx, e) = gx; R1(r_gy, e) = gy;
        R1(r_theta, e) = unif(r, 0, 2 * M_PI);
    } else if (g->c.social_metrics || g->c.side_preference) {
        R1(r_px, e) = 0; R1(r_py, e) = -R; R1(r_gx, e) = 0; R1(r_gy, e) = R; R1(r_theta, e) = M_PI / 2;
    } else {
        double px = 0, py = 0, gx = 0, gy = 0;
        for (int t = 0;; ++t) {
            px = unif(r, -R, R); py = unif(r, -R, R); gx = unif(r, -R, R); gy = unif(r, -R, R);
            if (np_norm2(px - gx, py - gy) >= 6) break;
            if (t + 1 >= g->c.max_tries) { ++ovf; break; }
        }
        R1(r_px, e) = px; R1(r_py, e) = py; R1(r_gx, e) = gx; R1(r_gy, e) = gy; R1(r_theta, e) = M_PI / 2;
    }
    /* humans (crowd_sim.py:251-259, 359-393) */
    for (int i = 0; i < N; ++i) {
        double vpref = g->c.human_vpref, rad = g->c.human_radius;
        if (g->c.randomize_attributes) { vpref = unif(r, 0.5, 1.5); rad = unif(r, 0.3, 0.5); }
        double px = 0, py = 0, gx = 0, gy = 0, hd = 0, vp = 0;
        for (int t = 0;; ++t) {
            create_agent_attributes(g, e, r, sc, vpref, rad, &px, &py, &gx, &gy, &hd, &vp);
            int collide = 0;
            for (int a = 0; a <= i; ++a) {   /* [self.robot] + self.humans (humans so far) */
                double min_dist, ax, ay;
                if (a == 0) {
                    ax = R1(r_px, e); ay = R1(r_py, e);
                    min_dist = g->c.kinematics == CN_UNICYCLE ? R / 2 : rad + R1(r_radius, e) + g->c.discomfort_dist;
                } else {
                    ax = H(h_px, e, a - 1); ay = H(h_py, e, a - 1);
                    min_dist = rad + H(h_r, e, a - 1) + g->c.discomfort_dist;
                }
                if (np_norm2(px - ax, py - ay) < min_dist) { collide = 1; break; }
            }
            if (!collide) break;
            if (t + 1 >= g->c.max_tries) { ++ovf; break; }
        }
        H(h_px, e, i) = px; H(h_py, e, i) = py; H(h_gx, e, i) = gx; H(h_gy, e, i) = gy;
        H(h_vx, e, i) = 0; H(h_vy, e, i) = 0; H(h_theta, e, i) = hd; H(h_vpref, e, i) = vp; H(h_r, e, i) = rad;
        g->s.o_dmask[(int64_t)e * N + i] = 0;
        g->s.o_r[(int64_t)e * N + i] = 0;
        g->s.o_vmax[(int64_t)e * N + i] = 0;
    }
    R1(case_counter, e) = (R1(case_counter, e) + g->c.nenv) % g->case_size;
    gen_obs(g, e, 1, robot_node, temporal, spatial);
    R1(potential, e) = -fabs(np_norm2(R1(r_px, e) - R1(r_gx, e), R1(r_py, e) - R1(r_gy, e)));
    R1(reset_count, e) += 1;
    R1(ep_return, e) = 0.0; R1(ep_len, e) = 0;
    /* CrowdSim.last_acceleration is set only in configure() (crowd_sim.py:208): it carries over
     * across episodes, so it is NOT cleared here */
    if (g->A > 10) memset(&g->s.o_perm[(int64_t)e * N * g->A], 0, (size_t)N * g->A);
    R1(flags, e) = 0;
    R1(overflow, e) = ovf;
}

/* update_human_goals_randomly (crowd_sim.py:724-766) */
static void goals_randomly(ref_engine *g, int e)
{
    const int N = g->N;
    rng_t r = {&g->s.mt[(int64_t)e * CN_MT_N], &g->s.mt_pos[e], g->c.rng_mode == CN_RNG_PHILOX};
    for (int i = 0; i < N; ++i) {
        if (H(h_vpref, e, i) == 0) continue;
        if (rnd(r) <= g->c.goal_change_chance) {
            double gx = 0, gy = 0;
            for (int t = 0;; ++t) {
                const double angle = rnd(r) * M_PI * 2;
                const double vp = H(h_vpref, e, i) == 0 ? 1.0 : H(h_vpref, e, i);
                const double gxn = (rnd(r) - 0.5) * vp, gyn = (rnd(r) - 0.5) * vp;
                gx = g->c.circle_radius * cos(angle) + gxn;
                gy = g->c.circle_radius * sin(angle) + gyn;
                int collide = 0;
                for (int a = -1; a < N; ++a) {
                    if (a == i) continue;
                    double ax, ay, agx, agy, ar;
                    if (a < 0) { ax = R1(r_px, e); ay = R1(r_py, e); agx = R1(r_gx, e); agy = R1(r_gy, e); ar = R1(r_radius, e); }
                    else { ax = H(h_px, e, a); ay = H(h_py, e, a); agx = H(h_gx, e, a); agy = H(h_gy, e, a); ar = H(h_r, e, a); }
                    const double md = H(h_r, e, i) + ar + g->c.discomfort_dist;
                    if (np_norm2(gx - ax, gy - ay) < md || np_norm2(gx - agx, gy - agy) < md) { collide = 1; break; }
                }
                if (!collide) break;
                if (t + 1 >= g->c.max_tries) { R1(overflow, e) += 1; break; }
            }
            H(h_gx, e, i) = gx; H(h_gy, e, i) = gy;
        }
    }
}

/* update_human_goal (crowd_sim.py:769-811) */
static void human_goal(ref_engine *g, int e, int i)
{
    const int N = g->N;
    rng_t r = {&g->s.mt[(int64_t)e * CN_MT_N], &g->s.mt_pos[e], g->c.rng_mode == CN_RNG_PHILOX};
    if (rnd(r) <= g->c.end_goal_change_chance) {
        if (g->c.random_radii) H(h_r, e, i) += unif(r, -0.1, 0.1);
        if (g->c.random_v_pref) H(h_vpref, e, i) += unif(r, -0.1, 0.1);
        double gx = 0, gy = 0;
        for (int t = 0;; ++t) {
            double px, py, hd, vp;
            create_agent_attributes(g, e, r, R1(scenario, e), H(h_vpref, e, i), H(h_r, e, i), &px, &py, &gx, &gy, &hd, &vp);
            int collide = 0;
            for (int a = -1; a < N; ++a) {
                if (a == i) continue;
                double ax, ay, agx, agy, ar;
                if (a < 0) { ax = R1(r_px, e); ay = R1(r_py, e); agx = R1(r_gx, e); agy = R1(r_gy, e); ar = R1(r_radius, e); }
                else { ax = H(h_px, e, a); ay = H(h_py, e, a); agx = H(h_gx, e, a); agy = H(h_gy, e, a); ar = H(h_r, e, a); }
                const double md = H(h_r, e, i) + ar + g->c.discomfort_dist;
                if (np_norm2(gx - ax, gy - ay) < md || np_norm2(gx - agx, gy - agy) < md) { collide = 1; break; }
            }
            if (!collide) break;
            if (t + 1 >= g->c.max_tries) { R1(overflow, e) += 1; break; }
        }
        H(h_gx, e, i) = gx; H(h_gy, e, i) = gy;
    }
}

/* Agent.compute_position, unicycle (agent.py:185-194): R is float32 (np.float32 v / w); the first
 * sin/cos takes theta as-is (python float at the first step -> float64 trig, np.float32 later ->
 * float32 trig), the second takes theta + r, which is always float32. */
static void unicycle_position(double px, double py, double th, int th_f32, float v, float r, float tr, double dt,
                              double *ox, double *oy)
{
    if (fabsf(r) < 0.0001f) { *ox = px - 0.0 + 0.0; *oy = py + 0.0 - 0.0; return; }
    const float w = r / (float)dt;
    const float R = v / w;
    double t1x, t1y;
    if (th_f32) { t1x = (double)(R * np_sinf((float)th)); t1y = (double)(R * np_cosf((float)th)); }
    else { t1x = (double)R * sin(th); t1y = (double)R * cos(th); }
    const double t2x = (double)(R * np_sinf(tr)), t2y = (double)(R * np_cosf(tr));
    *ox = px - t1x + t2x;
    *oy = py + t1y - t2y;
}

/* ------------------------------------------------------------------------------------------------ */
/* CrowdSimDict.step (crowd_sim_dict.py:205-271) + VecEnv auto-reset + Monitor                        */
/* ------------------------------------------------------------------------------------------------ */
static void env_step(ref_engine *g, int e, const float *actions, float *robot_node, float *temporal, float *spatial,
                     float *reward_out, uint8_t *done_out, int8_t *event_out, float *info_out, double *epr_out,
                     int32_t *epl_out)
{
    const int N = g->N, M = g->M;
    const int holo = g->c.kinematics == CN_HOLONOMIC;
    const double dt = g->c.time_step;
    /* --- clip_action (srnn.py:18-48), float32 --- */
    float a0 = actions[(int64_t)e * 2], a1 = actions[(int64_t)e * 2 + 1];
    double avx = 0, avy = 0;      /* ActionXY */
    float av = 0, ar = 0;         /* ActionRot */
    if (holo) {
        const float n = np_norm2f(a0, a1);
        if ((double)n > R1(r_vpref, e)) {
            const float vp = (float)R1(r_vpref, e);
            a0 = a0 / n * vp; a1 = a1 / n * vp;
        }
        avx = a0; avy = a1;
    } else {
        a0 = np_clipf(a0, -0.1f, 0.1f);
        a1 = np_clipf(a1, -0.1f, 0.1f);
        /* desiredVelocity[0] = clip(dv + action.v, -v_pref, v_pref)  (float32, crowd_sim_dict.py:211-217) */
        const float vp = (float)R1(r_vpref, e);
        float dv = (float)R1(r_dv, e) + a0;
        dv = np_clipf(dv, -vp, vp);
        R1(r_dv, e) = dv;
        av = dv; ar = a1;
    }

    /* --- human actions from the PRE-move state (crowd_sim.py:1121-1161) --- */
    double nvx[64], nvy[64];
    obs_t o[64];
    if (g->c.human_policy == CN_POLICY_ORCA && !(R1(flags, e) & CN_FLAG_ORCA_FROZEN)) {
        /* first ORCA.predict of the episode creates each human's simulator (orca.py:85-109) */
        for (int i = 0; i < N; ++i) {
            human_obs(g, e, i, o);
            uint32_t dm = 0;
            for (int k = 0; k < M; ++k) dm |= (uint32_t)o[k].dummy << k;
            g->s.o_dmask[(int64_t)e * N + i] = dm;
            g->s.o_r[(int64_t)e * N + i] = (float)(H(h_r, e, i) + 0.01 + g->c.orca_safety_space);
            g->s.o_vmax[(int64_t)e * N + i] = (float)H(h_vpref, e, i);
            if (g->A > 10)
                for (int a = 0; a < g->A; ++a) g->s.o_perm[((int64_t)e * N + i) * g->A + a] = (uint8_t)a;
        }
        R1(flags, e) |= CN_FLAG_ORCA_FROZEN;
    }
    for (int i = 0; i < N; ++i) {
        human_obs(g, e, i, o);
        if (g->c.human_policy == CN_POLICY_ORCA) orca_predict(g, e, i, o, &nvx[i], &nvy[i]);
        else sf_predict(g, e, i, o, &nvx[i], &nvy[i]);
    }

    /* --- calc_reward on the PRE-move state (crowd_sim.py:907-1094) --- */
    const double rpx = R1(r_px, e), rpy = R1(r_py, e), rr = R1(r_radius, e);
    double dmin = INFINITY;
    int collision = 0, vr_viol = 0, agg = 0, nz_viol = 0;
    double rcx[4], rcy[4];
    const int rf32 = (R1(flags, e) & CN_FLAG_ROBOT_F32) != 0;
    vel_rect(rpx, rpy, R1(r_vx, e), R1(r_vy, e), rr, rf32, rcx, rcy);
    double nzx[2][4], nzy[2][4];
    if (g->c.norm_zones) {
        norm_zone(rpx, rpy, R1(r_vx, e), R1(r_vy, e), rr, rf32, g->c.norm_zone_lhs, 1, nzx[0], nzy[0]);
        norm_zone(rpx, rpy, R1(r_vx, e), R1(r_vy, e), rr, rf32, g->c.norm_zone_lhs, 0, nzx[1], nzy[1]);
    }
    for (int i = 0; i < N; ++i) {
        const double dx = H(h_px, e, i) - rpx, dy = H(h_py, e, i) - rpy;
        const double cd = sqrt(dx * dx + dy * dy) - H(h_r, e, i) - rr;
        if (cd < 0) { collision = 1; break; }
        else if (cd < dmin) dmin = cd;
        if (g->c.norm_zones && !nz_viol) {
            for (int z = 0; z < 2; ++z)
                if (disc_quad_intersect(rpx, rpy, rr, nzx[z], nzy[z])) nz_viol = 1;
        }
        double hcx[4], hcy[4];
        const double hvx = H(h_vx, e, i), hvy = H(h_vy, e, i);
        vel_rect(H(h_px, e, i), H(h_py, e, i), hvx, hvy, H(h_r, e, i), 0, hcx, hcy);
        if (quads_intersect(rcx, rcy, hcx, hcy)) ++vr_viol;
        if (!(np_norm2(H(h_px, e, i) - H(h_gx, e, i), H(h_py, e, i) - H(h_gy, e, i)) < H(h_r, e, i))) ++agg;
    }
    const int reaching_goal = np_norm2(rpx - R1(r_gx, e), rpy - R1(r_gy, e)) < rr;
    if (!reaching_goal) ++agg;
    float *info = info_out ? info_out + (int64_t)e * CN_INFO_K : NULL;
    double side_l = 0, side_r = 0, sep = 0;
    /* commanded world-frame velocity of this step (holonomic: the action; unicycle: SURVEY §9-1) */
    double cvx, cvy;
    /* unicycle: theta + action.r is float32 (python float or np.float32 theta + np.float32 r; NEP 50) */
    const float tr = (float)R1(r_theta, e) + ar;
    const float th_new = np_modf(tr, (float)(2 * M_PI));
    if (holo) { cvx = avx; cvy = avy; }
    else { cvx = (double)(av * np_cosf(th_new)); cvy = (double)(av * np_sinf(th_new)); }
    if (g->c.side_preference) {
        double ex, ey;
        if (holo) { ex = rpx + (double)(float)(a0 * (float)dt); ey = rpy + (double)(float)(a1 * (float)dt); }
        else unicycle_position(rpx, rpy, R1(r_theta, e), rf32, av, ar, tr, dt, &ex, &ey);
        const double hy = H(h_py, e, 0), hr = H(h_r, e, 0);
        if (ey <= hy + hr && ey >= hy - hr) { if (ex < H(h_px, e, 0)) side_l = 1; else side_r = 1; }
        sep = np_norm2(H(h_px, e, 0) - rpx, H(h_py, e, 0) - rpy);
    }
    double jerk;
    if (holo) {
        const float fax = a0 - (float)R1(r_vx, e), fay = a1 - (float)R1(r_vy, e);
        const float dax = fax - (float)R1(last_ax, e), day = fay - (float)R1(last_ay, e);
        jerk = (double)(dax * dax + day * day);
        R1(last_ax, e) = fax; R1(last_ay, e) = fay;
    } else {
        /* action.vx/vy (patched) are np.float32; robot.vx is int 0 or np.float32 */
        const float ax = (float)cvx - (float)R1(r_vx, e), ay = (float)cvy - (float)R1(r_vy, e);
        const float dax = ax - (float)R1(last_ax, e), day = ay - (float)R1(last_ay, e);
        jerk = (double)(dax * dax + day * day);
        R1(last_ax, e) = ax; R1(last_ay, e) = ay;
    }
    const double dist_to_goal = np_norm2(rpx - R1(r_gx, e), rpy - R1(r_gy, e));
    const int inside = inside_world(rpx, rpy, rr, g->c.square_width / 2);
    double speed;
    if (holo) speed = (double)sqrtf(a0 * a0 + a1 * a1);
    else { const float fx = (float)cvx, fy = (float)cvy; speed = (double)sqrtf(fx * fx + fy * fy); }
    const double gt = R1(gtime, e);
    double reward;
    int done, event;
    if (gt >= g->c.time_limit - 1) { reward = 0; done = 1; event = CN_EV_TIMEOUT; }
    else if (collision || !inside) { reward = g->c.collision_penalty; done = 1; event = CN_EV_COLLISION; }
    else if (reaching_goal) {
        reward = g->c.success_reward;
        if (g->c.time_factor) reward *= (g->c.time_limit - gt) / g->c.time_limit;
        done = 1; event = CN_EV_REACHGOAL;
    } else if (dmin < g->c.discomfort_dist) {
        reward = (dmin - g->c.discomfort_dist) * g->c.discomfort_penalty_factor;
        done = 0; event = CN_EV_DANGER;
    } else {
        const double pc = dist_to_goal;
        reward = g->c.potential_factor * (-fabs(pc) - R1(potential, e));
        R1(potential, e) = -fabs(pc);
        if (g->c.norm_zones && nz_viol) reward += g->c.norm_zone_penalty;
        done = 0; event = CN_EV_NOTHING;
    }
    if (!holo) {
        /* rotational / backwards penalties in float32 (crowd_sim.py:1080-1092) */
        const float r_spin = -2.0f * (ar * ar);
        const float r_back = av < 0 ? -2.0f * fabsf(av) : 0.0f;
        if (event == CN_EV_DANGER || event == CN_EV_NOTHING) reward = reward + (double)r_spin + (double)r_back;
        else reward = (double)(((float)reward + r_spin) + r_back);  /* python int + np.float32 -> float32 */
    }
    if (info) {
        info[CN_INFO_AGG_NAV_TIME] = (float)agg;
        info[CN_INFO_PATH_VIOLATION] = (float)vr_viol;
        info[CN_INFO_PERSONAL_VIOLATION] = dmin < g->c.min_personal_space ? 1.0f : 0.0f;
        info[CN_INFO_JERK_COST] = (float)jerk;
        info[CN_INFO_DIST_TO_GOAL] = (float)dist_to_goal;
        info[CN_INFO_SPEED_VIOLATION] = speed > g->c.max_walking_speed ? 1.0f : 0.0f;
        info[CN_INFO_MIN_DIST] = (float)dmin;
        info[CN_INFO_SCENARIO] = (float)R1(scenario, e);
        info[CN_INFO_SIDE_LEFT] = (float)side_l;
        info[CN_INFO_SIDE_RIGHT] = (float)side_r;
        info[CN_INFO_SEPARATION] = (float)sep;
    }

    /* --- kinematics (agent.py:172-212) --- */
    if (holo) {
        R1(r_px, e) = rpx + (double)(float)(a0 * (float)dt);
        R1(r_py, e) = rpy + (double)(float)(a1 * (float)dt);
        R1(r_vx, e) = avx; R1(r_vy, e) = avy;
    } else {
        double nx, ny;
        unicycle_position(rpx, rpy, R1(r_theta, e), rf32, av, ar, tr, dt, &nx, &ny);
        R1(r_px, e) = nx; R1(r_py, e) = ny;
        R1(r_theta, e) = th_new;
        R1(r_vx, e) = cvx; R1(r_vy, e) = cvy;
    }
    R1(flags, e) |= CN_FLAG_ROBOT_F32;
    for (int i = 0; i < N; ++i) {
        H(h_px, e, i) = H(h_px, e, i) + nvx[i] * dt;
        H(h_py, e, i) = H(h_py, e, i) + nvy[i] * dt;
        H(h_vx, e, i) = nvx[i]; H(h_vy, e, i) = nvy[i];
    }
    R1(gtime, e) = R1(gtime, e) + dt;
    gen_obs(g, e, 0, robot_node, temporal, spatial);

    /* Monitor bookkeeping */
    R1(ep_return, e) += reward;
    R1(ep_len, e) += 1;
    if (reward_out) reward_out[e] = (float)reward;
    if (done_out) done_out[e] = (uint8_t)done;
    if (event_out) event_out[e] = (int8_t)event;
    if (epr_out) epr_out[e] = R1(ep_return, e);
    if (epl_out) epl_out[e] = R1(ep_len, e);

    if (!done) {
        /* goal changes (crowd_sim_dict.py:260-269); skipped when done: reset reseeds and respawns */
        if (g->c.random_goal_changing && np_mod(R1(gtime, e), 5.0) == 0.0) goals_randomly(g, e);
        if (g->c.end_goal_changing)
            for (int i = 0; i < N; ++i)
                if (np_norm2(H(h_gx, e, i) - H(h_px, e, i), H(h_gy, e, i) - H(h_py, e, i)) < H(h_r, e, i)) human_goal(g, e, i);
    } else {
        env_reset(g, e, robot_node, temporal, spatial);
    }
    for (int i = 0; i < N; ++i)
        if (!(H(h_px, e, i) == H(h_px, e, i)) || !(H(h_py, e, i) == H(h_py, e, i))) R1(flags, e) |= CN_FLAG_NAN;
    if (info) info[CN_INFO_OVERFLOW] = (float)R1(overflow, e);
}

/* ------------------------------------------------------------------------------------------------ */
/* exported API (mirrors include/crowdnav.h with the cnref_ prefix; all pointers are HOST pointers)   */
/* ------------------------------------------------------------------------------------------------ */
EXPORT int cnref_create(const cn_config *cfg, ref_engine **out)
{
    if (!cfg || !out) return fail(CN_EINVAL, "null argument");
    if (cfg->num_envs <= 0 || cfg->human_num <= 0 || cfg->human_num > 31) return fail(CN_EINVAL, "bad E/N");
    if (cfg->num_scenarios <= 0) return fail(CN_EINVAL, "no scenario");
    ref_engine *g = (ref_engine *)calloc(1, sizeof *g);
    g->c = *cfg;
    if (g->c.max_tries <= 0) g->c.max_tries = 1000;
    g->E = cfg->num_envs; g->N = cfg->human_num;
    g->A = cn_sim_agents(g->N, cfg->robot_visible); g->M = g->A - 1;
    g->bytes = cn_state_layout(g->E, g->N, cfg->robot_visible, NULL);
    g->blob = aligned_alloc(256, (size_t)g->bytes);
    memset(g->blob, 0, (size_t)g->bytes);
    cn_state_bind(&g->s, g->blob, g->E, g->N, cfg->robot_visible);
    switch (cfg->phase) {
    case CN_PHASE_TRAIN: g->case_size = 4294967295LL - 2000; g->counter_offset = 2000; break;
    case CN_PHASE_VAL: g->case_size = cfg->val_size; g->counter_offset = 0; break;
    default: g->case_size = cfg->test_size; g->counter_offset = 1000; break;
    }
    *out = g;
    return 0;
}
EXPORT void cnref_destroy(ref_engine *g) { if (g) { free(g->rows); free(g->blob); free(g); } }
/* mixed engine group (cn_create_mixed): env e is row rows[e] of the whole engine; seeds and round-robin
 * scenarios use the global index env_offset + rows[e] */
EXPORT int cnref_set_rows(ref_engine *g, const int32_t *rows)
{
    free(g->rows);
    g->rows = NULL;
    if (!rows) return 0;
    g->rows = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->E);
    if (!g->rows) return fail(CN_ENOMEM, "rows");
    memcpy(g->rows, rows, sizeof(int32_t) * (size_t)g->E);
    return 0;
}
EXPORT int64_t cnref_state_bytes(ref_engine *g) { return g->bytes; }
EXPORT void *cnref_state_ptr(ref_engine *g) { return g->blob; }

EXPORT int cnref_reset(ref_engine *g, float *robot_node, float *temporal, float *spatial)
{
#pragma omp parallel for schedule(dynamic, 16)
    for (int e = 0; e < g->E; ++e) env_reset(g, e, robot_node, temporal, spatial);
    return 0;
}

EXPORT int cnref_step(ref_engine *g, const float *actions, float *robot_node, float *temporal, float *spatial,
                      float *reward, uint8_t *done, int8_t *event, float *info, double *ep_return, int32_t *ep_len)
{
#pragma omp parallel for schedule(dynamic, 16)
    for (int e = 0; e < g->E; ++e)
        env_step(g, e, actions, robot_node, temporal, spatial, reward, done, event, info, ep_return, ep_len);
    return 0;
}

EXPORT int cnref_get_state(ref_engine *g, void *dst) { memcpy(dst, g->blob, (size_t)g->bytes); return 0; }
EXPORT int cnref_set_state(ref_engine *g, const void *src) { memcpy(g->blob, src, (size_t)g->bytes); return 0; }
EXPORT void cnref_set_threads(int n)
{
#ifdef _OPENMP
    omp_set_num_threads(n);
#else
    (void)n;
#endif
}
