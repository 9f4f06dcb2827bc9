// Masked GRU sequence kernels for the DSRNN policy.
//
// The reference runs its three GRUs (srnn_model.py:52-104, RNNBase._forward_gru) as torch nn.GRU calls over
// the segments between episode starts; every segment boundary re-enters cuDNN/MIOpen with the hidden state
// multiplied by the mask. Here a sequence of T steps is:
//   gi  = x @ W_ih^T + b_ih            one GEMM over all T*B rows (hipBLASLt, from the torch wrapper)
//   per step t:
//     gh = hm_t @ W_hh^T + b_hh        one GEMM (B x H -> B x 3H)
//     cn_gru_fwd_step                  gates + new state + the next step's masked state, one pass
//   backward, per step t (reversed):
//     cn_gru_bwd_step                  gate gradients from the saved gates, one pass
//     acc += dgh_t @ W_hh              one GEMM
//   then dW_ih, dW_hh, db_*, dx as single GEMMs / reductions over all T*B rows.
// Gate math and operation order follow ATen's GRU cell (the reference's nn.GRU):
//   r = sigmoid(gh_r + gi_r), z = sigmoid(gh_z + gi_z), n = tanh(gi_n + r * gh_n), h' = (h - n) * z + n.
// Memory-bound elementwise work: each thread handles 4 consecutive hidden units (16-byte accesses).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <initializer_list>

#include "../../include/crowdnav.h"

int cn_set_error(int code, const char *msg);

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// gi, gh: [B][3H] (r | z | n blocks); hm: [B][H] the masked previous state; m_next: [B] or null;
// h_out: [B][H]; hm_next: [B][H] or null (= h_out * m_next); save: [B][4H] (r | z | n | gh_n) or null;
// h_out2: a second copy of h_out in a grouped row layout (row b at (b / g2) * ld2 + (b % g2) * H), or null.
__global__ __launch_bounds__(256) void cn_gru_fwd_kernel(int64_t B, int H, const float *__restrict__ gi,
                                                         const float *__restrict__ gh,
                                                         const float *__restrict__ hm,
                                                         const float *__restrict__ m_next, float *__restrict__ h_out,
                                                         float *__restrict__ hm_next, float *__restrict__ save,
                                                         float *__restrict__ h_out2, int64_t g2, int64_t ld2)
{
    const int H4 = H >> 2;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * H4) return;
    const int64_t b = i / H4;
    const int j = (int)(i - b * H4) * 4;
    const float4 ir = *(const float4 *)(gi + b * 3 * H + j);
    const float4 iz = *(const float4 *)(gi + b * 3 * H + H + j);
    const float4 in = *(const float4 *)(gi + b * 3 * H + 2 * H + j);
    const float4 hr = *(const float4 *)(gh + b * 3 * H + j);
    const float4 hz = *(const float4 *)(gh + b * 3 * H + H + j);
    const float4 hn = *(const float4 *)(gh + b * 3 * H + 2 * H + j);
    const float4 hp = *(const float4 *)(hm + b * H + j);
    float4 r, z, n, h;
#define CN_GATE(c)                                 \
    r.c = sigm(hr.c + ir.c);                       \
    z.c = sigm(hz.c + iz.c);                       \
    n.c = tanhf(in.c + hn.c * r.c);                \
    h.c = (hp.c - n.c) * z.c + n.c;
    CN_GATE(x) CN_GATE(y) CN_GATE(z) CN_GATE(w)
#undef CN_GATE
    *(float4 *)(h_out + b * H + j) = h;
    if (h_out2) *(float4 *)(h_out2 + (b / g2) * ld2 + (b % g2) * H + j) = h;
    if (hm_next) {
        const float m = m_next ? m_next[b] : 1.0f;
        *(float4 *)(hm_next + b * H + j) = make_float4(h.x * m, h.y * m, h.z * m, h.w * m);
    }
    if (save) {
        float *s = save + b * 4 * H + j;
        *(float4 *)(s) = r;
        *(float4 *)(s + H) = z;
        *(float4 *)(s + 2 * H) = n;
        *(float4 *)(s + 3 * H) = hn;
    }
}

// Gradient of step t. g = acc * m_next + dout_t is dL/dh_t (acc = dL/dhm_{t+1} from the later step, or
// dL/dh_T at the last step with m_next = null). Writes dgi_t, dgh_t [B][3H] and acc <- g * z (the direct
// path of dL/dhm_t; the caller adds dgh_t @ W_hh).
__global__ __launch_bounds__(256) void cn_gru_bwd_kernel(int64_t B, int H, float *__restrict__ acc,
                                                         const float *__restrict__ m_next,
                                                         const float *__restrict__ dout,
                                                         const float *__restrict__ save,
                                                         const float *__restrict__ hm, float *__restrict__ dgi,
                                                         float *__restrict__ dgh)
{
    const int H4 = H >> 2;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * H4) return;
    const int64_t b = i / H4;
    const int j = (int)(i - b * H4) * 4;
    const float m = m_next ? m_next[b] : 1.0f;
    float4 g = *(const float4 *)(acc + b * H + j);
    g = make_float4(g.x * m, g.y * m, g.z * m, g.w * m);
    if (dout) {
        const float4 d = *(const float4 *)(dout + b * H + j);
        g = make_float4(g.x + d.x, g.y + d.y, g.z + d.z, g.w + d.w);
    }
    const float *s = save + b * 4 * H + j;
    const float4 r = *(const float4 *)(s), z = *(const float4 *)(s + H), n = *(const float4 *)(s + 2 * H),
                 hn = *(const float4 *)(s + 3 * H);
    const float4 hp = *(const float4 *)(hm + b * H + j);
    float4 a, dr, dz, dn, dhn;
#define CN_GBWD(c)                                              \
    {                                                           \
        const float dnc = g.c * (1.0f - z.c) * (1.0f - n.c * n.c); \
        const float dzc = g.c * (hp.c - n.c) * z.c * (1.0f - z.c); \
        const float drc = dnc * hn.c * r.c * (1.0f - r.c);      \
        a.c = g.c * z.c;                                        \
        dr.c = drc;                                             \
        dz.c = dzc;                                             \
        dn.c = dnc;                                             \
        dhn.c = dnc * r.c;                                      \
    }
    CN_GBWD(x) CN_GBWD(y) CN_GBWD(z) CN_GBWD(w)
#undef CN_GBWD
    *(float4 *)(acc + b * H + j) = a;
    *(float4 *)(dgi + b * 3 * H + j) = dr;
    *(float4 *)(dgi + b * 3 * H + H + j) = dz;
    *(float4 *)(dgi + b * 3 * H + 2 * H + j) = dn;
    *(float4 *)(dgh + b * 3 * H + j) = dr;
    *(float4 *)(dgh + b * 3 * H + H + j) = dz;
    *(float4 *)(dgh + b * 3 * H + 2 * H + j) = dhn;
}

// The same step with the bias gradients folded in (the reference's autograd sums dgi / dgh over all T*B
// rows for b_ih / b_hh: two passes over [T][B][3H] each). Workgroup = CN_GB_RW rows x H columns, thread
// (row slot, 4 columns); besides dgi / dgh it writes the workgroup's column sums of dr | dz | dn | dhn to
// part [blocks][4H] (row slots summed in order through LDS); cn_gru_bias_reduce adds the partials of all
// steps in order (deterministic).
#define CN_GB_RW 16
// COMB: the gate gradients go once to g = [dn | dr | dz | dhn] per row (4H; dgi's r / z columns equal dgh's,
// so dgh = g[:, H:4H] and dgi = g[:, 0:3H] with the input weights' rows taken in the order n, r, z) instead of
// the separate [dr | dz | dn] and [dr | dz | dhn] (6H): 2H fewer floats written per row and step
template <bool COMB>
__global__ __launch_bounds__(256) void cn_gru_bwd_bias_kernel(int64_t B, int H, float *__restrict__ acc,
                                                              const float *__restrict__ m_next,
                                                              const float *__restrict__ dout,
                                                              const float *__restrict__ save,
                                                              const float *__restrict__ hm, float *__restrict__ dgi,
                                                              float *__restrict__ dgh, float *__restrict__ part)
{
    __shared__ float4 red[256][4];
    const int H4 = H >> 2, slots = 256 / H4;   // H in {64, 128, 256}: 16 / 8 / 4 row slots
    const int rs = (int)threadIdx.x / H4, j = ((int)threadIdx.x - rs * H4) * 4;
    float4 sr = make_float4(0.f, 0.f, 0.f, 0.f), sz = sr, sn = sr, shn = sr;
    const int64_t b0 = (int64_t)blockIdx.x * CN_GB_RW;
    for (int k = rs; k < CN_GB_RW; k += slots) {
        const int64_t b = b0 + k;
        if (b >= B) break;
        const float m = m_next ? m_next[b] : 1.0f;
        float4 g = *(const float4 *)(acc + b * H + j);
        g = make_float4(g.x * m, g.y * m, g.z * m, g.w * m);
        if (dout) {
            const float4 d = *(const float4 *)(dout + b * H + j);
            g = make_float4(g.x + d.x, g.y + d.y, g.z + d.z, g.w + d.w);
        }
        const float *s = save + b * 4 * H + j;
        const float4 r = *(const float4 *)(s), z = *(const float4 *)(s + H), n = *(const float4 *)(s + 2 * H),
                     hn = *(const float4 *)(s + 3 * H);
        const float4 hp = *(const float4 *)(hm + b * H + j);
        float4 a, dr, dz, dn, dhn;
#define CN_GBWD(c)                                              \
    {                                                           \
        const float dnc = g.c * (1.0f - z.c) * (1.0f - n.c * n.c); \
        const float dzc = g.c * (hp.c - n.c) * z.c * (1.0f - z.c); \
        const float drc = dnc * hn.c * r.c * (1.0f - r.c);      \
        a.c = g.c * z.c;                                        \
        dr.c = drc;                                             \
        dz.c = dzc;                                             \
        dn.c = dnc;                                             \
        dhn.c = dnc * r.c;                                      \
        sr.c += drc; sz.c += dzc; sn.c += dnc; shn.c += dhn.c;  \
    }
        CN_GBWD(x) CN_GBWD(y) CN_GBWD(z) CN_GBWD(w)
#undef CN_GBWD
        *(float4 *)(acc + b * H + j) = a;
        if (COMB) {
            float *gr = dgi + b * 4 * H + j;
            *(float4 *)(gr) = dn;
            *(float4 *)(gr + H) = dr;
            *(float4 *)(gr + 2 * H) = dz;
            *(float4 *)(gr + 3 * H) = dhn;
        } else {
            *(float4 *)(dgi + b * 3 * H + j) = dr;
            *(float4 *)(dgi + b * 3 * H + H + j) = dz;
            *(float4 *)(dgi + b * 3 * H + 2 * H + j) = dn;
            *(float4 *)(dgh + b * 3 * H + j) = dr;
            *(float4 *)(dgh + b * 3 * H + H + j) = dz;
            *(float4 *)(dgh + b * 3 * H + 2 * H + j) = dhn;
        }
    }
    red[threadIdx.x][0] = sr; red[threadIdx.x][1] = sz; red[threadIdx.x][2] = sn; red[threadIdx.x][3] = shn;
    __syncthreads();
    if (rs != 0) return;
    for (int q = 1; q < slots; ++q) {
        const float4 *o = red[q * H4 + threadIdx.x];
        sr.x += o[0].x; sr.y += o[0].y; sr.z += o[0].z; sr.w += o[0].w;
        sz.x += o[1].x; sz.y += o[1].y; sz.z += o[1].z; sz.w += o[1].w;
        sn.x += o[2].x; sn.y += o[2].y; sn.z += o[2].z; sn.w += o[2].w;
        shn.x += o[3].x; shn.y += o[3].y; shn.z += o[3].z; shn.w += o[3].w;
    }
    float *pw = part + (int64_t)blockIdx.x * 4 * H + j;
    *(float4 *)(pw) = sr;
    *(float4 *)(pw + H) = sz;
    *(float4 *)(pw + 2 * H) = sn;
    *(float4 *)(pw + 3 * H) = shn;
}

// db_ih = (sum dr, sum dz, sum dn), db_hh = (sum dr, sum dz, sum dhn) over the rows of part [rows][4H]
// (every step's workgroup partials), in two deterministic passes: CN_GB_RC row chunks x 64-column slices
// (thread = column, the workgroup's 4 waves stride the chunk's rows, LDS sum in wave order) into
// work [CN_GB_RC][4H], then the chunks in order.
#define CN_GB_RC 64
__global__ __launch_bounds__(256) void cn_gru_bias_part2_kernel(int64_t rows, int H, const float *__restrict__ part,
                                                                float *__restrict__ work)
{
    __shared__ float red[4][64];
    const int col = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6, rc = blockIdx.y;
    const int64_t chunk = (rows + CN_GB_RC - 1) / CN_GB_RC, r0 = rc * chunk;
    const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
    float s = 0.0f;
    if (col < 4 * H)
        for (int64_t r = r0 + w; r < r1; r += 4) s += part[r * 4 * H + col];
    red[w][threadIdx.x & 63] = s;
    __syncthreads();
    if (w != 0 || col >= 4 * H) return;
    work[(int64_t)rc * 4 * H + col] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

__global__ __launch_bounds__(256) void cn_gru_bias_final_kernel(int H, const float *__restrict__ work,
                                                                float *__restrict__ db_ih, float *__restrict__ db_hh)
{
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= 4 * H) return;
    float s = 0.0f;
    for (int rc = 0; rc < CN_GB_RC; ++rc) s += work[rc * 4 * H + col];
    const int gate = col / H, u = col - gate * H;
    if (gate < 2) { db_ih[col] = s; db_hh[col] = s; }
    else if (gate == 2) db_ih[2 * H + u] = s;
    else db_hh[2 * H + u] = s;
}

inline unsigned grid_for(int64_t B, int H) { return (unsigned)((B * (H / 4) + 255) / 256); }

// ------------------------------------------------------------------------------------------------
// Fused recurrent step: gh = hm W_hh^T + b_hh on the f32-input matrix cores with the gate arithmetic of
// cn_gru_fwd_kernel in the epilogue, so gh ([B][3H], 63 MB at C4's 20,480 x 256) never goes to HBM.
// Workgroup tile: GF_BM = 128 rows x GF_BU = 32 hidden units, i.e. the r, z and n columns of those units
// (96 of W_hh's rows); 4 waves, wave w owns rows 32w .. 32w + 31 and one 32x32 accumulator per gate
// (v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulation). K (= H) streams through LDS in chunks
// of 32: the next chunk's global loads are in flight while the current one is multiplied.
// The k pair of an MFMA is a permutation of K (lane half p of step (c, q) holds k = 8c + 4p + q for A
// and B alike), so every lane reads 16-byte LDS vectors. Rows are padded to 36 floats in LDS (the 32 rows
// of a b128 read land on distinct bank groups).
// Grid: XCD-aware -- workgroup id x runs on XCD x % 8; the 8 unit tiles (H = 256) of one row tile are
// given consecutive ids on the same XCD, so the row tile's hm rows are fetched into that XCD's L2 once.
// ------------------------------------------------------------------------------------------------
constexpr int GF_BM = 128, GF_BU = 32, GF_KC = 32, GF_LD = GF_KC + 4;
typedef float gf_f32x16 __attribute__((ext_vector_type(16)));

// One GRU (segment) of a fused-step launch: two independent GRUs with the same H (the DSRNN's spatial and
// temporal edge RNNs) share one launch, the row tiles of the second following the first's.
struct GfSeg {
    int64_t B;
    const float *gi, *hm, *w_hh, *b_hh, *m_next;
    float *h_out, *hm_next, *save, *h_out2;
    int64_t g2, ld2;
    // input projection in the kernel (template XM): gi = x W_ih^T + b_ih from x [B][F], w_ih [3H][F], b_ih [3H]
    const float *x, *w_ih, *b_ih;
    int64_t F;
};
struct GfArgs {
    GfSeg s0, s1;
    int rt0, rt_total, unit_tiles, H;
};
// XM (input projection in the kernel): the K loop first runs the F / 32 chunks of x against W_ih (r and z into
// the same accumulators as their recurrent parts, n into a fourth one: gi_n stays separate from gh_n), then
// the H / 32 chunks of hm against W_hh; the epilogue adds b_ih and b_hh. gi ([B][3H], 3 of the 10 floats the
// step moves per output, and its T * B * 3H buffer) is never materialised.
template <bool XM>
__global__ __launch_bounds__(256, 3) void cn_gru_fused_kernel(const GfArgs P)
{
    // LDS: one A / B chunk buffer during the K loop, then the three gate accumulators of the tile
    // (sC[g][row][unit], rows padded to LDC = 33) for the epilogue's row-major pass. 50.7 KB in all, so three
    // workgroups fit per CU: another workgroup's MFMAs cover one's barriers and epilogue (measured 92 us vs
    // 99 us for the double-buffered 64.5 KB form at two per CU).
    constexpr int SA = GF_BM * GF_LD, SB = 3 * GF_BU * GF_LD, LDC = 33;
    constexpr int SMEM = (SA + SB) > 3 * GF_BM * LDC ? (SA + SB) : 3 * GF_BM * LDC;
    __shared__ __attribute__((aligned(16))) float smem[SMEM];
    float *const sA0 = smem, *const sB0 = smem + SA;
    const int bid = blockIdx.x;
    const int xcd = bid & 7, k = bid >> 3;
    const int unit_tiles = P.unit_tiles, H = P.H;
    const int ut = k % unit_tiles;
    int rt = (k / unit_tiles) * 8 + xcd;
    if (rt >= P.rt_total) return;  // grid padding (whole workgroup, before any barrier)
    const bool second = rt >= P.rt0;
    const GfSeg S = second ? P.s1 : P.s0;
    if (second) rt -= P.rt0;
    const int64_t B = S.B;
    const float *__restrict__ gi = S.gi, *__restrict__ hm = S.hm, *__restrict__ w_hh = S.w_hh,
                                  *__restrict__ b_hh = S.b_hh, *__restrict__ m_next = S.m_next;
    float *__restrict__ h_out = S.h_out, *__restrict__ hm_next = S.hm_next, *__restrict__ save = S.save,
                        *__restrict__ h_out2 = S.h_out2;
    const int64_t g2 = S.g2, ld2 = S.ld2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row0 = (int64_t)rt * GF_BM;
    const int u0 = ut * GF_BU;

    // global -> register staging: A = 128 rows x 32 floats (4 float4 per thread), B = 96 rows (3 per thread).
    // Plain scalars (no captured arrays): the loads must stay in flight across the chunk's MFMAs. The same
    // thread -> (row, 4 columns) map serves the epilogue: thread t owns units u0 + lc .. + 3 of rows lr + 32 i.
    const int lc = (tid & 7) * 4, lr = tid >> 3;
    // rows past B (last row tile) read row B - 1 instead: rows are independent and those are never stored
    int64_t ar[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ar[i] = min(row0 + lr + 32 * i, B - 1);
    const float *pa0 = hm + ar[0] * H + lc, *pa1 = hm + ar[1] * H + lc, *pa2 = hm + ar[2] * H + lc,
                *pa3 = hm + ar[3] * H + lc;
    const float *pb0 = w_hh + (int64_t)(u0 + lr) * H + lc;
    const int64_t b_step = (int64_t)H * H;
    float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2;
#define GF_GLOAD(kc)                                                         \
    ra0 = *(const float4 *)(pa0 + (kc));                                     \
    ra1 = *(const float4 *)(pa1 + (kc));                                     \
    ra2 = *(const float4 *)(pa2 + (kc));                                     \
    ra3 = *(const float4 *)(pa3 + (kc));                                     \
    rb0 = *(const float4 *)(pb0 + (kc));                                     \
    rb1 = *(const float4 *)(pb0 + b_step + (kc));                            \
    rb2 = *(const float4 *)(pb0 + 2 * b_step + (kc));
#define GF_LSTORE(buf)                                                                    \
    {                                                                                     \
        float *da = sA0 + (buf) * SA + lr * GF_LD + lc, *db = sB0 + (buf) * SB + lr * GF_LD + lc; \
        *(float4 *)(da) = ra0;                                                            \
        *(float4 *)(da + 32 * GF_LD) = ra1;                                               \
        *(float4 *)(da + 64 * GF_LD) = ra2;                                               \
        *(float4 *)(da + 96 * GF_LD) = ra3;                                               \
        *(float4 *)(db) = rb0;                                                            \
        *(float4 *)(db + GF_BU * GF_LD) = rb1;                                            \
        *(float4 *)(db + 2 * GF_BU * GF_LD) = rb2;                                        \
    }
    const int li = lane & 31, p4 = (lane >> 5) * 4;
#define GF_MMA(buf, A2)                                                                                      \
    {                                                                                                        \
        const float *a_base = sA0 + (buf) * SA + (wave * 32 + li) * GF_LD + p4;                              \
        const float *b_base = sB0 + (buf) * SB + li * GF_LD + p4;                                            \
        _Pragma("unroll") for (int c = 0; c < GF_KC / 8; ++c)                                                \
        {                                                                                                    \
            const float4 a = *(const float4 *)(a_base + 8 * c);                                              \
            float4 bv[3];                                                                                    \
            _Pragma("unroll") for (int g = 0; g < 3; ++g) bv[g] = *(const float4 *)(b_base + g * GF_BU * GF_LD + 8 * c); \
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bv[0].x, acc[0], 0, 0, 0);                   \
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bv[1].x, acc[1], 0, 0, 0);                   \
            A2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bv[2].x, A2, 0, 0, 0);                           \
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bv[0].y, acc[0], 0, 0, 0);                   \
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bv[1].y, acc[1], 0, 0, 0);                   \
            A2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bv[2].y, A2, 0, 0, 0);                           \
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bv[0].z, acc[0], 0, 0, 0);                   \
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bv[1].z, acc[1], 0, 0, 0);                   \
            A2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bv[2].z, A2, 0, 0, 0);                           \
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bv[0].w, acc[0], 0, 0, 0);                   \
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bv[1].w, acc[1], 0, 0, 0);                   \
            A2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bv[2].w, A2, 0, 0, 0);                           \
        }                                                                                                    \
    }

    gf_f32x16 acc[3], acc_in;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = 0.0f;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc_in[e] = 0.0f;

    const int nch = H / GF_KC;
    float4 eg[4][3], eh[4];
#define GF_EPI_LOAD()                                                                    \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                       \
    {                                                                                    \
        if (!XM) {                                                                       \
            const float *gib = gi + ar[i] * 3 * H + u0 + lc;                             \
            _Pragma("unroll") for (int g = 0; g < 3; ++g) eg[i][g] = *(const float4 *)(gib + g * H); \
        }                                                                                \
        eh[i] = *(const float4 *)(hm + ar[i] * H + u0 + lc);                             \
    }
    if (XM) {
        // x chunks first (A = x rows, B = W_ih rows; n into acc_in), then the recurrent ones. Two loops, and
        // the x addresses formed per load, so no second address set stays live across the recurrent chunks.
        const int64_t F = S.F;
        const int ncx = (int)(F / GF_KC);
        const float *__restrict__ xx = S.x, *__restrict__ wih = S.w_ih;
#define GF_GLOAD_X(kc)                                                                        \
    {                                                                                         \
        ra0 = *(const float4 *)(xx + ar[0] * F + lc + (kc));                                  \
        ra1 = *(const float4 *)(xx + ar[1] * F + lc + (kc));                                  \
        ra2 = *(const float4 *)(xx + ar[2] * F + lc + (kc));                                  \
        ra3 = *(const float4 *)(xx + ar[3] * F + lc + (kc));                                  \
        const float *xb = wih + (int64_t)(u0 + lr) * F + lc + (kc);                           \
        rb0 = *(const float4 *)(xb);                                                          \
        rb1 = *(const float4 *)(xb + (int64_t)H * F);                                         \
        rb2 = *(const float4 *)(xb + (int64_t)2 * H * F);                                     \
    }
        GF_GLOAD_X(0)
        GF_LSTORE(0)
        __syncthreads();
        for (int ch = 0; ch < ncx; ++ch) {
            if (ch + 1 < ncx) {
                GF_GLOAD_X((ch + 1) * GF_KC)
            } else {
                GF_GLOAD(0)   // the first recurrent chunk
            }
            GF_MMA(0, acc_in)
            __syncthreads();
            GF_LSTORE(0)
            __syncthreads();
        }
#undef GF_GLOAD_X
    } else {
        GF_GLOAD(0)
        GF_LSTORE(0)
        __syncthreads();
    }
    for (int ch = 0; ch + 1 < nch; ++ch) {
        GF_GLOAD((ch + 1) * GF_KC)  // in flight during this chunk's MFMAs
        GF_MMA(0, acc[2])
        __syncthreads();
        GF_LSTORE(0)
        __syncthreads();
    }
    // last chunk (a recurrent one): the epilogue's operands (gi's three gate blocks unless XM, and hm of this
    // thread's 4 x 4 outputs) are fetched while its MFMAs run
    GF_EPI_LOAD()
#undef GF_EPI_LOAD
    GF_MMA(0, acc[2])
    __syncthreads();  // every wave is done reading the chunk buffers before sC overwrites them
#undef GF_GLOAD
#undef GF_LSTORE
#undef GF_MMA

    // accumulators -> LDS: lane holds unit li of rows (e & 3) + 8 (e >> 2) + 4 (lane >> 5) of its wave's 32.
    // XM: the input part of n (acc_in) goes through region 2 first; gi_r / gi_z are b_ih alone (their x parts
    // are in acc r / z) and gi_n = acc_in + b_ih_n
#define GF_TO_LDS(g, A)                                                                                        \
    _Pragma("unroll") for (int e = 0; e < 16; ++e)                                                           \
        smem[((g) * GF_BM + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * LDC + li] = (A)[e];
    GF_TO_LDS(0, acc[0])
    GF_TO_LDS(1, acc[1])
    if (XM) {
        GF_TO_LDS(2, acc_in)
        __syncthreads();
        const float *b_ih = S.b_ih;
        const float4 bir = *(const float4 *)(b_ih + u0 + lc), biz = *(const float4 *)(b_ih + H + u0 + lc),
                     bin = *(const float4 *)(b_ih + 2 * H + u0 + lc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float *pc = smem + (2 * GF_BM + lr + 32 * i) * LDC + lc;
            eg[i][0] = bir;
            eg[i][1] = biz;
            eg[i][2] = make_float4(pc[0] + bin.x, pc[1] + bin.y, pc[2] + bin.z, pc[3] + bin.w);
        }
        __syncthreads();
    }
    GF_TO_LDS(2, acc[2])
#undef GF_TO_LDS
    __syncthreads();

    const float4 br = *(const float4 *)(b_hh + u0 + lc), bz = *(const float4 *)(b_hh + H + u0 + lc),
                 bn = *(const float4 *)(b_hh + 2 * H + u0 + lc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = lr + 32 * i;
        const int64_t b = row0 + row;
        if (b >= B) continue;
        const float *pcr = smem + (0 * GF_BM + row) * LDC + lc;
        const float4 cr = make_float4(pcr[0], pcr[1], pcr[2], pcr[3]);
        const float *pcz = smem + (1 * GF_BM + row) * LDC + lc;
        const float4 cz = make_float4(pcz[0], pcz[1], pcz[2], pcz[3]);
        const float *pcn = smem + (2 * GF_BM + row) * LDC + lc;
        const float4 cn = make_float4(pcn[0], pcn[1], pcn[2], pcn[3]);
        const float4 ir = eg[i][0], iz = eg[i][1], in = eg[i][2], hp = eh[i];
        float4 hr, hz, hn, r, z, n, h;
#define CN_GATE(c)                                 \
    hr.c = cr.c + br.c;                            \
    hz.c = cz.c + bz.c;                            \
    hn.c = cn.c + bn.c;                            \
    r.c = sigm(hr.c + ir.c);                       \
    z.c = sigm(hz.c + iz.c);                       \
    n.c = tanhf(in.c + hn.c * r.c);                \
    h.c = (hp.c - n.c) * z.c + n.c;
        CN_GATE(x) CN_GATE(y) CN_GATE(z) CN_GATE(w)
#undef CN_GATE
        const int64_t o = b * H + u0 + lc;
        *(float4 *)(h_out + o) = h;
        if (h_out2) {
            float *d = h_out2 + (b / g2) * ld2 + (b % g2) * H + u0 + lc;
            d[0] = h.x;
            d[1] = h.y;
            d[2] = h.z;
            d[3] = h.w;
        }
        if (hm_next) {
            const float m = m_next ? m_next[b] : 1.0f;
            *(float4 *)(hm_next + o) = make_float4(h.x * m, h.y * m, h.z * m, h.w * m);
        }
        if (save) {
            float *sv = save + b * 4 * H + u0 + lc;
            *(float4 *)(sv) = r;
            *(float4 *)(sv + H) = z;
            *(float4 *)(sv + 2 * H) = n;
            *(float4 *)(sv + 3 * H) = hn;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Fused backward step: the recurrent GEMM of step t, acc_t = a_t + g_t[:, H:4H] W_hh (K = 3H; a_t = the
// direct path dL/dh_t * z_t), on the f32 matrix cores with the gate gradients of step t - 1 in its epilogue:
//   gacc = acc_t * m_t + dout_{t-1}                       (dL/dh_{t-1})
//   dn = gacc (1 - z) (1 - n^2), dz = gacc (hm - n) z (1 - z), dr = dn gh_n r (1 - r), dhn = dn r
//   a_{t-1} = gacc z;  g_{t-1} = [dn | dr | dz | dhn];  column sums of dr | dz | dn | dhn -> part
// so acc_t never goes to HBM and the backward is one launch per step (cn_gru_bwd_seq). Modes per launch: no
// GEMM (gk = null: the first step, acc = dL/dh_{T-1} comes in through a) and no gates (g = null: the last
// step, a <- acc_0 = dL/dhm_0). Same tiling as cn_gru_fused_kernel: 128 rows x 32 hidden units per
// workgroup, wave w owns rows 32w .. 32w + 31 with one 32x32 accumulator (v_mfma_f32_32x32x2_f32), K in
// chunks of 32 through double-buffered LDS (46 KB: three workgroups per CU), XCD-aware tile order.
// The B operand is W_hh^T [H][3H] (row u = unit u's weights over the 3H gate gradients, contiguous in K).
// ------------------------------------------------------------------------------------------------
struct GbSeg {
    int64_t B;
    const float *gk;      // g_t [B][4H]: the K operand is its columns H .. 4H (dr | dz | dhn); null: no GEMM
    const float *wt;      // W_hh^T [H][3H]
    float *a;             // [B][H]: in a_t (or dL/dh_{T-1}), out a_{t-1} (gates) or acc_t (no gates)
    const float *m_next;  // [B] m_t, or null (= 1)
    const float *dout;    // [B][H] dL/d out_{t-1}, or null
    const float *save;    // [B][4H] r | z | n | gh_n of step t - 1
    const float *hm;      // [B][H] masked state entering step t - 1
    float *g;             // [B][4H] out g_{t-1}, or null: no gates
    float *part;          // [row tiles][4H] out: the workgroup's column sums
};
struct GbArgs {
    GbSeg s0, s1;
    int rt0, rt_total, unit_tiles, H;
};

__global__ __launch_bounds__(256, 3) void cn_gru_bwd_fused_kernel(const GbArgs P)
{
    constexpr int SA = GF_BM * GF_LD, SB = GF_BU * GF_LD, LDC = 33;
    __shared__ __attribute__((aligned(16))) float smem[2 * (SA + SB)];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, k = bid >> 3;
    const int unit_tiles = P.unit_tiles, H = P.H;
    const int ut = k % unit_tiles;
    int rt = (k / unit_tiles) * 8 + xcd;
    if (rt >= P.rt_total) return;  // grid padding (whole workgroup, before any barrier)
    const bool second = rt >= P.rt0;
    const GbSeg S = second ? P.s1 : P.s0;
    if (second) rt -= P.rt0;
    const int64_t B = S.B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row0 = (int64_t)rt * GF_BM;
    const int u0 = ut * GF_BU;
    const int lc = (tid & 7) * 4, lr = tid >> 3;
    const int li = lane & 31, p4 = (lane >> 5) * 4;
    int64_t ar[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ar[i] = min(row0 + lr + 32 * i, B - 1);

    gf_f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
    // the gate records of the epilogue's 4 x 4 outputs (thread: units u0 + lc .. + 3 of rows lr + 32 i) are
    // fetched during the last chunk; the other operands (a, dout, hm: one float4 per row each) in the epilogue
    float4 es[4][4];
    const bool gates = S.g != nullptr;
#define GB_EPI_LOAD()                                                                                   \
    if (gates) {                                                                                        \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                  \
        {                                                                                               \
            const float *sv = S.save + ar[i] * 4 * H + u0 + lc;                                         \
            _Pragma("unroll") for (int q = 0; q < 4; ++q) es[i][q] = *(const float4 *)(sv + q * H);    \
        }                                                                                               \
    }

    if (S.gk) {
        const int K3 = 3 * H, ldg = 4 * H;
        const float *pa0 = S.gk + ar[0] * ldg + H + lc, *pa1 = S.gk + ar[1] * ldg + H + lc,
                    *pa2 = S.gk + ar[2] * ldg + H + lc, *pa3 = S.gk + ar[3] * ldg + H + lc;
        const float *pb = S.wt + (int64_t)(u0 + lr) * K3 + lc;
        float4 ra0, ra1, ra2, ra3, rb;
#define GB_GLOAD(kc)                           \
    ra0 = *(const float4 *)(pa0 + (kc));       \
    ra1 = *(const float4 *)(pa1 + (kc));       \
    ra2 = *(const float4 *)(pa2 + (kc));       \
    ra3 = *(const float4 *)(pa3 + (kc));       \
    rb = *(const float4 *)(pb + (kc));
#define GB_LSTORE(buf)                                                                          \
    {                                                                                           \
        float *da = smem + (buf) * SA + lr * GF_LD + lc, *db = smem + 2 * SA + (buf) * SB + lr * GF_LD + lc; \
        *(float4 *)(da) = ra0;                                                                  \
        *(float4 *)(da + 32 * GF_LD) = ra1;                                                     \
        *(float4 *)(da + 64 * GF_LD) = ra2;                                                     \
        *(float4 *)(da + 96 * GF_LD) = ra3;                                                     \
        *(float4 *)(db) = rb;                                                                   \
    }
#define GB_MMA(buf)                                                                             \
    {                                                                                           \
        const float *a_base = smem + (buf) * SA + (wave * 32 + li) * GF_LD + p4;                \
        const float *b_base = smem + 2 * SA + (buf) * SB + li * GF_LD + p4;                     \
        _Pragma("unroll") for (int c = 0; c < GF_KC / 8; ++c)                                   \
        {                                                                                       \
            const float4 av = *(const float4 *)(a_base + 8 * c);                                \
            const float4 bv = *(const float4 *)(b_base + 8 * c);                                \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc, 0, 0, 0);               \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc, 0, 0, 0);               \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc, 0, 0, 0);               \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc, 0, 0, 0);               \
        }                                                                                       \
    }
        const int nch = K3 / GF_KC;
        GB_GLOAD(0)
        GB_LSTORE(0)
        __syncthreads();
        for (int ch = 0; ch + 1 < nch; ++ch) {
            GB_GLOAD((ch + 1) * GF_KC)  // in flight during this chunk's MFMAs
            GB_MMA(ch & 1)
            GB_LSTORE((ch + 1) & 1)     // the other buffer: its last readers passed the previous barrier
            __syncthreads();
        }
        GB_EPI_LOAD()
        GB_MMA((nch - 1) & 1)
        __syncthreads();  // every wave is done reading the chunk buffers before sC overwrites them
#undef GB_GLOAD
#undef GB_LSTORE
#undef GB_MMA
    } else {
        GB_EPI_LOAD()
    }
#undef GB_EPI_LOAD
    // accumulator -> LDS (sC [128][LDC]): lane holds unit li of rows (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
    float *const sC = smem;
#pragma unroll
    for (int e = 0; e < 16; ++e) sC[(wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * LDC + li] = acc[e];
    __syncthreads();

    float4 sr = make_float4(0.f, 0.f, 0.f, 0.f), sz = sr, sn = sr, shn = sr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = lr + 32 * i;
        const int64_t b = row0 + row;
        if (b >= B) continue;
        const int64_t o = b * H + u0 + lc;
        const float *pc = sC + row * LDC + lc;
        const float4 ai = *(const float4 *)(S.a + o);
        const float4 v = make_float4(pc[0] + ai.x, pc[1] + ai.y, pc[2] + ai.z, pc[3] + ai.w);
        if (!gates) {
            *(float4 *)(S.a + o) = v;
            continue;
        }
        const float m = S.m_next ? S.m_next[b] : 1.0f;
        const float4 d = S.dout ? *(const float4 *)(S.dout + o) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 hp = *(const float4 *)(S.hm + o);
        const float4 r = es[i][0], z = es[i][1], n = es[i][2], hn = es[i][3];
        float4 a, dr, dz, dn, dhn;
#define CN_GBWD(c)                                                  \
    {                                                               \
        const float gc = v.c * m + d.c;                             \
        const float dnc = gc * (1.0f - z.c) * (1.0f - n.c * n.c);   \
        const float dzc = gc * (hp.c - n.c) * z.c * (1.0f - z.c);   \
        const float drc = dnc * hn.c * r.c * (1.0f - r.c);          \
        a.c = gc * z.c;                                             \
        dr.c = drc;                                                 \
        dz.c = dzc;                                                 \
        dn.c = dnc;                                                 \
        dhn.c = dnc * r.c;                                          \
        sr.c += drc; sz.c += dzc; sn.c += dnc; shn.c += dhn.c;      \
    }
        CN_GBWD(x) CN_GBWD(y) CN_GBWD(z) CN_GBWD(w)
#undef CN_GBWD
        *(float4 *)(S.a + o) = a;
        float *gr = S.g + b * 4 * H + u0 + lc;
        *(float4 *)(gr) = dn;
        *(float4 *)(gr + H) = dr;
        *(float4 *)(gr + 2 * H) = dz;
        *(float4 *)(gr + 3 * H) = dhn;
    }
    if (!gates) return;
    // column sums of the tile (32 units x 4 gates) over its 128 rows: thread rows in order through LDS
    float *const red = smem + GF_BM * LDC;
    float *rw = red + tid * 16;
    *(float4 *)(rw) = sr;
    *(float4 *)(rw + 4) = sz;
    *(float4 *)(rw + 8) = sn;
    *(float4 *)(rw + 12) = shn;
    __syncthreads();
    if (tid >= 4 * GF_BU) return;
    const int q = tid / GF_BU, cu = tid - q * GF_BU;
    const float *src = red + (cu >> 2) * 16 + q * 4 + (cu & 3);
    float s = 0.0f;
    for (int r = 0; r < 32; ++r) s += src[r * 8 * 16];
    S.part[(int64_t)rt * 4 * H + q * H + u0 + cu] = s;
}

// ------------------------------------------------------------------------------------------------
// The act() tail of the Box-action policy (distributions.py:74-94 DiagGaussian + FixedNormal, with the
// reference's operation order and torch's float32 arithmetic): std = exp(0 + logstd) (AddBias on zeros),
// action = eps * std + mean (sample; eps = torch.randn) or mean (mode), and
//   log_prob = sum_a [ -((action - mean)^2) / (2 std^2) - log(std) - log(sqrt(2 pi)) ]
// one thread per env: ~15 tiny torch launches per act() in one (the HIP-graph rollout replays them all).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cn_gaussian_act_kernel(int64_t E, int A, const float *__restrict__ mean,
                                                              const float *__restrict__ logstd,
                                                              const float *__restrict__ eps,
                                                              float *__restrict__ action, float *__restrict__ logp)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const float c = 0.9189385332046727f;   // math.log(math.sqrt(2 * math.pi)) as torch's float32 scalar
    float lp = 0.0f;
    for (int a = 0; a < A; ++a) {
        const float sd = expf(0.0f + logstd[a]);
        const float mu = mean[e * A + a];
        const float x = eps ? eps[e * A + a] * sd + mu : mu;
        action[e * A + a] = x;
        const float d = x - mu;
        const float var = sd * sd;
        const float t = -(d * d) / (2.0f * var) - logf(sd) - c;
        lp = a ? lp + t : t;
    }
    logp[e] = lp;
}

// ------------------------------------------------------------------------------------------------
// Split-K variants for launches with few rows (the DSRNN node GRU: 2,048 x 128 per PPO minibatch, the
// rollout's 4,096-row node step): with 128-row tiles such a launch has fewer workgroups than CUs and each
// wave runs the whole K chain (node GRU: 16 row tiles x 4 unit tiles = 64 workgroups, 5 us of MFMA per
// wave). Here a workgroup owns 32 rows x 32 hidden units and its 4 waves split K (wave w takes K chunks
// w, w + 4, ...), loading their MFMA operands straight from global memory into registers in the
// instruction's layout (lane (i, p) holds row / unit i at k = 8q + 4p .. + 3 of chunk q: no LDS staging);
// the 4 partial tiles are summed through LDS in wave order (deterministic), then the same epilogue
// arithmetic as the 128-row kernels runs with one output row x 4 units per thread.
// ------------------------------------------------------------------------------------------------
constexpr int SK_BM = 32;

template <bool XM>
__global__ __launch_bounds__(256) void cn_gru_fused_sk_kernel(const GfArgs P)
{
    __shared__ float sP[4][XM ? 4 : 3][SK_BM][33];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, k = bid >> 3;
    const int unit_tiles = P.unit_tiles, H = P.H;
    const int ut = k % unit_tiles;
    int rt = (k / unit_tiles) * 8 + xcd;
    if (rt >= P.rt_total) return;  // grid padding (whole workgroup, before any barrier)
    const bool second = rt >= P.rt0;
    const GfSeg S = second ? P.s1 : P.s0;
    if (second) rt -= P.rt0;
    const int64_t B = S.B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, p4 = (lane >> 5) * 4;
    const int64_t row0 = (int64_t)rt * SK_BM;
    const int u0 = ut * GF_BU;
    // epilogue map: thread -> row er, units u0 + lc .. + 3; its operands are requested first
    const int er = tid >> 3, lc = (tid & 7) * 4;
    const int64_t eb = min(row0 + er, B - 1);
    float4 eg[3];
    if (!XM) {
#pragma unroll
        for (int g = 0; g < 3; ++g) eg[g] = *(const float4 *)(S.gi + eb * 3 * H + g * H + u0 + lc);
    }
    const float4 hp = *(const float4 *)(S.hm + eb * H + u0 + lc);

    // XM: chunks 0 .. F/32 - 1 are x against W_ih (n into acc[3]), then hm against W_hh
    gf_f32x16 acc[XM ? 4 : 3];
#pragma unroll
    for (int g = 0; g < (XM ? 4 : 3); ++g)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = 0.0f;
    const float *pa = S.hm + min(row0 + li, B - 1) * H + p4;
    const float *pb = S.w_hh + (int64_t)(u0 + li) * H + p4;
    const int64_t b_step = (int64_t)H * H;
    const int nch = H / GF_KC;
    const int64_t F = XM ? S.F : 0;
    const int ncx = (int)(F / GF_KC);
    const float *xa = XM ? S.x + min(row0 + li, B - 1) * F + p4 : nullptr;
    const float *xb = XM ? S.w_ih + (int64_t)(u0 + li) * F + p4 : nullptr;
    for (int c = wave; c < ncx + nch; c += 4) {
        const bool isx = c < ncx;
        const float *ap = isx ? xa + c * GF_KC : pa + (c - ncx) * GF_KC;
        const float *bp = isx ? xb + c * GF_KC : pb + (c - ncx) * GF_KC;
        const int64_t bs = isx ? (int64_t)H * F : b_step;
        float4 a[4], b[3][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = *(const float4 *)(ap + 8 * q);
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q) b[g][q] = *(const float4 *)(bp + g * bs + 8 * q);
        if (XM && isx) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].x, b[0][q].x, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].x, b[1][q].x, acc[1], 0, 0, 0);
                acc[XM ? 3 : 2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].x, b[2][q].x, acc[XM ? 3 : 2], 0, 0, 0);
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].y, b[0][q].y, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].y, b[1][q].y, acc[1], 0, 0, 0);
                acc[XM ? 3 : 2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].y, b[2][q].y, acc[XM ? 3 : 2], 0, 0, 0);
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].z, b[0][q].z, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].z, b[1][q].z, acc[1], 0, 0, 0);
                acc[XM ? 3 : 2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].z, b[2][q].z, acc[XM ? 3 : 2], 0, 0, 0);
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].w, b[0][q].w, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].w, b[1][q].w, acc[1], 0, 0, 0);
                acc[XM ? 3 : 2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].w, b[2][q].w, acc[XM ? 3 : 2], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].x, b[g][q].x, acc[g], 0, 0, 0);
#pragma unroll
                for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].y, b[g][q].y, acc[g], 0, 0, 0);
#pragma unroll
                for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].z, b[g][q].z, acc[g], 0, 0, 0);
#pragma unroll
                for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].w, b[g][q].w, acc[g], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < (XM ? 4 : 3); ++g)
#pragma unroll
        for (int e = 0; e < 16; ++e) sP[wave][g][(e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)][li] = acc[g][e];
    __syncthreads();
    const int64_t b = row0 + er;
    if (b >= B) return;
    float cs[3][4];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cs[g][j] = ((sP[0][g][er][lc + j] + sP[1][g][er][lc + j]) + sP[2][g][er][lc + j]) + sP[3][g][er][lc + j];
    const float4 cr = make_float4(cs[0][0], cs[0][1], cs[0][2], cs[0][3]);
    const float4 cz = make_float4(cs[1][0], cs[1][1], cs[1][2], cs[1][3]);
    const float4 cn = make_float4(cs[2][0], cs[2][1], cs[2][2], cs[2][3]);
    const float *b_hh = S.b_hh;
    const float4 br = *(const float4 *)(b_hh + u0 + lc), bz = *(const float4 *)(b_hh + H + u0 + lc),
                 bn = *(const float4 *)(b_hh + 2 * H + u0 + lc);
    if (XM) {
        const float *b_ih = S.b_ih;
        float ci[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) ci[j] = ((sP[0][XM ? 3 : 0][er][lc + j] + sP[1][XM ? 3 : 0][er][lc + j]) +
                                             sP[2][XM ? 3 : 0][er][lc + j]) + sP[3][XM ? 3 : 0][er][lc + j];
        const float4 bin = *(const float4 *)(b_ih + 2 * H + u0 + lc);
        eg[0] = *(const float4 *)(b_ih + u0 + lc);
        eg[1] = *(const float4 *)(b_ih + H + u0 + lc);
        eg[2] = make_float4(ci[0] + bin.x, ci[1] + bin.y, ci[2] + bin.z, ci[3] + bin.w);
    }
    const float4 ir = eg[0], iz = eg[1], in = eg[2];
    float4 hr, hz, hn, r, z, n, h;
#define CN_GATE(c)                                 \
    hr.c = cr.c + br.c;                            \
    hz.c = cz.c + bz.c;                            \
    hn.c = cn.c + bn.c;                            \
    r.c = sigm(hr.c + ir.c);                       \
    z.c = sigm(hz.c + iz.c);                       \
    n.c = tanhf(in.c + hn.c * r.c);                \
    h.c = (hp.c - n.c) * z.c + n.c;
    CN_GATE(x) CN_GATE(y) CN_GATE(z) CN_GATE(w)
#undef CN_GATE
    const int64_t o = b * H + u0 + lc;
    *(float4 *)(S.h_out + o) = h;
    if (S.h_out2) {
        float *d = S.h_out2 + (b / S.g2) * S.ld2 + (b % S.g2) * H + u0 + lc;
        d[0] = h.x;
        d[1] = h.y;
        d[2] = h.z;
        d[3] = h.w;
    }
    if (S.hm_next) {
        const float m = S.m_next ? S.m_next[b] : 1.0f;
        *(float4 *)(S.hm_next + o) = make_float4(h.x * m, h.y * m, h.z * m, h.w * m);
    }
    if (S.save) {
        float *sv = S.save + b * 4 * H + u0 + lc;
        *(float4 *)(sv) = r;
        *(float4 *)(sv + H) = z;
        *(float4 *)(sv + 2 * H) = n;
        *(float4 *)(sv + 3 * H) = hn;
    }
}

__global__ __launch_bounds__(256) void cn_gru_bwd_sk_kernel(const GbArgs P)
{
    __shared__ float sP[4][SK_BM][33];
    __shared__ float red[256 * 16];
    const int bid = blockIdx.x;
    const int xcd = bid & 7, k = bid >> 3;
    const int unit_tiles = P.unit_tiles, H = P.H;
    const int ut = k % unit_tiles;
    int rt = (k / unit_tiles) * 8 + xcd;
    if (rt >= P.rt_total) return;  // grid padding (whole workgroup, before any barrier)
    const bool second = rt >= P.rt0;
    const GbSeg S = second ? P.s1 : P.s0;
    if (second) rt -= P.rt0;
    const int64_t B = S.B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, p4 = (lane >> 5) * 4;
    const int64_t row0 = (int64_t)rt * SK_BM;
    const int u0 = ut * GF_BU;
    const int er = tid >> 3, lc = (tid & 7) * 4;
    const int64_t eb = min(row0 + er, B - 1);
    const bool gates = S.g != nullptr;
    const int64_t eo = eb * H + u0 + lc;
    // epilogue operands first (they do not depend on the GEMM)
    const float4 ai = *(const float4 *)(S.a + eo);
    float4 es[4], d = make_float4(0.f, 0.f, 0.f, 0.f), hp = d;
    float m = 1.0f;
    if (gates) {
        const float *sv = S.save + eb * 4 * H + u0 + lc;
#pragma unroll
        for (int q = 0; q < 4; ++q) es[q] = *(const float4 *)(sv + q * H);
        hp = *(const float4 *)(S.hm + eo);
        if (S.dout) d = *(const float4 *)(S.dout + eo);
        if (S.m_next) m = S.m_next[eb];
    }
    gf_f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
    if (S.gk) {
        const int K3 = 3 * H;
        const float *pa = S.gk + min(row0 + li, B - 1) * 4 * H + H + p4;
        const float *pb = S.wt + (int64_t)(u0 + li) * K3 + p4;
        const int nch = K3 / GF_KC;
        for (int c = wave; c < nch; c += 4) {
            const int kc = c * GF_KC;
            float4 a[4], bv[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] = *(const float4 *)(pa + kc + 8 * q);
                bv[q] = *(const float4 *)(pb + kc + 8 * q);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].x, bv[q].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].y, bv[q].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].z, bv[q].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q].w, bv[q].w, acc, 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) sP[wave][(e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)][li] = acc[e];
    __syncthreads();
    const int64_t b = row0 + er;
    const bool live = b < B;
    float4 sr = make_float4(0.f, 0.f, 0.f, 0.f), sz = sr, sn = sr, shn = sr;
    if (live) {
        float cs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) cs[j] = ((sP[0][er][lc + j] + sP[1][er][lc + j]) + sP[2][er][lc + j]) + sP[3][er][lc + j];
        const float4 v = make_float4(cs[0] + ai.x, cs[1] + ai.y, cs[2] + ai.z, cs[3] + ai.w);
        const int64_t o = b * H + u0 + lc;
        if (!gates) {
            *(float4 *)(S.a + o) = v;
        } else {
            const float4 r = es[0], z = es[1], n = es[2], hn = es[3];
            float4 a, dr, dz, dn, dhn;
#define CN_GBWD(c)                                                  \
    {                                                               \
        const float gc = v.c * m + d.c;                             \
        const float dnc = gc * (1.0f - z.c) * (1.0f - n.c * n.c);   \
        const float dzc = gc * (hp.c - n.c) * z.c * (1.0f - z.c);   \
        const float drc = dnc * hn.c * r.c * (1.0f - r.c);          \
        a.c = gc * z.c;                                             \
        dr.c = drc;                                                 \
        dz.c = dzc;                                                 \
        dn.c = dnc;                                                 \
        dhn.c = dnc * r.c;                                          \
        sr.c = drc; sz.c = dzc; sn.c = dnc; shn.c = dhn.c;          \
    }
            CN_GBWD(x) CN_GBWD(y) CN_GBWD(z) CN_GBWD(w)
#undef CN_GBWD
            *(float4 *)(S.a + o) = a;
            float *gr = S.g + b * 4 * H + u0 + lc;
            *(float4 *)(gr) = dn;
            *(float4 *)(gr + H) = dr;
            *(float4 *)(gr + 2 * H) = dz;
            *(float4 *)(gr + 3 * H) = dhn;
        }
    }
    if (!gates) return;
    // column sums of the tile (32 units x 4 gates) over its 32 rows, in row order through LDS
    float *rw = red + tid * 16;
    *(float4 *)(rw) = sr;
    *(float4 *)(rw + 4) = sz;
    *(float4 *)(rw + 8) = sn;
    *(float4 *)(rw + 12) = shn;
    __syncthreads();
    if (tid >= 4 * GF_BU) return;
    const int q = tid / GF_BU, cu = tid - q * GF_BU;
    const float *src = red + (cu >> 2) * 16 + q * 4 + (cu & 3);
    float s = 0.0f;
    for (int r = 0; r < SK_BM; ++r) s += src[r * 8 * 16];
    S.part[(int64_t)rt * 4 * H + q * H + u0 + cu] = s;
}

// CUs of the current device (256 on the MI355X), read once per device: the split-K choice below, and with
// it the workspace sizing of cn_gru_bwd_seq_work_elems, follows the part it runs on
static int device_cus()
{
    static int cached[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}

// 128-row tiles unless that leaves fewer workgroups than CUs (then the split-K kernels, 32-row tiles)
static inline bool use_split_k(int64_t rows, int H)
{
    return (rows + GF_BM - 1) / GF_BM * (H / GF_BU) < device_cus();
}
static inline int64_t row_tile(int64_t rows_total, int H) { return use_split_k(rows_total, H) ? SK_BM : GF_BM; }

// ------------------------------------------------------------------------------------------------
// Generalized advantage estimation (storage.py:132-177, use_gae with use_proper_time_limits): one thread per
// env scans the steps backwards with the reference's float32 operation order
//   delta = ((r[s] + (gamma * v[s+1]) * m[s+1]) - v[s]);  gae = delta + (gl * m[s+1]) * gae;  gae *= bm[s+1]
//   ret[s] = gae + v[s]
// (gl = gamma * gae_lambda rounded once to float, as torch's scalar operands are): ~11 tiny torch launches
// per step (1,400 per rollout) in one.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cn_gae_kernel(int T, int64_t E, float gamma, float gl, int time_limits,
                                                     const float *__restrict__ r, const float *__restrict__ v,
                                                     const float *__restrict__ m, const float *__restrict__ bm,
                                                     float *__restrict__ ret)
{
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    float gae = 0.0f;
    for (int s = T - 1; s >= 0; --s) {
        const float v1 = v[(int64_t)(s + 1) * E + e], m1 = m[(int64_t)(s + 1) * E + e], v0 = v[(int64_t)s * E + e];
        const float delta = (r[(int64_t)s * E + e] + (gamma * v1) * m1) - v0;
        gae = delta + (gl * m1) * gae;
        if (time_limits) gae = gae * bm[(int64_t)(s + 1) * E + e];
        ret[(int64_t)s * E + e] = gae + v0;
    }
}

static int launch_fwd_fused(hipStream_t st, GfArgs &P, int64_t B0, int64_t B1, int H)
{
    const int64_t bm = row_tile(B0 + B1, H);
    const int64_t rt0 = (B0 + bm - 1) / bm, rt1 = (B1 + bm - 1) / bm;
    const int ut = H / GF_BU;
    const int64_t grid = (rt0 + rt1 + 7) / 8 * 8 * ut;
    if (grid > 0x7fffffff) return cn_set_error(CN_EINVAL, "fused GRU step: B too large");
    P.rt0 = (int)rt0;
    P.rt_total = (int)(rt0 + rt1);
    P.unit_tiles = ut;
    P.H = H;
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    const bool xm = P.s0.x != nullptr;
    if (bm == SK_BM) {
        if (xm)
            hipLaunchKernelGGL(cn_gru_fused_sk_kernel<true>, dim3((unsigned)grid), dim3(256), 0, st, P);
        else
            hipLaunchKernelGGL(cn_gru_fused_sk_kernel<false>, dim3((unsigned)grid), dim3(256), 0, st, P);
    } else {
        if (xm)
            hipLaunchKernelGGL(cn_gru_fused_kernel<true>, dim3((unsigned)grid), dim3(256), 0, st, P);
        else
            hipLaunchKernelGGL(cn_gru_fused_kernel<false>, dim3((unsigned)grid), dim3(256), 0, st, P);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

}  // namespace

extern "C" {

int cn_gru_fwd_step(void *stream, int64_t B, int H, const float *gi, const float *gh, const float *hm,
                    const float *m_next, float *h_out, float *hm_next, float *save)
{
    return cn_gru_fwd_step_scatter(stream, B, H, gi, gh, hm, m_next, h_out, hm_next, save, nullptr, 1, 0);
}

int cn_gru_fwd_step_scatter(void *stream, int64_t B, int H, const float *gi, const float *gh, const float *hm,
                         const float *m_next, float *h_out, float *hm_next, float *save, float *h_out2, int64_t g2,
                         int64_t ld2)
{
    if (B <= 0 || H <= 0 || (H & 3)) return cn_set_error(CN_EINVAL, "cn_gru_fwd_step: B > 0 and H % 4 == 0 required");
    if (!gi || !gh || !hm || !h_out) return cn_set_error(CN_EINVAL, "cn_gru_fwd_step: null operand");
    if (B * (H / 4) > (int64_t)0xffffffff * 256) return cn_set_error(CN_EINVAL, "cn_gru_fwd_step: B too large");
    if (h_out2 && (g2 <= 0 || ld2 < g2 * H || (ld2 & 3) || ((uintptr_t)h_out2 & 15)))
        return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_scatter: g2 > 0, ld2 >= g2 * H, ld2 % 4 == 0, 16-byte aligned h_out2");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gru_fwd_kernel, dim3(grid_for(B, H)), dim3(256), 0, (hipStream_t)stream, B, H, gi, gh,
                       hm, m_next, h_out, hm_next, save, h_out2, h_out2 ? g2 : (int64_t)1, ld2);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_gru_fwd_fused(void *stream, int64_t B, int H, const float *gi, const float *hm, const float *w_hh,
                     const float *b_hh, const float *m_next, float *h_out, float *hm_next, float *save, float *h_out2,
                     int64_t g2, int64_t ld2)
{
    if (B <= 0 || H <= 0 || H % GF_BU) return cn_set_error(CN_EINVAL, "cn_gru_fwd_fused: B > 0 and H % 32 == 0 required");
    if (!gi || !hm || !w_hh || !b_hh || !h_out) return cn_set_error(CN_EINVAL, "cn_gru_fwd_fused: null operand");
    // every operand the kernel touches with 16-byte vectors (float4 loads of hm, w_hh, gi, b_hh; float4 stores
    // of h_out, hm_next, save); h_out2 is checked below
    if ((((uintptr_t)hm) | ((uintptr_t)w_hh) | ((uintptr_t)gi) | ((uintptr_t)b_hh) | ((uintptr_t)h_out) |
         ((uintptr_t)hm_next) | ((uintptr_t)save)) & 15)
        return cn_set_error(CN_EINVAL, "cn_gru_fwd_fused: hm, w_hh, gi, b_hh, h_out, hm_next and save must be 16-byte aligned");
    if (h_out2 && (g2 <= 0 || ld2 < g2 * H))
        return cn_set_error(CN_EINVAL, "cn_gru_fwd_fused: g2 > 0 and ld2 >= g2 * H required");
    GfArgs P{};
    P.s0 = GfSeg{B, gi, hm, w_hh, b_hh, m_next, h_out, hm_next, save, h_out2, h_out2 ? g2 : (int64_t)1, ld2,
                 nullptr, nullptr, nullptr, 0};
    P.s1 = P.s0;
    return launch_fwd_fused((hipStream_t)stream, P, B, 0, H);
}

int cn_gae(void *stream, int T, int64_t E, float gamma, float gamma_lambda, int use_proper_time_limits,
           const float *rewards, const float *values, const float *masks, const float *bad_masks, float *returns)
{
    if (T <= 0 || E <= 0) return cn_set_error(CN_EINVAL, "cn_gae: T > 0 and E > 0 required");
    if (!rewards || !values || !masks || !returns || (use_proper_time_limits && !bad_masks))
        return cn_set_error(CN_EINVAL, "cn_gae: null operand");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gae_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T, E, gamma,
                       gamma_lambda, use_proper_time_limits, rewards, values, masks, bad_masks, returns);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_gaussian_act(void *stream, int64_t E, int A, const float *mean, const float *logstd, const float *eps,
                    float *action, float *logp)
{
    if (E <= 0 || A <= 0 || A > 64) return cn_set_error(CN_EINVAL, "cn_gaussian_act: E > 0 and 0 < A <= 64 required");
    if (!mean || !logstd || !action || !logp) return cn_set_error(CN_EINVAL, "cn_gaussian_act: null operand");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gaussian_act_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       E, A, mean, logstd, eps, action, logp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

static bool aligned16(std::initializer_list<const void *> ps)
{
    for (const void *p : ps)
        if ((uintptr_t)p & 15) return false;
    return true;
}

int cn_gru_fwd_step_group(void *stream, int H, int nseg, const cn_gru_step_seg *segs)
{
    if (H <= 0 || H % GF_BU || nseg < 1 || nseg > 2 || !segs)
        return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: H % 32 == 0 and 1 <= nseg <= 2 required");
    GfArgs P{};
    for (int s = 0; s < nseg; ++s) {
        const cn_gru_step_seg &q = segs[s];
        if (q.B <= 0 || !q.hm || !q.w_hh || !q.b_hh || !q.h_out)
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: B > 0 and hm, w_hh, b_hh, h_out required");
        if ((q.x != nullptr) != (segs[0].x != nullptr))
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: every GRU of a call passes gi, or every GRU x");
        if (q.x ? (!q.w_ih || !q.b_ih || q.F <= 0 || q.F % GF_KC) : !q.gi)
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: gi, or x with w_ih, b_ih and F % 32 == 0, required");
        if (!aligned16({q.gi, q.x, q.w_ih, q.b_ih, q.hm, q.w_hh, q.b_hh, q.h_out}))
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: every array must be 16-byte aligned");
        if (q.h_out2 && (q.g2 <= 0 || q.ld2 < q.g2 * H))
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_step_group: g2 > 0 and ld2 >= g2 * H required");
        GfSeg g{q.B, q.gi, q.hm, q.w_hh, q.b_hh, nullptr, q.h_out, nullptr, nullptr, q.h_out2,
                q.h_out2 ? q.g2 : (int64_t)1, q.ld2, q.x, q.w_ih, q.b_ih, q.F};
        (s ? P.s1 : P.s0) = g;
    }
    if (nseg == 1) P.s1 = P.s0;
    return launch_fwd_fused((hipStream_t)stream, P, segs[0].B, nseg > 1 ? segs[1].B : 0, H);
}

int cn_gru_fwd_seq(void *stream, int T, int H, int nseg, const cn_gru_seq_fwd *segs)
{
    if (T <= 0 || H <= 0 || H % GF_BU || nseg < 1 || nseg > 2 || !segs)
        return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: T > 0, H % 32 == 0 and 1 <= nseg <= 2 required");
    for (int s = 0; s < nseg; ++s) {
        const cn_gru_seq_fwd &q = segs[s];
        if (q.B <= 0 || q.nh < 1 || q.nh > T) return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: B > 0 and 1 <= nh <= T required");
        // step t reads hm[t % nh] in every workgroup while others write their columns of hm[(t + 1) % nh]: with
        // nh == 1 and T > 1 those are the same rows (a cross-workgroup race); the backward reads hm of every step
        if (T > 1 && q.nh < 2) return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: nh >= 2 required when T > 1");
        if (q.save && q.nh != T) return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: nh == T required with save");
        if (!q.w_hh || !q.b_hh || !q.m || !q.out || !q.hm) return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: null operand");
        if ((q.x != nullptr) != (segs[0].x != nullptr))
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: every GRU of a call passes gi, or every GRU x / w_ih / b_ih");
        if (q.x ? (!q.w_ih || !q.b_ih || q.F <= 0 || q.F % GF_KC) : !q.gi)
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: gi, or x with w_ih, b_ih and F % 32 == 0, required");
        if (!aligned16({q.gi, q.w_hh, q.b_hh, q.out, q.hm, q.save, q.x, q.w_ih, q.b_ih}))
            return cn_set_error(CN_EINVAL, "cn_gru_fwd_seq: every array must be 16-byte aligned");
    }
    const int64_t B1 = nseg > 1 ? segs[1].B : 0;
    for (int t = 0; t < T; ++t) {
        GfArgs P{};
        for (int s = 0; s < nseg; ++s) {
            const cn_gru_seq_fwd &q = segs[s];
            const bool last = t + 1 == T;
            const int64_t BH = q.B * H;
            GfSeg g{q.B, q.gi ? q.gi + t * 3 * BH : nullptr, q.hm + (t % q.nh) * BH, q.w_hh, q.b_hh,
                    last ? nullptr : q.m + (t + 1) * q.B, q.out + t * BH,
                    last ? nullptr : q.hm + ((t + 1) % q.nh) * BH, q.save ? q.save + t * 4 * BH : nullptr, nullptr,
                    1, 0,
                    q.x ? q.x + t * q.B * q.F : nullptr, q.w_ih, q.b_ih, q.F};
            (s ? P.s1 : P.s0) = g;
        }
        if (nseg == 1) P.s1 = P.s0;
        const int rc = launch_fwd_fused((hipStream_t)stream, P, segs[0].B, B1, H);
        if (rc) return rc;
    }
    return CN_OK;
}

// workspace of cn_gru_bwd_seq: per GRU the bias partials [T][row tiles][4H], then cn_gru_bias_reduce's work
static int64_t bwd_part_rows(int64_t B, int64_t bm) { return (B + bm - 1) / bm; }

int64_t cn_gru_bwd_seq_work_elems(int T, int H, int nseg, const cn_gru_seq_bwd *segs)
{
    if (T <= 0 || H <= 0 || nseg < 1 || nseg > 2 || !segs) return 0;
    const int64_t rows = segs[0].B + (nseg > 1 ? segs[1].B : 0);
    const int64_t bm = row_tile(rows, H);
    int64_t n = (int64_t)CN_GB_RC * 4 * H;
    for (int s = 0; s < nseg; ++s) n += (int64_t)T * bwd_part_rows(segs[s].B, bm) * 4 * H;
    return n;
}

int cn_gru_bwd_seq(void *stream, int T, int H, int nseg, const cn_gru_seq_bwd *segs, float *work, int64_t work_elems)
{
    if (T <= 0 || H <= 0 || H % GF_BU || nseg < 1 || nseg > 2 || !segs)
        return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: T > 0, H % 32 == 0 and 1 <= nseg <= 2 required");
    if (!work) return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: null workspace");
    for (int s = 0; s < nseg; ++s) {
        const cn_gru_seq_bwd &q = segs[s];
        if (q.B <= 0) return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: B > 0 required");
        if (!q.w_hh_t || !q.m || !q.save || !q.hm || !q.acc || !q.g || !q.db_ih || !q.db_hh)
            return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: null operand");
        if (!aligned16({q.w_hh_t, q.dout, q.save, q.hm, q.acc, q.g}))
            return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: w_hh_t, dout, save, hm, acc and g must be 16-byte aligned");
    }
    // the row tiling (and with it the workspace) follows the CU count of the CURRENT device: a workspace sized on
    // another device may be too small for this one's choice
    if (work_elems < cn_gru_bwd_seq_work_elems(T, H, nseg, segs))
        return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: workspace smaller than cn_gru_bwd_seq_work_elems on this device");
    const int ut = H / GF_BU;
    const int64_t bm = row_tile(segs[0].B + (nseg > 1 ? segs[1].B : 0), H);
    const int64_t rt0 = bwd_part_rows(segs[0].B, bm), rt1 = nseg > 1 ? bwd_part_rows(segs[1].B, bm) : 0;
    const int64_t grid = (rt0 + rt1 + 7) / 8 * 8 * ut;
    if (grid > 0x7fffffff) return cn_set_error(CN_EINVAL, "cn_gru_bwd_seq: B too large");
    float *part[2] = {work, work + (int64_t)T * rt0 * 4 * H};
    float *red = part[1] + (int64_t)T * rt1 * 4 * H;
    // launch j = 0 .. T: the GEMM of step T - j (none at j = 0) and the gates of step T - 1 - j (none at j = T)
    for (int j = 0; j <= T; ++j) {
        GbArgs P{};
        P.rt0 = (int)rt0;
        P.rt_total = (int)(rt0 + rt1);
        P.unit_tiles = ut;
        P.H = H;
        for (int s = 0; s < nseg; ++s) {
            const cn_gru_seq_bwd &q = segs[s];
            const int64_t BH = q.B * H, rt = s ? rt1 : rt0;
            const int tk = T - j, tg = T - 1 - j;
            const bool gates = tg >= 0;
            GbSeg g{q.B,
                    j ? q.g + tk * 4 * BH : nullptr,
                    q.w_hh_t,
                    q.acc,
                    (gates && tg + 1 < T) ? q.m + (tg + 1) * q.B : nullptr,
                    (gates && q.dout) ? q.dout + tg * BH : nullptr,
                    gates ? q.save + tg * 4 * BH : nullptr,
                    gates ? q.hm + tg * BH : nullptr,
                    gates ? q.g + tg * 4 * BH : nullptr,
                    gates ? part[s] + tg * rt * 4 * H : nullptr};
            (s ? P.s1 : P.s0) = g;
        }
        if (nseg == 1) P.s1 = P.s0;
        (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
        if (bm == SK_BM)
            hipLaunchKernelGGL(cn_gru_bwd_sk_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, P);
        else
            hipLaunchKernelGGL(cn_gru_bwd_fused_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, P);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return cn_set_error(CN_EHIP, hipGetErrorString(e));
    }
    // bias gradients: every step's workgroup partials of each GRU, summed in a fixed order
    for (int s = 0; s < nseg; ++s) {
        const int rc = cn_gru_bias_reduce(stream, (int64_t)T * (s ? rt1 : rt0), H, part[s], segs[s].db_ih,
                                          segs[s].db_hh, red);
        if (rc) return rc;
    }
    return CN_OK;
}

int64_t cn_gru_bias_blocks(int64_t B) { return (B + CN_GB_RW - 1) / CN_GB_RW; }

int cn_gru_bwd_step_bias(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                         const float *save, const float *hm, float *dgi, float *dgh, float *part)
{
    if (B <= 0 || !(H == 64 || H == 128 || H == 256)) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step_bias: H in {64, 128, 256}");
    if (!acc || !save || !hm || !dgi || !dgh || !part) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step_bias: null operand");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gru_bwd_bias_kernel<false>, dim3((unsigned)cn_gru_bias_blocks(B)), dim3(256), 0, (hipStream_t)stream,
                       B, H, acc, m_next, dout, save, hm, dgi, dgh, part);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_gru_bwd_step_gates(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                          const float *save, const float *hm, float *g, float *part)
{
    if (B <= 0 || !(H == 64 || H == 128 || H == 256)) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step_gates: H in {64, 128, 256}");
    if (!acc || !save || !hm || !g || !part) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step_gates: null operand");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gru_bwd_bias_kernel<true>, dim3((unsigned)cn_gru_bias_blocks(B)), dim3(256), 0, (hipStream_t)stream,
                       B, H, acc, m_next, dout, save, hm, g, nullptr, part);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int64_t cn_gru_bias_work_elems(int H) { return (int64_t)CN_GB_RC * 4 * H; }

int cn_gru_bias_reduce(void *stream, int64_t rows, int H, const float *part, float *db_ih, float *db_hh,
                       float *work)
{
    if (rows <= 0 || H <= 0 || (H & 3)) return cn_set_error(CN_EINVAL, "cn_gru_bias_reduce: bad shape");
    if (!part || !db_ih || !db_hh || !work) return cn_set_error(CN_EINVAL, "cn_gru_bias_reduce: null operand");
    (void)hipGetLastError();
    hipLaunchKernelGGL(cn_gru_bias_part2_kernel, dim3((unsigned)((4 * H + 63) / 64), CN_GB_RC), dim3(256), 0,
                       (hipStream_t)stream, rows, H, part, work);
    hipLaunchKernelGGL(cn_gru_bias_final_kernel, dim3((unsigned)((4 * H + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, H, (const float *)work, db_ih, db_hh);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_gru_bwd_step(void *stream, int64_t B, int H, float *acc, const float *m_next, const float *dout,
                    const float *save, const float *hm, float *dgi, float *dgh)
{
    if (B <= 0 || H <= 0 || (H & 3)) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step: B > 0 and H % 4 == 0 required");
    if (!acc || !save || !hm || !dgi || !dgh) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step: null operand");
    if (B * (H / 4) > (int64_t)0xffffffff * 256) return cn_set_error(CN_EINVAL, "cn_gru_bwd_step: B too large");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_gru_bwd_kernel, dim3(grid_for(B, H)), dim3(256), 0, (hipStream_t)stream, B, H, acc,
                       m_next, dout, save, hm, dgi, dgh);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Attention pooling of the spatial edge states (EdgeAttention.forward, srnn_model.py:320-333):
//   out[r][h] = sum_n hs[r][n][h] * attn[r][n]          (the reference's bmm(hs^T, attn))
// and its gradient. HBM-bound: one read of hs forward; one read of hs + one write of d_hs backward.
// One thread per (r, 4 consecutive h); the backward reduces d_attn[r][n] = sum_h dout[r][h] hs[r][n][h]
// over the row's H / 4 threads with a fixed-order tree (deterministic).
// ------------------------------------------------------------------------------------------------
namespace {

__global__ __launch_bounds__(256) void cn_attn_pool_fwd_kernel(int64_t R, int N, int H, const float *__restrict__ hs,
                                                               const float *__restrict__ attn,
                                                               float *__restrict__ out)
{
    const int H4 = H >> 2;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R * H4) return;
    const int64_t r = i / H4;
    const int j = (int)(i - r * H4) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int n = 0; n < N; ++n) {
        const float a = attn[r * N + n];
        const float4 v = *(const float4 *)(hs + (r * N + n) * H + j);
        acc.x += v.x * a; acc.y += v.y * a; acc.z += v.z * a; acc.w += v.w * a;
    }
    *(float4 *)(out + r * H + j) = acc;
}

// block = 256 threads = 256 / (H / 4) rows; H / 4 must be a power of two <= 64 (one wave or less per row)
template <int HQ>
__global__ __launch_bounds__(256) void cn_attn_pool_bwd_kernel(int64_t R, int N, const float *__restrict__ hs,
                                                               const float *__restrict__ attn,
                                                               const float *__restrict__ dout,
                                                               float *__restrict__ dhs, float *__restrict__ dattn)
{
    constexpr int H = HQ * 4;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = i / HQ;
    const int q = (int)(i - r * HQ);
    const bool ok = r < R;
    const int j = q * 4;
    const float4 g = ok ? *(const float4 *)(dout + r * H + j) : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int n = 0; n < N; ++n) {
        float part = 0.0f;
        if (ok) {
            const float a = attn[r * N + n];
            const float4 v = *(const float4 *)(hs + (r * N + n) * H + j);
            *(float4 *)(dhs + (r * N + n) * H + j) = make_float4(g.x * a, g.y * a, g.z * a, g.w * a);
            part = ((g.x * v.x + g.y * v.y) + g.z * v.z) + g.w * v.w;
        }
#pragma unroll
        for (int o = HQ / 2; o; o >>= 1) part += __shfl_xor(part, o);
        if (ok && q == 0) dattn[r * N + n] = part;
    }
}

// ------------------------------------------------------------------------------------------------
// Whole spatial-edge attention of EdgeAttention.forward (srnn_model.py:256-333) in one pass over hs:
//   score[r][n] = scale * sum_k te[r][k] (Ws hs[r][n] + bs)[k]  = scale * (hs[r][n] . u[r] + c[r]),
//   u = te Ws (R x H), c = te . bs (host GEMM / GEMV, R x A x H: 1/10 of the reference's R*N x H x A),
//   attn = softmax_n(score), out[r] = sum_n attn[r][n] hs[r][n].
// The reference materialises spatial_embed (R*N x 64), the product with temporal_embed and its sum,
// then reads hs again for the pooling; here hs is read once (the first 16 of a row's N vectors stay in
// registers between the score and pooling passes). Same quantity, reassociated (fp32 rounding level).
// One thread per (row, 4 consecutive h): HQ = H / 4 lanes per row, rows never straddle a wave; the
// row's scores go through LDS (lane 0 of the row writes, the row's lanes read after a barrier).
// ------------------------------------------------------------------------------------------------
#define CN_SA_MAXN 64
// NR: a row's first NR edge vectors stay in registers between the two passes (the rest are read again).
// Instantiated for NR = 10 (N <= 10: C4's rows; backward 79 instead of 103 VGPRs, 6 instead of 4 waves per
// SIMD: 2.05 -> 1.65 ms at C4's 262,144 x 10 x 256, 3.0 -> 3.75 TB/s; forward 0.90 -> 0.85 ms,
// tools/probe_attn.py) and NR = 16.

template <int HQ, int NR>
__global__ __launch_bounds__(256) void cn_spatial_attn_fwd_kernel(int64_t R, int N, float scale,
                                                                  const float *__restrict__ hs,
                                                                  const float *__restrict__ u,
                                                                  const float *__restrict__ c,
                                                                  float *__restrict__ out, float *__restrict__ attn)
{
    constexpr int H = HQ * 4, RB = 256 / HQ;
    __shared__ float sc[RB][CN_SA_MAXN];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = i / HQ;
    const int q = (int)(i - r * HQ), rl = (int)threadIdx.x / HQ;
    const bool ok = r < R;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 uu = ok ? *(const float4 *)(u + r * H + q * 4) : z4;
    const float cr = ok ? c[r] : 0.f;
    const float *hr = hs + (ok ? r : 0) * (int64_t)N * H + q * 4;
    float4 vc[NR];
    float mx = -INFINITY;
    auto score = [&](int n, const float4 &v) {
        float part = ((uu.x * v.x + uu.y * v.y) + uu.z * v.z) + uu.w * v.w;
#pragma unroll
        for (int o = HQ / 2; o; o >>= 1) part += __shfl_xor(part, o);
        const float s = (part + cr) * scale;
        if (q == 0) sc[rl][n] = s;
        mx = fmaxf(mx, s);
    };
#pragma unroll
    for (int n = 0; n < NR; ++n)
        if (n < N) {
            vc[n] = ok ? *(const float4 *)(hr + n * H) : z4;
            score(n, vc[n]);
        }
    for (int n = NR; n < N; ++n) score(n, ok ? *(const float4 *)(hr + n * H) : z4);
    __syncthreads();
    float den = 0.f;
    for (int n = 0; n < N; ++n) den += expf(sc[rl][n] - mx);
    float4 acc = z4;
    auto pool = [&](int n, const float4 &v) {
        const float a = expf(sc[rl][n] - mx) / den;
        acc.x += v.x * a; acc.y += v.y * a; acc.z += v.z * a; acc.w += v.w * a;
        if (ok && q == 0) attn[r * N + n] = a;
    };
#pragma unroll
    for (int n = 0; n < NR; ++n)
        if (n < N) pool(n, vc[n]);
    for (int n = NR; n < N; ++n) pool(n, ok ? *(const float4 *)(hr + n * H) : z4);
    if (ok) *(float4 *)(out + r * H + q * 4) = acc;
}

// Gradient: p[n] = dout[r] . hs[r][n] (+ the caller's d attn), s = sum_n attn[n] p[n],
// dscore[n] = scale * attn[n] (p[n] - s) (softmax backward), then
//   dhs[r][n] = attn[n] dout[r] + dscore[n] u[r],  du[r] = sum_n dscore[n] hs[r][n],  dc[r] = sum_n dscore[n].
// hs is read once (as forward); dhs written once (it is the spatial GRU output's whole gradient).
template <int HQ, int NR>
__global__ __launch_bounds__(256) void cn_spatial_attn_bwd_kernel(int64_t R, int N, float scale,
                                                                  const float *__restrict__ hs,
                                                                  const float *__restrict__ u,
                                                                  const float *__restrict__ attn,
                                                                  const float *__restrict__ dout,
                                                                  const float *__restrict__ dattn,
                                                                  float *__restrict__ dhs, float *__restrict__ du,
                                                                  int64_t ldu, float *__restrict__ dc, int64_t ldc)
{
    constexpr int H = HQ * 4, RB = 256 / HQ;
    __shared__ float sp[RB][CN_SA_MAXN];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = i / HQ;
    const int q = (int)(i - r * HQ), rl = (int)threadIdx.x / HQ;
    const bool ok = r < R;
    const int64_t rr = ok ? r : 0;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g = ok ? *(const float4 *)(dout + r * H + q * 4) : z4;
    const float4 uu = ok ? *(const float4 *)(u + r * H + q * 4) : z4;
    const float *hr = hs + rr * (int64_t)N * H + q * 4;
    float4 vc[NR];
    float s = 0.f;
    auto grad = [&](int n, const float4 &v) {
        float part = ((g.x * v.x + g.y * v.y) + g.z * v.z) + g.w * v.w;
#pragma unroll
        for (int o = HQ / 2; o; o >>= 1) part += __shfl_xor(part, o);
        if (dattn) part += dattn[rr * N + n];
        if (q == 0) sp[rl][n] = part;
        s += attn[rr * N + n] * part;
    };
#pragma unroll
    for (int n = 0; n < NR; ++n)
        if (n < N) {
            vc[n] = ok ? *(const float4 *)(hr + n * H) : z4;
            grad(n, vc[n]);
        }
    for (int n = NR; n < N; ++n) grad(n, ok ? *(const float4 *)(hr + n * H) : z4);
    __syncthreads();
    float4 acc = z4;
    float dcs = 0.f;
    float *dr = dhs + rr * (int64_t)N * H + q * 4;
    auto back = [&](int n, const float4 &v) {
        const float a = attn[rr * N + n];
        const float ds = scale * (a * (sp[rl][n] - s));
        acc.x += ds * v.x; acc.y += ds * v.y; acc.z += ds * v.z; acc.w += ds * v.w;
        dcs += ds;
        if (ok)
            *(float4 *)(dr + n * H) = make_float4(a * g.x + ds * uu.x, a * g.y + ds * uu.y, a * g.z + ds * uu.z,
                                                  a * g.w + ds * uu.w);
    };
#pragma unroll
    for (int n = 0; n < NR; ++n)
        if (n < N) back(n, vc[n]);
    for (int n = NR; n < N; ++n) back(n, ok ? *(const float4 *)(hr + n * H) : z4);
    if (ok) {
        *(float4 *)(du + r * ldu + q * 4) = acc;
        if (q == 0) dc[r * ldc] = dcs;
    }
}


// ------------------------------------------------------------------------------------------------
// Skinny weight gradient of a Linear layer applied to K >> 1 rows (PPO minibatch: T*B or T*B*N rows):
//   dW[a][j] = sum_k dy'[k][a] x[k][j],  db[a] = sum_k dy'[k][a],  dy' = dy * (relu_out > 0) if given
// for layers whose output or input width is tiny (the DSRNN input encoders: 2 / 3 / 7 inputs; the action
// mean and value heads: 2 / 1 outputs), where a library GEMM walks all of K with a handful of output
// tiles (4.1 ms for the spatial encoder's 64 x 2 gradient over 2.6 M rows). HBM-bound:
// one pass over dy (+ the ReLU output) and x. Each workgroup owns a contiguous run of rows and keeps the
// m*n + m sums of its rows in registers (thread t: slots t, t + 256, ...); the per-workgroup partials are
// then summed in workgroup order by a second kernel (deterministic, no atomics).
// ------------------------------------------------------------------------------------------------
#define CN_WG_MAXSLOT 1024
#define CN_WG_NARROW 8

// Layout: each thread owns VEC consecutive columns of the WIDE operand (dy if DYWIDE, else x; <= 256
// columns, TW = ceil(wide / VEC) threads per row, 256 / TW rows in flight) and all columns of the NARROW
// one (<= 8); rows are read as coalesced vectors. The 256 / TW row slots are summed through LDS in slot
// order, then one partial row of m * n + m sums per workgroup.
template <int VEC, bool DYWIDE>
__global__ __launch_bounds__(256) void cn_wgrad_part_kernel(int64_t K, int m, int n, int TW, int64_t rows,
                                                            const float *__restrict__ dy,
                                                            const float *__restrict__ mo,
                                                            const float *__restrict__ x,
                                                            float *__restrict__ part)
{
    __shared__ float red[256 * (VEC * CN_WG_NARROW + CN_WG_NARROW)];
    constexpr int NA = CN_WG_NARROW, NB = VEC > NA ? VEC : NA;
    const int wide = DYWIDE ? m : n, nar = DYWIDE ? n : m;
    const int RP = 256 / TW, tr = (int)threadIdx.x / TW, tc = (int)threadIdx.x - tr * TW;
    const int c0 = tc * VEC;
    const bool act = tr < RP && c0 < wide;
    const int64_t k0 = (int64_t)blockIdx.x * rows;
    const int64_t k1 = k0 + rows < K ? k0 + rows : K;
    float acc[VEC][NA], dbs[NB];
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int u = 0; u < NA; ++u) acc[v][u] = 0.0f;
#pragma unroll
    for (int u = 0; u < NB; ++u) dbs[u] = 0.0f;
    if (act) {
        for (int64_t k = k0 + tr; k < k1; k += RP) {
            float w[VEC], q[NA];
            const float *wr = DYWIDE ? dy + k * m : x + k * n;
            if (VEC == 4) {
                const float4 t = *(const float4 *)(wr + c0);
                w[0] = t.x; w[1] = t.y; w[2] = t.z; w[3] = t.w;
                if (DYWIDE && mo) {
                    const float4 o = *(const float4 *)(mo + k * m + c0);
                    w[0] = o.x > 0.0f ? w[0] : 0.0f; w[1] = o.y > 0.0f ? w[1] : 0.0f;
                    w[2] = o.z > 0.0f ? w[2] : 0.0f; w[3] = o.w > 0.0f ? w[3] : 0.0f;
                }
            } else {
#pragma unroll
                for (int v = 0; v < VEC; ++v) {
                    w[v] = c0 + v < wide ? wr[c0 + v] : 0.0f;
                    if (DYWIDE && mo && c0 + v < wide && !(mo[k * m + c0 + v] > 0.0f)) w[v] = 0.0f;
                }
            }
            const float *qr = DYWIDE ? x + k * n : dy + k * m;
#pragma unroll
            for (int u = 0; u < NA; ++u) {
                q[u] = u < nar ? qr[u] : 0.0f;
                if (!DYWIDE && mo && u < nar && !(mo[k * m + u] > 0.0f)) q[u] = 0.0f;
            }
#pragma unroll
            for (int v = 0; v < VEC; ++v)
#pragma unroll
                for (int u = 0; u < NA; ++u) acc[v][u] += w[v] * q[u];
            if (DYWIDE) {
#pragma unroll
                for (int v = 0; v < VEC; ++v) dbs[v] += w[v];
            } else {
#pragma unroll
                for (int u = 0; u < NA; ++u) dbs[u] += q[u];
            }
        }
    }
    // sum the RP row slots in slot order: thread (tr, tc) stores its sums, then thread tc of slot 0 adds up
    constexpr int SL = VEC * NA + NA;
    float *mine = red + threadIdx.x * SL;
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int u = 0; u < NA; ++u) mine[v * NA + u] = acc[v][u];
#pragma unroll
    for (int u = 0; u < NA; ++u) mine[VEC * NA + u] = u < NB ? dbs[u] : 0.0f;
    __syncthreads();
    if (tr != 0 || c0 >= wide) return;
    for (int r = 1; r < RP; ++r) {
        const float *o = red + (r * TW + tc) * SL;
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
            for (int u = 0; u < NA; ++u) acc[v][u] += o[v * NA + u];
#pragma unroll
        for (int u = 0; u < NB; ++u) dbs[u] += o[VEC * NA + u];
    }
    const int P = m * n;
    float *pw = part + (int64_t)blockIdx.x * (P + m);
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
        if (c0 + v >= wide) continue;
#pragma unroll
        for (int u = 0; u < NA; ++u) {
            if (u >= nar) continue;
            if (DYWIDE) pw[(c0 + v) * n + u] = acc[v][u];   // dW[a = c0 + v][j = u]
            else pw[u * n + c0 + v] = acc[v][u];            // dW[a = u][j = c0 + v]
        }
        if (DYWIDE) pw[P + c0 + v] = dbs[v];
    }
    if (!DYWIDE && tc == 0)
        for (int u = 0; u < nar; ++u) pw[P + u] = dbs[u];
}

// out[p] = sum over the G workgroup partials in workgroup order (one workgroup per output: strided
// sequential sums, then a fixed-order LDS tree)
__global__ __launch_bounds__(256) void cn_wgrad_sum_kernel(int G, int m, int n, const float *__restrict__ part,
                                                           float *__restrict__ dW, float *__restrict__ db)
{
    __shared__ float red[256];
    const int P = m * n, S = P + m;
    const int p = blockIdx.x;
    float s = 0.0f;
    for (int g = threadIdx.x; g < G; g += 256) s += part[(int64_t)g * S + p];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (p < P) dW[p] = red[0];
        else if (db) db[p - P] = red[0];
    }
}

// rows per workgroup and workgroup count of cn_wgrad for K rows (about four workgroups per CU)
static inline void wgrad_grid(int64_t K, int64_t &rows, int &G)
{
    rows = (K + 1023) / 1024;
    if (rows < 64) rows = 64;
    G = (int)((K + rows - 1) / rows);
}

}  // namespace

extern "C" {

int64_t cn_wgrad_work_elems(int64_t K, int m, int n)
{
    if (K <= 0 || m <= 0 || n <= 0) return 0;
    int64_t rows;
    int G;
    wgrad_grid(K, rows, G);
    return (int64_t)G * (m * n + m);
}

int cn_wgrad(void *stream, int64_t K, int m, int n, const float *dy, const float *relu_out, const float *x,
             float *dW, float *db, float *work)
{
    if (K <= 0 || m <= 0 || n <= 0 || m * n + m > CN_WG_MAXSLOT || (m < n ? m : n) > CN_WG_NARROW ||
        (m > n ? m : n) > 256)
        return cn_set_error(CN_EINVAL, "cn_wgrad: need K > 0, min(m, n) <= 8, max(m, n) <= 256");
    if (!dy || !x || !dW || !work) return cn_set_error(CN_EINVAL, "cn_wgrad: null operand");
    int64_t rows;
    int G;
    wgrad_grid(K, rows, G);
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    const bool dywide = m >= n;
    const int wide = dywide ? m : n;
    const bool v4 = (wide & 3) == 0 && ((uintptr_t)(dywide ? dy : x) & 15) == 0 &&
                    (!dywide || !relu_out || ((uintptr_t)relu_out & 15) == 0);
    const int TW = v4 ? wide / 4 : wide;
    if (dywide && v4)
        hipLaunchKernelGGL((cn_wgrad_part_kernel<4, true>), dim3(G), dim3(256), 0, (hipStream_t)stream, K, m, n, TW,
                           rows, dy, relu_out, x, work);
    else if (dywide)
        hipLaunchKernelGGL((cn_wgrad_part_kernel<1, true>), dim3(G), dim3(256), 0, (hipStream_t)stream, K, m, n, TW,
                           rows, dy, relu_out, x, work);
    else if (v4)
        hipLaunchKernelGGL((cn_wgrad_part_kernel<4, false>), dim3(G), dim3(256), 0, (hipStream_t)stream, K, m, n, TW,
                           rows, dy, relu_out, x, work);
    else
        hipLaunchKernelGGL((cn_wgrad_part_kernel<1, false>), dim3(G), dim3(256), 0, (hipStream_t)stream, K, m, n, TW,
                           rows, dy, relu_out, x, work);
    hipLaunchKernelGGL(cn_wgrad_sum_kernel, dim3(m * n + m), dim3(256), 0, (hipStream_t)stream, G, m, n,
                       (const float *)work, dW, db);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_attn_pool_fwd(void *stream, int64_t R, int N, int H, const float *hs, const float *attn, float *out)
{
    if (R <= 0 || N <= 0 || H <= 0 || (H & 3)) return cn_set_error(CN_EINVAL, "cn_attn_pool_fwd: bad shape");
    if (!hs || !attn || !out) return cn_set_error(CN_EINVAL, "cn_attn_pool_fwd: null operand");
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    hipLaunchKernelGGL(cn_attn_pool_fwd_kernel, dim3(grid_for(R, H)), dim3(256), 0, (hipStream_t)stream, R, N, H, hs,
                       attn, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_attn_pool_bwd(void *stream, int64_t R, int N, int H, const float *hs, const float *attn, const float *dout,
                     float *dhs, float *dattn)
{
    if (R <= 0 || N <= 0 || !(H == 256 || H == 128 || H == 64))
        return cn_set_error(CN_EINVAL, "cn_attn_pool_bwd: H must be 64, 128 or 256");
    if (!hs || !attn || !dout || !dhs || !dattn) return cn_set_error(CN_EINVAL, "cn_attn_pool_bwd: null operand");
    const unsigned grid = grid_for(R, H);
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
    if (H == 256)
        hipLaunchKernelGGL(cn_attn_pool_bwd_kernel<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, R, N, hs, attn,
                           dout, dhs, dattn);
    else if (H == 128)
        hipLaunchKernelGGL(cn_attn_pool_bwd_kernel<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, R, N, hs, attn,
                           dout, dhs, dattn);
    else
        hipLaunchKernelGGL(cn_attn_pool_bwd_kernel<16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, R, N, hs, attn,
                           dout, dhs, dattn);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

static int sa_check(const char *who, int64_t R, int N, int H, std::initializer_list<const void *> vec,
                    std::initializer_list<const void *> other)
{
    if (R <= 0 || N <= 0 || N > CN_SA_MAXN || !(H == 256 || H == 128 || H == 64))
        return cn_set_error(CN_EINVAL, who);
    for (const void *p : vec)
        if (!p || ((uintptr_t)p & 15)) return cn_set_error(CN_EINVAL, who);
    for (const void *p : other)
        if (!p) return cn_set_error(CN_EINVAL, who);
    return CN_OK;
}

int cn_spatial_attn_fwd(void *stream, int64_t R, int N, int H, float scale, const float *hs, const float *u,
                        const float *c, float *out, float *attn)
{
    if (sa_check("cn_spatial_attn_fwd: H in {64, 128, 256}, 1 <= N <= 64, non-null operands, hs / u / out "
                 "16-byte aligned", R, N, H, {hs, u, out}, {c, attn}))
        return CN_EINVAL;
    const unsigned grid = grid_for(R, H);
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
#define CN_SA_FWD(HQ, NR) \
    hipLaunchKernelGGL((cn_spatial_attn_fwd_kernel<HQ, NR>), dim3(grid), dim3(256), 0, (hipStream_t)stream, R, N, scale, \
                       hs, u, c, out, attn)
    if (N <= 10) {
        if (H == 256) CN_SA_FWD(64, 10);
        else if (H == 128) CN_SA_FWD(32, 10);
        else CN_SA_FWD(16, 10);
    } else {
        if (H == 256) CN_SA_FWD(64, 16);
        else if (H == 128) CN_SA_FWD(32, 16);
        else CN_SA_FWD(16, 16);
    }
#undef CN_SA_FWD
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

int cn_spatial_attn_bwd(void *stream, int64_t R, int N, int H, float scale, const float *hs, const float *u,
                        const float *attn, const float *dout, const float *dattn, float *dhs, float *du, int64_t ldu,
                        float *dc, int64_t ldc)
{
    if (sa_check("cn_spatial_attn_bwd: H in {64, 128, 256}, 1 <= N <= 64, non-null operands, hs / u / dout / "
                 "dhs / du 16-byte aligned, ldu >= H and a multiple of 4, ldc >= 1", R, N, H, {hs, u, dout, dhs, du},
                 {attn, dc}) || ldu < H || (ldu & 3) || ldc < 1)
        return cn_set_error(CN_EINVAL, "cn_spatial_attn_bwd: bad shape, stride or operand");
    const unsigned grid = grid_for(R, H);
    (void)hipGetLastError();   // a stale error of an earlier call (any library) is not this launch's
#define CN_SA_BWD(HQ, NR) \
    hipLaunchKernelGGL((cn_spatial_attn_bwd_kernel<HQ, NR>), dim3(grid), dim3(256), 0, (hipStream_t)stream, R, N, scale, hs, u, attn, dout, dattn, dhs, du, ldu, dc, ldc)
    if (N <= 10) {
        if (H == 256) CN_SA_BWD(64, 10);
        else if (H == 128) CN_SA_BWD(32, 10);
        else CN_SA_BWD(16, 10);
    } else {
        if (H == 256) CN_SA_BWD(64, 16);
        else if (H == 128) CN_SA_BWD(32, 16);
        else CN_SA_BWD(16, 16);
    }
#undef CN_SA_BWD
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? CN_OK : cn_set_error(CN_EHIP, hipGetErrorString(e));
}

}  // extern "C"
