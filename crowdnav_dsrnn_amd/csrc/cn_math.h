// cn_math.h — numerics shared by the HIP engine kernels (gfx950).
//
// The reference computes in numpy 2.2 (NEP 50 scalar promotion) and RVO2 (float32 C++, no FMA
// contraction). The engine is compiled with -ffp-contract=off and spells out every fused op that the
// reference itself fuses (numpy's OpenBLAS ddot: np.linalg.norm / np.dot of float64 2-vectors).
// Division and square roots use the correctly rounded forms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CN_PI 3.141592653589793

namespace cn {

// IEEE correctly rounded sqrt / division. NOTE: HIP's __fsqrt_rn maps to __ocml_native_sqrt_f32
// (approximate) unless OCML_BASIC_ROUNDED_OPERATIONS is defined, so the builtins are used: without
// !fpmath metadata the AMDGPU backend lowers llvm.sqrt.f32/f64 and fdiv to correctly rounded sequences.
__device__ __forceinline__ double dsqrt(double x) { return __builtin_sqrt(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ double ddiv(double a, double b) { return a / b; }
__device__ __forceinline__ float fdiv(float a, float b) { return a / b; }

// np.linalg.norm of a float64 2-vector: sqrt(fma(b, b, a*a))  (OpenBLAS ddot tail loop is fused)
__device__ __forceinline__ double np_norm2(double a, double b) { return dsqrt(__fma_rn(b, b, a * a)); }
// np.linalg.norm((a, b)) < md, exactly, without the square root except within ~2^-48 of the boundary:
// rn(sqrt(x)) < md  <=>  x < md^2 away from equality (numerics).
__device__ __forceinline__ bool norm_lt(double a, double b, double md)
{
    const double x = __fma_rn(b, b, a * a);
    if (md > 0) {
        const double t = md * md;
        if (x < t * (1.0 - 0x1p-48)) return true;
        if (x > t * (1.0 + 0x1p-48)) return false;
    }
    return dsqrt(x) < md;
}
// np.linalg.norm of a float32 2-vector: plain float32
__device__ __forceinline__ float np_norm2f(float a, float b) { return fsqrt(a * a + b * b); }
// np.dot of float64 2-vectors
__device__ __forceinline__ double np_dot2(double a0, double a1, double b0, double b1) { return __fma_rn(a1, b1, a0 * b0); }

__device__ __forceinline__ double np_mod(double a, double b)
{
    double m = fmod(a, b);
    if (m != 0.0) { if ((b < 0) != (m < 0)) m += b; }
    else m = copysign(0.0, b);
    return m;
}
__device__ __forceinline__ float np_modf(float a, float b)
{
    float m = fmodf(a, b);
    if (m != 0.0f) { if ((b < 0) != (m < 0)) m += b; }
    else m = copysignf(0.0f, b);
    return m;
}

// numpy 2.x float32 sin/cos (Cody-Waite + minimax polynomials with FMA): np.sin/np.cos on float32
// scalars in the reference use this, not libm; bit-exact replica (see oracle/cpu_ref.c).
__device__ inline float np_sincosf(float x, bool want_cos)
{
    const float max_cody = want_cos ? 71476.0625f : 117435.992f;
    if (!(fabsf(x) <= max_cody)) return want_cos ? cosf(x) : sinf(x);
    float q = x * 0x1.45f306p-1f;
    q = q + 0x1.800000p+23f;
    q = q - 0x1.800000p+23f;
    float r = __fmaf_rn(q, -0x1.921fb0p+00f, x);
    r = __fmaf_rn(q, -0x1.5110b4p-22f, r);
    r = __fmaf_rn(q, -0x1.846988p-48f, r);
    const float r2 = r * r;
    float c = __fmaf_rn(0x1.98e616p-16f, r2, -0x1.6c06dcp-10f);
    c = __fmaf_rn(c, r2, 0x1.55553cp-05f);
    c = __fmaf_rn(c, r2, -0x1.000000p-01f);
    c = __fmaf_rn(c, r2, 0x1.000000p+00f);
    float s = __fmaf_rn(0x1.7d3bbcp-19f, r2, -0x1.a06bbap-13f);
    s = __fmaf_rn(s, r2, 0x1.11119ap-07f);
    s = __fmaf_rn(s, r2, -0x1.555556p-03f);
    s = __fmaf_rn(s, r2, 0.0f);
    s = __fmaf_rn(s, r, r);
    const int iq = (int)q + (want_cos ? 1 : 0);
    float out = (iq & 1) == 0 ? s : c;
    if ((iq & 2) == 2) out = 0.0f - out;
    return out;
}
__device__ __forceinline__ float np_sinf(float x) { return np_sincosf(x, false); }
__device__ __forceinline__ float np_cosf(float x) { return np_sincosf(x, true); }
__device__ __forceinline__ float np_clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// ---------------------------------------------------------------------------------------------
// numpy legacy MT19937 (mt19937_seed / mt19937_gen / mt19937_next / mt19937_next_double)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mt_temper(uint32_t y)
{
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c)
{
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11; the Random123 constants) for CN_RNG_PHILOX. Word q of an episode's
// stream is word (q & 3) of philox(counter = (q >> 2, 0, 0, 0), key = (seed, CN_PHILOX_K1)); a double is
// two consecutive words converted like numpy's random_sample ((a >> 5) * 2^26 + (b >> 6)) / 2^53.
// Draws always start at even word positions, so both words of a double come from one counter block.
// ---------------------------------------------------------------------------------------------
#define CN_PHILOX_K1 0x43726f77u
__device__ __forceinline__ uint4 philox4x32_10(uint32_t c0, uint32_t k0, uint32_t k1)
{
    uint32_t x0 = c0, x1 = 0, x2 = 0, x3 = 0;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * x0, hi0 = __umulhi(0xD2511F53u, x0);
        const uint32_t lo1 = 0xCD9E8D57u * x2, hi1 = __umulhi(0xCD9E8D57u, x2);
        x0 = hi1 ^ x1 ^ k0; x1 = lo1; x2 = hi0 ^ x3 ^ k1; x3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(x0, x1, x2, x3);
}
__device__ __forceinline__ double philox_dbl(uint32_t key, int q)
{
    const uint4 w = philox4x32_10((uint32_t)q >> 2, key, CN_PHILOX_K1);
    const uint32_t a = (q & 2) ? w.z : w.x, b = (q & 2) ? w.w : w.y;
    return ((int32_t)(a >> 5) * 67108864.0 + (int32_t)(b >> 6)) / 9007199254740992.0;
}

}  // namespace cn
