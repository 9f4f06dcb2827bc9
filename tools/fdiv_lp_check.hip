// Check of cn_engine.hip's fdiv_lp (the linear programs' short IEEE division) and of fsqrt_lp (the same
// idea for sqrt: exact, but C2-neutral, not kept) against the compiler's correctly rounded f32 division
// and sqrt, bit for bit. Division, over random operands with both signs:
//   sweep 1: numerators with random exponents in [2^-40, 2^40] and zeros, divisors |b| in (RVO_EPSILON, 2^40];
//   sweep 2 (the whole numerator range): numerators of EVERY exponent, 2^-149 (denormals, exponent field 0)
//            to 2^127, and zeros; divisors in the linear programs' domain |b| in (RVO_EPSILON, 2]
//            (determinants of unit vectors). Sweep 2 also counts the unguarded form (no tiny-numerator
//            branch) to show where the guard matters.
// sqrt over all 2^32 inputs (NaNs compared as NaN).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/bin/fdiv_lp_check tools/fdiv_lp_check.hip
//   tools/bin/fdiv_lp_check [billions]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__device__ __forceinline__ float fdiv_lp_unguarded(float a, float b)
{
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
    const float q0 = a * y1;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y1, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), y1, q1);
}

// as in cn_engine.hip
__device__ __forceinline__ float fdiv_lp(float a, float b)
{
    if (__builtin_expect(__builtin_fabsf(a) < 0x1p-96f, 0)) return a / b;
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
    const float q0 = a * y1;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y1, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), y1, q1);
}

__device__ __forceinline__ float fsqrt_lp(float x)
{
    if (__builtin_fabsf(x) < 0x1p-96f && x != 0.0f) return __builtin_sqrtf(x);   // tiny / denormal x: full sequence
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    float r = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
    r = __builtin_fmaf(-su, s, x) > 0.0f ? su : r;
    return r;
}

__global__ void check_sqrt(uint64_t base, unsigned long long *bad, float *ex)
{
    const uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i > 0xffffffffull) return;
    const float x = __uint_as_float((uint32_t)i);
    const float q = __builtin_sqrtf(x), p = fsqrt_lp(x);
    const bool same = (q != q) ? (p != p) : (__float_as_uint(q) == __float_as_uint(p));
    if (!same) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 4) { ex[3 * k] = x; ex[3 * k + 1] = q; ex[3 * k + 2] = p; }
    }
}

__device__ __forceinline__ uint32_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

// random float with unbiased exponent in [emin, emax]; emin = -127 stands for the denormals (field 0)
__device__ __forceinline__ float rnd_float(uint64_t k, int emin, int emax)
{
    const uint32_t r0 = mix(k), r1 = mix(k ^ 0x9e3779b97f4a7c15ull);
    const int e = emin + (int)(r1 % (uint32_t)(emax - emin + 1));
    const uint32_t bits = ((uint32_t)(e + 127) << 23) | (r0 & 0x7fffffu) | ((r1 >> 31) << 31);
    return __uint_as_float(bits);
}

// sweep 2: numerator exponents -127 (denormal) .. 127 uniformly, divisors (RVO_EPSILON, 2]
__global__ void check_full(uint64_t base, uint64_t n, unsigned long long *bad, unsigned long long *bad_ug, float *ex)
{
    for (uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < base + n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        float a = rnd_float(2 * i, -127, 127);
        if ((mix(11 * i) & 1023u) == 0) a = 0.0f;
        float b = rnd_float(2 * i + 1, -17, 1);
        if (fabsf(b) <= 0.00001f || fabsf(b) > 2.0f) continue;
        const float q = a / b;
        if (q != q || __builtin_isinf(q)) continue;   // a / b overflows: outside the LP's finite quotients
        if (__float_as_uint(q) != __float_as_uint(fdiv_lp_unguarded(a, b))) atomicAdd(bad_ug, 1ull);
        const float p = fdiv_lp(a, b);
        if (__float_as_uint(q) != __float_as_uint(p)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 4) { ex[3 * k] = a; ex[3 * k + 1] = b; ex[3 * k + 2] = p; }
        }
    }
}

__global__ void check(uint64_t base, uint64_t n, unsigned long long *bad, float *ex)
{
    for (uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < base + n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        float a = rnd_float(2 * i, -40, 40);
        if ((mix(7 * i) & 1023u) == 0) a = 0.0f;
        float b = rnd_float(2 * i + 1, -16, 40);
        if (fabsf(b) <= 0.00001f) continue;
        const float q = a / b, p = fdiv_lp(a, b);
        if (__float_as_uint(q) != __float_as_uint(p)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 4) { ex[3 * k] = a; ex[3 * k + 1] = b; ex[3 * k + 2] = p; }
        }
    }
}

int main(int argc, char **argv)
{
    const double bn = argc > 1 ? atof(argv[1]) : 4.0;
    const uint64_t total = (uint64_t)(bn * 1e9), chunk = 1ull << 30;
    unsigned long long *bad;
    float *ex;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&ex, 48) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    for (uint64_t b0 = 0; b0 < total; b0 += chunk) {
        hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, b0, total - b0 < chunk ? total - b0 : chunk, bad, ex);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
    }
    unsigned long long h = 0;
    float e[12] = {0};
    (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(e, ex, 48, hipMemcpyDeviceToHost);
    printf("fdiv_lp vs IEEE division, sweep 1 (|a| in [2^-40, 2^40]): %llu mismatches in %.2e pairs\n", h, (double)total);
    for (int k = 0; k < 4 && k < (int)h; ++k) printf("  a=%a b=%a fdiv_lp=%a ieee=%a\n", e[3 * k], e[3 * k + 1], e[3 * k + 2], e[3 * k] / e[3 * k + 1]);
    unsigned long long *bad_ug;
    if (hipMalloc(&bad_ug, 8) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(bad_ug, 0, 8);
    for (uint64_t b0 = 0; b0 < total; b0 += chunk) {
        hipLaunchKernelGGL(check_full, dim3(16384), dim3(256), 0, 0, b0, total - b0 < chunk ? total - b0 : chunk, bad, bad_ug, ex);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
    }
    unsigned long long h2 = 0, hu = 0;
    (void)hipMemcpy(&h2, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&hu, bad_ug, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(e, ex, 48, hipMemcpyDeviceToHost);
    printf("fdiv_lp vs IEEE division, sweep 2 (every numerator exponent incl. denormals, |b| in (1e-5, 2]): "
           "%llu mismatches in %.2e pairs (unguarded form: %llu)\n", h2, (double)total, hu);
    for (int k = 0; k < 4 && k < (int)h2; ++k) printf("  a=%a b=%a fdiv_lp=%a ieee=%a\n", e[3 * k], e[3 * k + 1], e[3 * k + 2], e[3 * k] / e[3 * k + 1]);
    h += h2;
    unsigned long long hs = 0;
    (void)hipMemset(bad, 0, 8);
    for (uint64_t b0 = 0; b0 < (1ull << 32); b0 += 256ull * 65536ull) {
        hipLaunchKernelGGL(check_sqrt, dim3(65536), dim3(256), 0, 0, b0, bad, ex);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
    }
    (void)hipMemcpy(&hs, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(e, ex, 48, hipMemcpyDeviceToHost);
    printf("fsqrt_lp vs IEEE sqrt: %llu mismatches over all 2^32 inputs\n", hs);
    for (int k = 0; k < 4 && k < (int)hs; ++k) printf("  x=%a ieee=%a fsqrt_lp=%a\n", e[3 * k], e[3 * k + 1], e[3 * k + 2]);
    return (h || hs) ? 1 : 0;
}
