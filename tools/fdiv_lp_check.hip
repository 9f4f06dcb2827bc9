// Check of cn_engine.hip's fdiv_lp (the linear programs' short IEEE division) and of fsqrt_lp (the same
// idea for sqrt: exact, but C2-neutral, not kept) against the compiler's correctly rounded f32 division
// and sqrt, bit for bit: division over random
// operands (numerators with random exponents in [2^-40, 2^40] and zeros, divisors with |b| in
// (RVO_EPSILON, 2^40], both signs), sqrt over all 2^32 inputs (NaNs compared as NaN).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/bin/fdiv_lp_check tools/fdiv_lp_check.hip
//   tools/bin/fdiv_lp_check [billions]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__device__ __forceinline__ float fdiv_lp(float a, float b)
{
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

__device__ __forceinline__ float rnd_float(uint64_t k, int emin, int emax)
{
    const uint32_t r0 = mix(k), r1 = mix(k ^ 0x9e3779b97f4a7c15ull);
    const int e = emin + (int)(r1 % (uint32_t)(emax - emin + 1));
    const uint32_t bits = ((uint32_t)(e + 127) << 23) | (r0 & 0x7fffffu) | ((r1 >> 31) << 31);
    return __uint_as_float(bits);
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
    printf("fdiv_lp vs IEEE division: %llu mismatches in %.2e pairs\n", h, (double)total);
    for (int k = 0; k < 4 && k < (int)h; ++k) printf("  a=%a b=%a fdiv_lp=%a ieee=%a\n", e[3 * k], e[3 * k + 1], e[3 * k + 2], e[3 * k] / e[3 * k + 1]);
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
