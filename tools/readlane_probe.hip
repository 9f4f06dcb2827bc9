// Minimal reproduction attempt for the v_readlane broadcast failure noted in DESIGN.md §4 (VERDICT r01
// item 9). The goal pass of cn_engine.hip walks humans h in index order (a wave-uniform loop), and for a
// changing human evaluates J tries at once as (try t, agent a) lanes: the candidate (gx, gy) is computed
// only on valid lanes (t < J), a ballot of the per-agent hits selects the first try without a hit (win,
// a loop-carried wave-uniform value), and the winning try's goal is broadcast to the wave. Here the same
// structure runs three broadcasts of the winner's f64 goal side by side:
//   (a) __builtin_amdgcn_readlane on the two 32-bit halves (lane = win * NA), the original form;
//   (b) __shfl (ds_bpermute);
//   (c) an LDS store by the winning lane + wave barrier + load (the form cn_engine.hip uses).
// Every lane checks (a) and (b) against (c); mismatches are counted per wave.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o /tmp/readlane_probe tools/readlane_probe.hip
//   /tmp/readlane_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ double hash01(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return (x >> 8) * (1.0 / 16777216.0);
}

__global__ void __launch_bounds__(64) probe(int NA, int nh, int *mism_a, int *mism_b, double *sum)
{
    __shared__ double bx, by;
    const int lane = threadIdx.x;
    const uint32_t seed = blockIdx.x * 7919u;
    double acc = 0.0;
    int bad_a = 0, bad_b = 0;
    for (int h = 0; h < nh; ++h) {            // walk over the humans (wave-uniform)
        const int J = 64 / NA;
        int p = 0;
        for (int pass = 0; pass < 40; ++pass) {   // rejection passes
            const int t = lane / NA, a = lane - t * NA;
            const bool valid = t < J;
            double gx = 0.0, gy = 0.0;
            bool hit = true;
            if (valid) {
                const uint32_t q = seed + (uint32_t)(h * 100000 + (p + t) * 17);
                gx = 8.0 * hash01(q) - 4.0;
                gy = 8.0 * hash01(q + 1) - 4.0;
                const double ax = 8.0 * hash01(seed + 977u * (uint32_t)a + (uint32_t)h) - 4.0;
                const double ay = 8.0 * hash01(seed + 991u * (uint32_t)a + (uint32_t)h) - 4.0;
                hit = (gx - ax) * (gx - ax) + (gy - ay) * (gy - ay) < 0.9 * 0.9 * (1 + (pass < 3));
            }
            const uint64_t badm = __ballot(hit);
            const uint64_t gm = (1ull << NA) - 1ull;
            int win = -1;
            for (int k = 0; k < J; ++k)
                if (((badm >> (k * NA)) & gm) == 0) { win = k; break; }
            if (win < 0) { p += J; continue; }
            const int src = win * NA;
            // (a) readlane of both halves
            const uint64_t bits = (uint64_t)__double_as_longlong(gx);
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)bits, src);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(bits >> 32), src);
            const double ra = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
            // (b) ds_bpermute
            const double rb = __shfl(gx, src);
            // (c) LDS store by the winner
            if (lane == src) { bx = gx; by = gy; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double rc = bx;
            bad_a += ra != rc;
            bad_b += rb != rc;
            acc += rc + by;
            __builtin_amdgcn_wave_barrier();
            break;
        }
    }
    atomicAdd(mism_a, bad_a);
    atomicAdd(mism_b, bad_b);
    if (lane == 0) sum[blockIdx.x] = acc;
}

int main()
{
    int *ma, *mb;
    double *s;
    const int blocks = 4096;
    hipMalloc(&ma, 4); hipMalloc(&mb, 4); hipMalloc(&s, blocks * 8);
    int total_a = 0, total_b = 0;
    for (int NA = 2; NA <= 32; NA += 3) {
        hipMemset(ma, 0, 4); hipMemset(mb, 0, 4);
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, NA, 10, ma, mb, s);
        int ha = -1, hb = -1;
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel error\n"); return 2; }
        hipMemcpy(&ha, ma, 4, hipMemcpyDeviceToHost);
        hipMemcpy(&hb, mb, 4, hipMemcpyDeviceToHost);
        printf("NA=%2d readlane mismatches %d, shfl mismatches %d (lane-checks %d)\n", NA, ha, hb, blocks * 64 * 10);
        total_a += ha; total_b += hb;
    }
    printf("TOTAL readlane %d shfl %d\n", total_a, total_b);
    hipFree(ma); hipFree(mb); hipFree(s);
    return 0;
}
