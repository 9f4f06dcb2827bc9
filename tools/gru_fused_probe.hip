// Diagnostic timing of cn_gru_fwd_fused variants (not product code): build with
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off [-DCN_GF_PROBE_NOEPI] tools/gru_fused_probe.hip -o <bin>
// and run <bin> B H reps: prints the average launch time (HIP events) of the fused step at B x H.
#include "../crowdnav_dsrnn_amd/csrc/cn_gru.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int cn_set_error(int code, const char *msg)
{
    fprintf(stderr, "error %d: %s\n", code, msg);
    return code;
}

int main(int argc, char **argv)
{
    const int64_t B = argc > 1 ? atoll(argv[1]) : 20480;
    const int H = argc > 2 ? atoi(argv[2]) : 256;
    const int reps = argc > 3 ? atoi(argv[3]) : 100;
    std::vector<float> h((size_t)B * 4 * H);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
    float *gi, *hm, *w, *b, *m, *ho, *hn, *sv;
    hipMalloc(&gi, B * 3 * H * 4);
    hipMalloc(&hm, B * H * 4);
    hipMalloc(&w, 3 * H * H * 4);
    hipMalloc(&b, 3 * H * 4);
    hipMalloc(&m, B * 4);
    hipMalloc(&ho, B * H * 4);
    hipMalloc(&hn, B * H * 4);
    hipMalloc(&sv, B * 4 * H * 4);
    hipMemcpy(gi, h.data(), B * 3 * H * 4, hipMemcpyHostToDevice);
    hipMemcpy(hm, h.data(), B * H * 4, hipMemcpyHostToDevice);
    hipMemcpy(w, h.data(), 3 * H * H * 4, hipMemcpyHostToDevice);
    hipMemcpy(b, h.data(), 3 * H * 4, hipMemcpyHostToDevice);
    hipMemcpy(m, h.data(), B * 4, hipMemcpyHostToDevice);
    hipStream_t st;
    hipStreamCreate(&st);
    for (int i = 0; i < 5; ++i) cn_gru_fwd_fused(st, B, H, gi, hm, w, b, m, ho, hn, sv, nullptr, 1, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    for (int i = 0; i < reps; ++i) cn_gru_fwd_fused(st, B, H, gi, hm, w, b, m, ho, hn, sv, nullptr, 1, 0);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("B=%lld H=%d avg %.2f us  %.1f TFLOP/s\n", (long long)B, H, us, 6.0 * B * H * H / us / 1e6);
    return 0;
}
