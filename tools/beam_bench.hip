// Standalone timing of the beam-search kernel (k_beam.hip) on random log-probs with a per-phase wall-clock breakdown
// (built with -DBEAM_PROF):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DBEAM_PROF -I include tools/beam_bench.hip -o tools/beam_bench
//   ./tools/beam_bench [B L T beam]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../funasr_amd/csrc/k_beam.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill_f32(float* p, long long n, unsigned seed, float scale) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2246822519u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15; x *= 0x27d4eb2du; x ^= x >> 16;
    p[i] = ((x & 0xffffff) / 16777216.f - 0.5f) * scale;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 64, L = argc > 2 ? atoi(argv[2]) : 230, T = argc > 3 ? atoi(argv[3]) : 500;
    const int K = argc > 4 ? atoi(argv[4]) : 10, V = 8404, P = (int)(1.5 * K) < V ? (int)(1.5 * K) : V, nbest = 1;
    float *am, *x, *fs, *sc;
    int *lens, *ntok, *is, *tok, *ol;
    CK(hipMalloc(&am, (size_t)B * L * V * 4));
    CK(hipMalloc(&x, (size_t)B * T * V * 4));
    hipLaunchKernelGGL(fill_f32, dim3(((long long)B * L * V + 255) / 256), dim3(256), 0, 0, am, (long long)B * L * V, 1u, 6.f);
    hipLaunchKernelGGL(fill_f32, dim3(((long long)B * T * V + 255) / 256), dim3(256), 0, 0, x, (long long)B * T * V, 2u, 6.f);
    CK(pfm_logsoftmax_rows(am, (long long)B * L, V, V, 0));
    CK(pfm_logsoftmax_rows(x, (long long)B * T, V, V, 0));
    std::vector<int> hl(B, T), hn(B, L);
    CK(hipMalloc(&lens, B * 4));
    CK(hipMalloc(&ntok, B * 4));
    CK(hipMemcpy(lens, hl.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(ntok, hn.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&fs, (size_t)B * pfm_ctc_beam_fscratch(K, P, T, L, V) * 4));
    CK(hipMalloc(&is, (size_t)B * pfm_ctc_beam_iscratch(K, nbest, L, P, V) * 4));
    CK(hipMalloc(&tok, (size_t)B * nbest * (L + 1) * 4));
    CK(hipMalloc(&ol, (size_t)B * nbest * 4));
    CK(hipMalloc(&sc, (size_t)B * nbest * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&]() {
        CK(pfm_ctc_beam(am, L, x, T, lens, ntok, B, V, K, P, nbest, 0.3f, 0.f, 0, 0, 1, 2, 0, fs, is, tok, L + 1, ol, sc, nullptr, 0));
    };
    run();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    run();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("B=%d L=%d T=%d beam=%d: %.2f ms (%.1f us per position)\n", B, L, T, K, ms, ms * 1e3 / L);
#ifdef BEAM_PROF
    int khz = 100000;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    std::vector<unsigned long long> h((size_t)1024 * 8);
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(beam_prof), h.size() * 8));
    const char* nm[6] = {"pre-beam", "gather+rsum", "prefix recurrences", "per-hyp top-k", "sort-prune", "post-process"};
    double tot = 0;
    for (int q = 0; q < 6; ++q) {
        double s = 0;
        for (int b = 0; b < B; ++b) s += h[(size_t)b * 8 + q];
        s /= B;
        tot += s;
        printf("  %-20s %8.1f us per position\n", nm[q], s / (khz / 1000.0) / L);
    }
    printf("  %-20s %8.1f us per position (wall clock %d kHz)\n", "total", tot / (khz / 1000.0) / L, khz);
#endif
    std::vector<float> hs(B);
    std::vector<int> hl2(B);
    CK(hipMemcpy(hs.data(), sc, B * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hl2.data(), ol, B * 4, hipMemcpyDeviceToHost));
    double ssum = 0;
    long long lsum = 0;
    for (int b = 0; b < B; ++b) { ssum += hs[b]; lsum += hl2[b]; }
    printf("  scores sum %.6f (first %.7g), lengths sum %lld\n", ssum, hs[0], lsum);
    int h0[4];
    CK(hipMemcpy(h0, ol, 4 * 4 < B * 4 ? 16 : B * 4, hipMemcpyDeviceToHost));
    printf("  n-best lengths of utterances 0..3: %d %d %d %d\n", h0[0], B > 1 ? h0[1] : 0, B > 2 ? h0[2] : 0, B > 3 ? h0[3] : 0);
    return 0;
}
