// Standalone timing of the 128-row fused FFN kernel (k_ffn2.hip) and its diagnostic variants (VAR 1: no weight
// DMA, 2: no MFMA, 3: no DMA and no barriers, 4: L2-hot weights, 5: prologue / epilogue only, 6: burst DMA) on random data, HIP events, one process.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/ffn2_bench.hip -o tools/ffn2_bench
//   ./tools/ffn2_bench [M ...]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "../funasr_amd/csrc/k_ffn2.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill_bf16(bf16* p, long long n, unsigned seed, float scale) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((x & 0xffff) / 65536.f - 0.5f) * scale);
}
__global__ void fill_f32(float* p, long long n, unsigned seed, float scale, float off) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2246822519u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = off + ((x & 0xffff) / 65536.f - 0.5f) * scale;
}

template <int MODE, int VAR>
float run(int M, int reps, const float* X, const float* g, const float* be, const bf16* Wp, const float* b1, const float* b2,
          float* Xo, const float* gn, const float* bn, bf16* Xn, const bf16* O, const bf16* Fr, const float* bo,
          const float* c1) {
    CK(hipFuncSetAttribute((const void*)ffn2_kernel<MODE, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((ffn2_kernel<MODE, VAR>), dim3((M + BM - 1) / BM), dim3(256), LDS_BYTES, 0, X, M, g, be, 1e-12f,
                           Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((ffn2_kernel<MODE, VAR>), dim3((M + BM - 1) / BM), dim3(256), LDS_BYTES, 0, X, M, g, be, 1e-12f,
                           Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
    std::vector<int> Ms;
    for (int i = 1; i < argc; ++i) Ms.push_back(atoi(argv[i]));
    if (Ms.empty()) Ms = {16000, 32000};
    const int Mmax = 32768;
    const long long nx = (long long)Mmax * 512, nw = 2 * 262144 + 2097152 + 4 * 262144;   // MODE 6's stream
    float *X, *Xo, *vecs;
    bf16 *Wp, *O, *Fr, *Xn;
    CK(hipMalloc(&X, nx * 4));
    CK(hipMalloc(&Xo, nx * 4));
    CK(hipMalloc(&O, nx * 2));
    CK(hipMalloc(&Fr, nx * 2));
    CK(hipMalloc(&Xn, nx * 2 * 3));
    CK(hipMalloc(&Wp, nw * 2));
    CK(hipMalloc(&vecs, 16 * 2048 * 4));
    hipLaunchKernelGGL(fill_f32, dim3((nx + 255) / 256), dim3(256), 0, 0, X, nx, 1u, 4.f, 0.f);
    hipLaunchKernelGGL(fill_bf16, dim3((nx + 255) / 256), dim3(256), 0, 0, O, nx, 2u, 2.f);
    hipLaunchKernelGGL(fill_bf16, dim3((nx + 255) / 256), dim3(256), 0, 0, Fr, nx, 3u, 1.f);
    hipLaunchKernelGGL(fill_bf16, dim3((nw + 255) / 256), dim3(256), 0, 0, Wp, nw, 4u, 0.09f);
    hipLaunchKernelGGL(fill_f32, dim3(16 * 2048 / 256), dim3(256), 0, 0, vecs, 16LL * 2048, 5u, 0.2f, 0.f);
    CK(hipDeviceSynchronize());
    const float *g = vecs, *be = vecs + 2048, *b1 = vecs + 4096, *b2 = vecs + 6144, *gn = vecs + 8192, *bn = vecs + 10240,
                *bo = vecs + 12288, *c1 = vecs + 14336;
    // PMC passes: FFN2_ONLY=1 the OP kernel alone (MODE 1), FFN2_ONLY=4 the OP + next-QKV kernel (MODE 4, the default)
    // FFN2_ANAT=1: the anatomy of the default encoder launch (MODE 5, PFM_FAST_XW 7) and of MODE 4 / 6 beside it
    if (getenv("FFN2_ANAT") && atoi(getenv("FFN2_ANAT")) == 2) {   // the stream's VALU / wait-state diagnostics
        for (int M : Ms) {
            run<4, 0>(M, 8000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);   // ~2 s: sustained clock
            for (int round = 0; round < 2; ++round) {
                float t0 = run<4, 0>(M, 2000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                float t10 = run<4, 10>(M, 2000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                float t11 = run<4, 11>(M, 2000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                float t3 = run<4, 3>(M, 2000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                printf("M=%d MODE4 round %d: full %.1f  no-relu %.1f  no-nops %.1f  no-DMA/bar %.1f us\n", M, round, t0,
                       t10, t11, t3);
            }
        }
        return 0;
    }
    if (getenv("FFN2_ANAT")) {
        for (int M : Ms) {
            const double fl = 2.0 * M * 512.0 * (512 + 2048 + 2048 + 1536);
            const int reps = 20;
            float t;
            t = run<4, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE4 full       %8.1f us  %7.1f TF/s\n", M, t, fl / t / 1e6);
            t = run<6, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE6 full       %8.1f us  %7.1f TF/s (algorithmic)\n", M, t, fl / t / 1e6);
            t = run<5, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 full       %8.1f us  %7.1f TF/s (algorithmic)\n", M, t, fl / t / 1e6);
            t = run<5, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 no DMA     %8.1f us\n", M, t);
            t = run<5, 2>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 no MFMA    %8.1f us\n", M, t);
            t = run<5, 3>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 no DMA/bar %8.1f us\n", M, t);
            t = run<5, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 L2-hot W   %8.1f us\n", M, t);
            t = run<5, 5>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 pro/epi    %8.1f us\n", M, t);
            t = run<5, 7>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 no qkv st  %8.1f us\n", M, t);
            t = run<5, 8>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 no x2 st   %8.1f us\n", M, t);
            t = run<5, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE5 full again %8.1f us\n", M, t);
            t = run<4, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d MODE4 full again %8.1f us\n", M, t);
        }
        return 0;
    }
    // FFN2_TS=1: per-phase timeline of MODE 5 and MODE 4 (VAR 9: wave 0's s_memrealtime stamps, 100 MHz)
    if (getenv("FFN2_TS")) {
        const char* names[13] = {"vectors + prologue loads", "phase 0 (out-proj) stream", "transition (x, F loads, LN2)",
                                 "FFN stream", "x2 store issue", "LN1_next", "QKV pass 0 stream", "pass 0 stores",
                                 "QKV pass 1 stream", "pass 1 stores", "QKV pass 2 stream (+ v plane)",
                                 "pass 2 stores issue", "stores retire"};
        for (int M : Ms) {
            const int nb = (M + BM - 1) / BM;
            std::vector<unsigned long long> ts(16 * nb);
            for (int mode = 5; mode >= 3; --mode) {   // 3 here = MODE 4 without the relu VALU (VAR 12)
                // ~2 s of back-to-back launches first: the clock the chip holds under sustained load (DVFS)
                const float hot = mode == 5 ? run<5, 0>(M, 8000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1)
                                  : mode == 4 ? run<4, 0>(M, 8000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1)
                                              : run<4, 10>(M, 8000, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                printf("M=%d MODE%d sustained (8000 launches): %.1f us per launch\n", M, mode, hot);
                float t = mode == 5 ? run<5, 9>(M, 5, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1)
                        : mode == 4 ? run<4, 9>(M, 5, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1)
                                    : run<4, 12>(M, 5, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
                CK(hipMemcpy(ts.data(), Xo + (long long)M * 512, ts.size() * 8, hipMemcpyDeviceToHost));
                unsigned long long t0 = ~0ull, t1 = 0, e0 = ~0ull;
                for (int b = 0; b < nb; ++b) {
                    t0 = std::min(t0, ts[16 * b]);
                    t1 = std::max(t1, ts[16 * b + 13]);
                    e0 = std::min(e0, ts[16 * b + 13]);
                }
                printf("M=%d MODE%d launch %.1f us (events); stamps: first start -> last end %.1f us, start skew %.1f us, "
                       "end skew %.1f us\n", M, mode, t, (t1 - t0) / 100.0, 0.0, (t1 - e0) / 100.0);
                std::vector<double> clk;
                for (int b = 0; b < nb; ++b)
                    clk.push_back((double)(ts[16 * b + 15] - ts[16 * b + 14]) / (double)(ts[16 * b + 4] - ts[16 * b + 3]) * 0.1);
                std::sort(clk.begin(), clk.end());
                printf("  in-kernel shader clock over the FFN stream: median %.3f GHz (min %.3f, max %.3f)\n",
                       clk[clk.size() / 2], clk.front(), clk.back());
                double sk = 0;
                for (int b = 0; b < nb; ++b) sk = std::max(sk, (ts[16 * b] - t0) / 100.0);
                printf("  start skew (max over workgroups) %.1f us\n", sk);
                for (int i = 0; i < 13; ++i) {
                    double mn = 1e30, mx = 0, sum = 0;
                    for (int b = 0; b < nb; ++b) {
                        const double d = (ts[16 * b + i + 1] - ts[16 * b + i]) / 100.0;
                        mn = std::min(mn, d); mx = std::max(mx, d); sum += d;
                    }
                    printf("  %-32s mean %7.2f us  min %7.2f  max %7.2f\n", names[i], sum / nb, mn, mx);
                }
            }
        }
        return 0;
    }
    const char* only_env = getenv("FFN2_ONLY");
    const bool only = only_env != nullptr, only4 = only && atoi(only_env) == 4;
    for (int M : Ms) {
        const double fl1 = 2.0 * M * (2.0 * 512 * 2048 + 512.0 * 512), fl0 = 2.0 * M * 2.0 * 512 * 2048;
        const int reps = 20;
        float t;
        if (only4) {
            t = run<4, 0>(M, 5, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d OP+QKV full      %8.1f us  %7.1f TF/s\n", M, t, (fl1 + 2.0 * M * 1536 * 512) / t / 1e6);
            continue;
        }
        if (only) {
            t = run<1, 0>(M, 5, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
            printf("M=%6d OP   full        %8.1f us  %7.1f TF/s\n", M, t, fl1 / t / 1e6);
            continue;
        }
        t = run<1, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   full        %8.1f us  %7.1f TF/s\n", M, t, fl1 / t / 1e6);
        t = run<1, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   no DMA      %8.1f us\n", M, t);
        t = run<1, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   L2-hot W    %8.1f us\n", M, t);
        t = run<1, 2>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   no MFMA     %8.1f us\n", M, t);
        t = run<1, 3>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   no DMA/bar  %8.1f us  %7.1f TF/s\n", M, t, fl1 / t / 1e6);
        t = run<1, 6>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   burst DMA   %8.1f us\n", M, t);
        t = run<1, 5>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP   pro/epi     %8.1f us\n", M, t);
        t = run<4, 0>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d OP+QKV full      %8.1f us  %7.1f TF/s\n", M, t, (fl1 + 2.0 * M * 1536 * 512) / t / 1e6);
        t = run<0, 0>(M, reps, X, g, be, Wp + 262144, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, c1);
        printf("M=%6d FFN  full        %8.1f us  %7.1f TF/s\n", M, t, fl0 / t / 1e6);
    }
    return 0;
}
