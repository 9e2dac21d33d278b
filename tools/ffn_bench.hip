// Standalone timing of the 64-row fused FFN kernel (k_ffn.hip ffn_fused_kernel, OP mode as the fast encoder launches
// it) and its diagnostic variants on random data: VAR 0 the kernel, 1 no weight DMA (stale ring), 2 no MFMAs, 3 every
// tile streams ring tiles 0..3 of the layer (the weight stream L2-hot), 4 prologue + epilogue only, 5 VAR 1 without
// the per-tile barriers; then MODE 4 (the next layer's QKV projection as phase 3). HIP events, one process.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ffn_bench.hip -o tools/ffn_bench && ./tools/ffn_bench [M ...]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../funasr_amd/csrc/k_ffn.hip"

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

template <int VAR, int MODE>
float run(int M, int reps, const float* X, const float* g, const float* be, const bf16* Wp, const float* b1,
          const float* b2, float* Xo, const float* gn, const float* bn, bf16* Xn, const bf16* O, const bf16* Fr,
          const float* bo, const float* c1) {
    auto k = ffn_fused_kernel<VAR, MODE, 8, true, 3>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(k, dim3((M + BM - 1) / BM), dim3(512), LDS_BYTES, 0, X, M, g, be, 1e-12f, Wp, b1, b2, Xo, gn,
                           bn, Xn, O, Fr, bo, c1);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k, dim3((M + BM - 1) / BM), dim3(512), LDS_BYTES, 0, X, M, g, be, 1e-12f, Wp, b1, b2, Xo, gn,
                           bn, Xn, O, Fr, bo, c1);
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
    const long long nx = (long long)Mmax * 512, nw = (long long)(OP_TILES + NTILE + QK_TILES) * TILE / 2;
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
                *bo = vecs + 12288;
    for (int M : Ms) {
        const double fl = 2.0 * M * (2.0 * 512 * 2048 + 512.0 * 512);
        const int reps = 20;
        for (int round = 0; round < 2; ++round) {
            const float t0 = run<0, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t1 = run<1, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t2 = run<2, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t3 = run<3, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t4 = run<4, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t5 = run<5, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            printf("M=%6d OP: kernel %.1f us (%.0f TF/s) | no DMA %.1f | no MFMA %.1f | L2-hot W %.1f | pro/epi %.1f | "
                   "no DMA/bar %.1f\n", M, t0, fl / t0 / 1e6, t1, t2, t3, t4, t5);
            const float t6 = run<6, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            const float t7 = run<7, 1>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, nullptr);
            printf("M=%6d OP anatomy: O load + x1 loads + LN2 %.1f | + phase 0 %.1f | + epilogue (= pro/epi) %.1f\n", M, t7,
                   t6, t4);
            const float q0 = run<0, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, vecs + 14336);
            const float q1 = run<1, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, vecs + 14336);
            const float q2 = run<2, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, vecs + 14336);
            const float q3 = run<3, 4>(M, reps, X, g, be, Wp, b1, b2, Xo, gn, bn, Xn, O, Fr, bo, vecs + 14336);
            const double flq = fl + 2.0 * M * 512.0 * 1536;
            printf("M=%6d OP+QKV: kernel %.1f us (%.0f TF/s; +%.1f us over OP) | no DMA %.1f | no MFMA %.1f | L2-hot W %.1f\n",
                   M, q0, flq / q0 / 1e6, q0 - t0, q1, q2, q3);
        }
    }
    return 0;
}
