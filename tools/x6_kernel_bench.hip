// The EXACT-mode x6 GEMM (split-bf16: K' = 6 K over the segments of three A planes and three W planes) against the
// plain bf16 GEMM of the same K' on the same 256-tile kernel, calling the library's launcher directly (links
// libpfm_hip.so): isolates what the segment addressing costs. f32 output, C15 (the x6 default) and C17.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/x6_kernel_bench.hip -L funasr_amd/_lib -lpfm_hip \
//     -Wl,-rpath,'$ORIGIN/../funasr_amd/_lib' -o tools/x6_kernel_bench
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../funasr_amd/csrc/pfm_common.h"

hipError_t pfm_gemm_bf16_256(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                             const GemmEpi& epi, hipStream_t st);

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill(unsigned short* p, long long n, unsigned seed) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (unsigned short)(0x3c00u | (x & 0x807fu));
}

static float timeit(const std::vector<int>& cfgs, int cfg, const void* A, RowMap am, const void* W, long long ldw, int M,
                    int N, int K, const GemmEpi& e) {
    char buf[16];
    snprintf(buf, sizeof buf, "%d", cfg);
    setenv("PFM_GEMM_CFG", buf, 1);
    for (int i = 0; i < 3; ++i) CK(pfm_gemm_bf16_256(A, am, W, ldw, M, N, K, e, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    const int reps = 10;
    for (int i = 0; i < reps; ++i) CK(pfm_gemm_bf16_256(A, am, W, ldw, M, N, K, e, 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

int main() {
    struct S { const char* name; int M, N, K; };
    const S shapes[] = {{"qkv", 16000, 1536, 512}, {"out", 16000, 512, 512}, {"ffn1", 16000, 2048, 512},
                        {"ffn2", 16000, 512, 2048}};
    const long long far = 200LL * 1000 * 1000;   // weight planes this many elements apart (the arena's spacing)
    unsigned short *A6, *W6, *A3, *Wp;
    float* C;
    CK(hipMalloc(&A6, 16000LL * 6 * 2048 * 2));
    CK(hipMalloc(&W6, 2048LL * 6 * 2048 * 2));
    CK(hipMalloc(&A3, 16000LL * 3 * 2048 * 2));
    CK(hipMalloc(&Wp, (2 * far + 2048LL * 2048) * 2));
    CK(hipMalloc(&C, 16000LL * 2048 * 4));
    hipLaunchKernelGGL(fill, dim3((16000LL * 6 * 2048 + 255) / 256), dim3(256), 0, 0, A6, 16000LL * 6 * 2048, 1u);
    hipLaunchKernelGGL(fill, dim3((2048LL * 6 * 2048 + 255) / 256), dim3(256), 0, 0, W6, 2048LL * 6 * 2048, 2u);
    hipLaunchKernelGGL(fill, dim3((16000LL * 3 * 2048 + 255) / 256), dim3(256), 0, 0, A3, 16000LL * 3 * 2048, 3u);
    for (int p = 0; p < 3; ++p)
        hipLaunchKernelGGL(fill, dim3((2048LL * 2048 + 255) / 256), dim3(256), 0, 0, Wp + p * far, 2048LL * 2048, 4u + p);
    CK(hipDeviceSynchronize());
    for (const S& s : shapes) {
        GemmEpi e{};
        e.alpha = 1.f;
        e.out = C;
        e.out_map = rowmap_plain(s.N);
        e.out_dtype = DT_F32;
        const double fl = 2.0 * s.M * s.N * 6.0 * s.K;
        for (int cfg : {15, 17}) {
            const float tp = timeit({}, cfg, A6, rowmap_plain(6LL * s.K), W6, 6LL * s.K, s.M, s.N, 6 * s.K, e);
            GemmEpi x = e;
            x.x6_k = s.K; x.x6_ws = far; x.x6_terms = 6;
            const float tx = timeit({}, cfg, A3, rowmap_plain(3LL * s.K), Wp, s.K, s.M, s.N, 6 * s.K, x);
            GemmEpi xn = x;
            xn.x6_ws = (long long)s.N * s.K;   // planes adjacent
            const float tn = timeit({}, cfg, A3, rowmap_plain(3LL * s.K), Wp, s.K, s.M, s.N, 6 * s.K, xn);
            printf("%-5s M=%d N=%d K'=%d C%d: plain %.1f us (%.0f TF) | x6 %.1f us (%.0f TF) | x6 adjacent planes %.1f us\n",
                   s.name, s.M, s.N, 6 * s.K, cfg, tp, fl / tp / 1e6, tx, fl / tx / 1e6, tn);
        }
    }
    return 0;
}
