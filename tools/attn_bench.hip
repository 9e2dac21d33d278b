// Standalone timing of the bf16 encoder self-attention kernel (k_attn.hip attn_bf16_kernel<8, VAR>, fused
// FSMN epilogue on, as the fast encoder launches it) on random data: one utterance group (B = 32 x 500 x 500,
// 4 heads of 128) and the whole batch (B = 64). VAR: 0 product, 1 no K/V loads after tile 0, 2 no softmax,
// 3 no PV products, 4 no QK products, 5 no key loop. HIP events, one process.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/attn_bench.hip -o tools/attn_bench && ./tools/attn_bench
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "../funasr_amd/csrc/k_attn.hip"

hipError_t pfm_attention_small(int, const void*, RowMap, const void*, RowMap, const void*, RowMap, float*, void*,
                               long long, const int*, int, int, int, int, int, float, hipStream_t) {
    return hipErrorInvalidValue;
}
static PfmKnobs g_kn;
const PfmKnobs& pfm_knobs() { return g_kn; }

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void fill_bf16(bf16* p, long long n, unsigned seed, float scale) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((x & 0xffff) / 65536.f - 0.5f) * scale);
}
__global__ void fill_f32(float* p, long long n, unsigned seed, float scale) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2246822519u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((x & 0xffff) / 65536.f - 0.5f) * scale;
}

template <int VAR>
float run(const AttnArgs& a, int B, int T, int reps) {
    auto k = attn_bf16_kernel<8, VAR>;
    const int lds = LDS8_FS;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    dim3 grid((T + 255) / 256, 4, B), block(512);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, grid, block, lds, 0, a);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, grid, block, lds, 0, a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}

template <int VAR>
float run_x6(const AttnArgs& a, int B, int T, int reps) {
    auto k = attn_x6_kernel<VAR>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, X6_LDS));
    dim3 grid((T + 255) / 256, 4, B), block(512);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, grid, block, X6_LDS, 0, a);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, grid, block, X6_LDS, 0, a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}

// EXACT-mode attention (attn_x6_kernel: split-bf16 x6, f32 FSMN epilogue) as the exact encoder launches it, one group
void bench_x6(int reps) {
    const int T = 500, D = 512, B = 32;
    float *qkv, *fo, *fw;
    bf16* o3;
    int* lens;
    CK(hipMalloc(&qkv, (size_t)B * T * 3 * D * 4));
    CK(hipMalloc(&o3, (size_t)B * T * 3 * D * 2));
    CK(hipMalloc(&fo, (size_t)B * T * D * 4));
    CK(hipMalloc(&fw, 11 * D * 4));
    CK(hipMalloc(&lens, B * 4));
    const long long n = (long long)B * T * 3 * D;
    hipLaunchKernelGGL(fill_f32, dim3((n + 255) / 256), dim3(256), 0, 0, qkv, n, 7u, 4.f);
    hipLaunchKernelGGL(fill_f32, dim3((11 * D + 255) / 256), dim3(256), 0, 0, fw, 11LL * D, 2u, 0.5f);
    std::vector<int> hl(B, T);
    CK(hipMemcpy(lens, hl.data(), B * 4, hipMemcpyHostToDevice));
    AttnArgs a;
    a.q = qkv; a.qmap = rowmap_plain(3 * D); a.k = qkv + D; a.kmap = rowmap_plain(3 * D);
    a.v = qkv + 2 * D; a.vmap = rowmap_plain(3 * D); a.o = nullptr; a.ldo = 3 * D; a.o2 = o3; a.o2_dtype = DT_X3;
    a.klen = lens; a.Tq = T; a.Tk = T; a.scale = 1.f / sqrtf(128.f); a.fw = fw; a.fout = nullptr; a.fld = D; a.fD = D;
    a.fout32 = fo;
    const double fl = 6.0 * 4.0 * B * (double)T * T * 128 * 4;   // bf16 MFMA FLOPs issued (six products)
    for (int round = 0; round < 2; ++round) {
        const float t0 = run_x6<0>(a, B, T, reps), t1 = run_x6<1>(a, B, T, reps), t2 = run_x6<2>(a, B, T, reps),
                    t3 = run_x6<3>(a, B, T, reps), t4 = run_x6<4>(a, B, T, reps);
        AttnArgs an = a;
        an.fout32 = nullptr;
        const float t5 = run_x6<0>(an, B, T, reps);
        printf("x6 B=%d: kernel %.1f us (%.0f TF issued) | no staging %.1f | no softmax %.1f | no PV %.1f | no QK %.1f | "
               "no FSMN %.1f\n", B, t0, fl / t0 / 1e6, t1, t2, t3, t4, t5);
    }
}

int main(int argc, char** argv) {
    const int T = 500, H = 4, D = 512;
    const int Bmax = 64;
    bf16 *qkv, *ob, *fb;
    float* fw;
    int* lens;
    CK(hipMalloc(&qkv, (size_t)Bmax * T * 3 * D * 2));
    CK(hipMalloc(&ob, (size_t)Bmax * T * D * 2));
    CK(hipMalloc(&fb, (size_t)Bmax * T * D * 2));
    CK(hipMalloc(&fw, 11 * D * 4));
    CK(hipMalloc(&lens, Bmax * 4));
    long long n = (long long)Bmax * T * 3 * D;
    hipLaunchKernelGGL(fill_bf16, dim3((n + 255) / 256), dim3(256), 0, 0, qkv, n, 1u, 4.f);
    hipLaunchKernelGGL(fill_f32, dim3((11 * D + 255) / 256), dim3(256), 0, 0, fw, 11LL * D, 2u, 0.5f);
    std::vector<int> hl(Bmax, T);
    CK(hipMemcpy(lens, hl.data(), Bmax * 4, hipMemcpyHostToDevice));
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    bench_x6(reps);
    for (int B : {32, 64}) {
        AttnArgs a;
        a.q = qkv; a.qmap = rowmap_plain(3 * D);
        a.k = qkv + D; a.kmap = rowmap_plain(3 * D);
        a.v = qkv + 2 * D; a.vmap = rowmap_plain(3 * D);
        a.o = nullptr; a.ldo = D; a.o2 = ob; a.o2_dtype = DT_BF16; a.klen = lens; a.Tq = T; a.Tk = T;
        a.scale = 1.f / sqrtf(128.f); a.fw = fw; a.fout = fb; a.fld = D; a.fD = D;
        const double fl = 4.0 * B * (double)T * T * 128 * H;
        for (int round = 0; round < 2; ++round) {
            float t[8] = {run<0>(a, B, T, reps), run<1>(a, B, T, reps), run<2>(a, B, T, reps), run<3>(a, B, T, reps),
                          run<4>(a, B, T, reps), run<5>(a, B, T, reps), 0.f, 0.f};
            AttnArgs an = a;
            an.fout = nullptr;
            t[6] = run<0>(an, B, T, reps);
            printf("B=%d: kernel %.1f us (%.0f TF) | noKV %.1f | noSM %.1f | noPV %.1f | noQK %.1f | noLoop %.1f | "
                   "no FSMN %.1f\n", B, t[0], fl / t[0] / 1e6, t[1], t[2], t[3], t[4], t[5], t[6]);
        }
    }
    return 0;
}
