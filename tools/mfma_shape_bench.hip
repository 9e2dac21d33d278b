// Does the 16x16x32 bf16 MFMA shape sustain more FLOP/s than 32x32x16 in the fused FFN kernel's stream form?
// One wave per SIMD (256 threads, 512-register budget), one workgroup per CU, 256 workgroups; per step one
// ds_read_b128 weight fragment (1 KiB, read PD = 7 steps ahead, counted lgkmcnt) feeding 32 MFMA-cycles of work:
//   shape 0: one v_mfma_f32_32x32x16_bf16 into one of 16 f32x16 AGPR blocks (ffn2_kernel's form)
//   shape 1: two v_mfma_f32_16x16x32_bf16 (two 16-row groups) into f32x4 AGPR quads
// Random operands; ~2 s of back-to-back launches before the timed ones (the clock the chip holds under load); the
// in-kernel shader clock from s_memtime / s_memrealtime. Prints us per launch and TFLOP/s per shape, interleaved.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mfma_shape_bench.hip -o tools/mfma_shape_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int PD = 7, NB = 8, STEPS = 4096, RINGF = 64;   // 64 KiB of fragments, read cyclically

template <int SHAPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void stream_kernel(
    const bf16x8* __restrict__ wsrc, const bf16x8* __restrict__ asrc, float* out, unsigned long long* clk) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < RINGF * 64; i += 256) ((bf16x8*)smem)[i] = wsrc[i];
    bf16x8 act[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) act[k] = asrc[(blockIdx.x * 256 + tid) * 32 + k];
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)smem + lane * 16;
    bf16x8 wf[NB];
    auto rd = [&](int f, bf16x8& d) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"((f % RINGF) * 1024));
    };
#pragma unroll
    for (int f = 0; f < PD; ++f) rd(f, wf[f]);
    f32x16 acc[16];
    f32x4 q[64];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f32x16{};
#pragma unroll
    for (int i = 0; i < 64; ++i) q[i] = f32x4{};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < STEPS / 64; ++it) {
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            rd(s + PD, wf[(s + PD) % NB]);
            asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(wf[s % NB]) : "i"(PD));
            if constexpr (SHAPE == 0) {
                asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[s & 15]) : "v"(wf[s % NB]), "v"(act[s & 31]));
            } else {
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(q[(2 * s) & 63]) : "v"(wf[s % NB]), "v"(act[(2 * s) & 31]));
                asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(q[(2 * s + 1) & 63]) : "v"(wf[s % NB]), "v"(act[(2 * s + 1) & 31]));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]), "+v"(wf[4]), "+v"(wf[5]),
                 "+v"(wf[6]), "+v"(wf[7]));
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    if constexpr (SHAPE == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s += acc[i][lane & 15];
    } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) s += q[i][lane & 3];
    }
    out[blockIdx.x * 256 + tid] = s;
    if (tid == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

__global__ void fill(unsigned short* p, long long n, unsigned seed) {
    long long i = blockIdx.x * 256LL + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    // bf16 with exponent near 1.0 and random sign / mantissa
    p[i] = (unsigned short)(0x3f00u | (x & 0x807fu));
}

template <int SHAPE>
float run(int reps, const bf16x8* w, const bf16x8* a, float* out, unsigned long long* clk, double& ghz) {
    const int nb = 256, lds = RINGF * 1024;
    CK(hipFuncSetAttribute((const void*)stream_kernel<SHAPE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(stream_kernel<SHAPE>, dim3(nb), dim3(256), lds, 0, w, a, out, clk);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c(2 * nb);
    CK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> g;
    for (int b = 0; b < nb; ++b) g.push_back((double)c[2 * b] / (double)c[2 * b + 1] * 0.1);
    std::sort(g.begin(), g.end());
    ghz = g[nb / 2];
    return ms * 1e3f / reps;
}

int main() {
    const long long nw = RINGF * 64 * 8, na = 256LL * 256 * 32 * 8;
    unsigned short *w, *a;
    float* out;
    unsigned long long* clk;
    CK(hipMalloc(&w, nw * 2));
    CK(hipMalloc(&a, na * 2));
    CK(hipMalloc(&out, 256 * 256 * 4));
    CK(hipMalloc(&clk, 256 * 16));
    hipLaunchKernelGGL(fill, dim3((nw + 255) / 256), dim3(256), 0, 0, w, nw, 1u);
    hipLaunchKernelGGL(fill, dim3((na + 255) / 256), dim3(256), 0, 0, a, na, 2u);
    const double fl = 256.0 * 4 * STEPS * 32768.0;   // FLOP per launch (both shapes)
    double g;
    run<0>(4000, (bf16x8*)w, (bf16x8*)a, out, clk, g);   // sustained load first
    for (int r = 0; r < 3; ++r) {
        double g0, g1;
        const float t0 = run<0>(1500, (bf16x8*)w, (bf16x8*)a, out, clk, g0);
        const float t1 = run<1>(1500, (bf16x8*)w, (bf16x8*)a, out, clk, g1);
        printf("round %d: 32x32x16 %.1f us %.0f TF/s (clock %.3f GHz) | 16x16x32 %.1f us %.0f TF/s (clock %.3f GHz) | ratio %.3f\n",
               r, t0, fl / t0 / 1e6, g0, t1, fl / t1 / 1e6, g1, t0 / t1);
    }
    return 0;
}
