// Microbenchmark: cost of a dependent phase as a kernel boundary (a chain of tiny launches, eager and graphed) vs as a
// grid-wide barrier inside one persistent launch (G co-resident workgroups, agent-scope counter + generation word,
// bounded spin). Each phase: every workgroup reads one 16-B word another workgroup wrote in the previous phase.
//   tools/grid_barrier_bench [G] [phases]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ void grid_sync(unsigned* cnt, unsigned* gen, unsigned G, int* fail) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int it = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++it > (1 << 22)) { *fail = 1; break; }
            }
        }
    }
    __syncthreads();
    __threadfence();
}

__global__ __launch_bounds__(512) void persist(float4* buf, unsigned* cnt, unsigned* gen, int phases, int* fail) {
    const unsigned G = gridDim.x;
    float4 acc = make_float4(0, 0, 0, 0);
    for (int p = 0; p < phases; ++p) {
        if (threadIdx.x == 0) {
            const float4 v = buf[(blockIdx.x + 1) % G];
            acc.x += v.x + 1.f;
            buf[blockIdx.x] = acc;
        }
        grid_sync(cnt, gen, G, fail);
    }
}

__global__ __launch_bounds__(512) void step(float4* buf, int G) {
    if (threadIdx.x == 0) {
        float4 v = buf[(blockIdx.x + 1) % G];
        v.x += 1.f;
        buf[G + blockIdx.x] = v;
    }
}

int main(int argc, char** argv) {
    const int G = argc > 1 ? atoi(argv[1]) : 64, P = argc > 2 ? atoi(argv[2]) : 31;
    float4* buf;
    unsigned *cnt, *gen;
    int* fail;
    hipMalloc(&buf, 2 * G * sizeof(float4));
    hipMalloc(&cnt, 4); hipMalloc(&gen, 4); hipMalloc(&fail, 4);
    hipMemset(buf, 0, 2 * G * sizeof(float4)); hipMemset(cnt, 0, 4); hipMemset(gen, 0, 4); hipMemset(fail, 0, 4);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float ms;
    const int R = 200;
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(persist, dim3(G), dim3(512), 0, st, buf, cnt, gen, P, fail);
    hipEventRecord(a, st);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL(persist, dim3(G), dim3(512), 0, st, buf, cnt, gen, P, fail);
    hipEventRecord(b, st); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    int f = 0; hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
    printf("persistent G=%d: %.2f us per launch of %d phases = %.2f us per phase (fail %d)\n", G, ms * 1e3 / R, P,
           ms * 1e3 / R / P, f);
    for (int w = 0; w < 2; ++w) for (int p = 0; p < P; ++p) hipLaunchKernelGGL(step, dim3(G), dim3(512), 0, st, buf, G);
    hipEventRecord(a, st);
    for (int r = 0; r < R; ++r) for (int p = 0; p < P; ++p) hipLaunchKernelGGL(step, dim3(G), dim3(512), 0, st, buf, G);
    hipEventRecord(b, st); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("launch chain G=%d: %.2f us per %d launches = %.2f us per launch\n", G, ms * 1e3 / R, P, ms * 1e3 / R / P);
    hipGraph_t gph; hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int p = 0; p < P; ++p) hipLaunchKernelGGL(step, dim3(G), dim3(512), 0, st, buf, G);
    hipStreamEndCapture(st, &gph);
    hipGraphInstantiate(&ge, gph, nullptr, nullptr, 0);
    hipGraphLaunch(ge, st); hipStreamSynchronize(st);
    hipEventRecord(a, st);
    for (int r = 0; r < R; ++r) hipGraphLaunch(ge, st);
    hipEventRecord(b, st); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    printf("graph chain G=%d: %.2f us per %d launches = %.2f us per launch\n", G, ms * 1e3 / R, P, ms * 1e3 / R / P);
    return 0;
}
