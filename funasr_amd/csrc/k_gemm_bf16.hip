// bf16 MFMA GEMM family for the FAST-mode projections (gfx950).
//
//   C[M,N] = epi( A[M,K] . W[N,K]^T ),  A/W bf16 K-contiguous rows, f32 accumulate.
//
// Cfg<BM, BN, WGM, WGN, BK, NS>: block tile BM x BN on WGM x WGN waves; each wave owns a
// (BM/WGM) x (BN/WGN) tile = MI x NI blocks of v_mfma_f32_32x32x16_bf16; K-step BK; NS-stage
// LDS ring. Staging is global_load_lds_dwordx4 straight into LDS; an LDS-DMA writes lane-linear
// 1 KiB pieces, so the bank swizzle is applied on the SOURCE address: LDS slot s of row r holds
// logical 16-B chunk s ^ swz(r), which makes every ds_read_b128 fragment read (16 distinct rows
// per lane group, same chunk) conflict-free. Counted vmcnt waits + raw s_barrier per K-step.
// Epilogue: each wave re-lays its 32-row sub-tiles row-major in its own LDS slice; lanes then
// handle float4 column groups of whole rows (16-B bias/residual loads, 16-B f32 / 8-B bf16
// stores), or scan rows for the fused row-argmax of the output layer.
// Launcher contract: K % BK == 0, row strides % 8 == 0 (16-B aligned rows). Rows beyond M / N
// are clamped to valid memory and dropped in the epilogue.
#include <stdlib.h>

#include "pfm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int BM_, int BN_, int WGM_, int WGN_, int BK_, int NS_> struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, BK = BK_, NS = NS_;
    static constexpr int NW = WGM * WGN, NT = NW * 64;
    static constexpr int WTM = BM / WGM, WTN = BN / WGN;
    static constexpr int MI = WTM / 32, NI = WTN / 32;
    static constexpr int ROWB = BK * 2, CPR = ROWB / 16, RPP = 1024 / ROWB;
    static constexpr int TA = BM * ROWB, TW = BN * ROWB, STAGE = TA + TW;
    static constexpr int PA = TA / 1024 / NW, PW = TW / 1024 / NW;
    static constexpr int EP = WTN + 4;                 // staged epilogue row pitch (floats)
    static constexpr int EPW = 32 * EP * 4;            // epilogue LDS bytes per wave
    static constexpr int LDS = (NS * STAGE > NW * EPW) ? NS * STAGE : NW * EPW;
    static_assert(TA % (1024 * NW) == 0 && TW % (1024 * NW) == 0, "tile not divisible into DMA pieces");
    static_assert(WTN == 64, "epilogue / argmax partials assume 64-column wave tiles");
    __device__ static inline int swz(int row) { return CPR == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3); }
};

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

template <int P> __device__ __forceinline__ void wait_vm(int rem) {
    if (rem >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
    else if (rem == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class C>
__global__ __launch_bounds__(C::NT) void gemm_bf16_kernel(const bf16* __restrict__ A, RowMap amap,
                                                          const bf16* __restrict__ W, long long ldw, int M, int N,
                                                          int K, int tiles_n, GemmEpi epi) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BK = C::BK, NS = C::NS, ROWB = C::ROWB, MI = C::MI, NI = C::NI, PA = C::PA, PW = C::PW;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int m0 = tm * C::BM, n0 = tn * C::BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / C::WGN, wn = wid % C::WGN;
    const int fr = lane & 31, fh = lane >> 5;

    const bf16* ga[PA];
    const bf16* gw[PW];
    {
        const int sub = lane / C::CPR, slot = lane % C::CPR;
#pragma unroll
        for (int j = 0; j < PA; ++j) {
            const int row = C::RPP * (PA * wid + j) + sub;
            ga[j] = A + amap.off(min(m0 + row, M - 1)) + (slot ^ C::swz(row)) * 8;
        }
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            const int row = C::RPP * (PW * wid + j) + sub;
            gw[j] = W + (long long)min(n0 + row, N - 1) * ldw + (slot ^ C::swz(row)) * 8;
        }
    }
    auto stage = [&](int k0, int s) {
        unsigned char* base = smem + s * C::STAGE;
#pragma unroll
        for (int j = 0; j < PA; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void*)(ga[j] + k0), (lds_void*)(base + (PA * wid + j) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int j = 0; j < PW; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void*)(gw[j] + k0),
                                             (lds_void*)(base + C::TA + (PW * wid + j) * 1024), 16, 0, 0);
    };

    f32x16 acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    int aoff[MI], asw[MI], woff[NI], wsw[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int row = wm * C::WTM + i * 32 + fr;
        aoff[i] = row * ROWB;
        asw[i] = C::swz(row);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
        const int row = wn * C::WTN + j * 32 + fr;
        woff[j] = C::TA + row * ROWB;
        wsw[j] = C::swz(row);
    }

    const int nk = K / BK;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) stage(s * BK, s);
    for (int kt = 0; kt < nk; ++kt) {
        wait_vm<PA + PW>(min(NS - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NS - 1 < nk) stage((kt + NS - 1) * BK, (kt + NS - 1) % NS);
        const unsigned char* sb = smem + (kt % NS) * C::STAGE;
#pragma unroll
        for (int kq = 0; kq < BK / 16; ++kq) {
            const int c = 2 * kq + fh;
            bf16x8 af[MI], bfr[NI];
#pragma unroll
            for (int i = 0; i < MI; ++i) af[i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
#pragma unroll
            for (int j = 0; j < NI; ++j) bfr[j] = *(const bf16x8*)(sb + woff[j] + ((c ^ wsw[j]) << 4));
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- epilogue (C/D map: col = lane&31, row = (e&3) + 8(e>>2) + 4(lane>>5))
    if (epi.vec_ok || epi.amax_val) {
        constexpr int EP = C::EP;
        float* ep = (float*)(smem + wid * C::EPW);
        const bool f32o = epi.out_dtype == DT_F32;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
            for (int j = 0; j < NI; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) ep[((e & 3) + 8 * (e >> 2) + 4 * fh) * EP + j * 32 + fr] = acc[i][j][e];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (epi.amax_val) {
                // fused row-argmax of the output layer over this wave's 64 columns: 2 lanes per staged
                // row scan 32 columns each in order (first index wins ties, like torch.argmax)
                const int rr = lane >> 1, half = lane & 1;
                const int cb = n0 + wn * 64 + half * 32;
                float bv = -INFINITY;
                int bi = 0x7fffffff;
                for (int cc = 0; cc < 32; ++cc) {
                    const int col = cb + cc;
                    if (col < N) {
                        const float v = ep[rr * EP + half * 32 + cc] * epi.alpha + (epi.bias ? epi.bias[col] : 0.f);
                        if (v > bv) { bv = v; bi = col; }
                    }
                }
                const float ov = __shfl_xor(bv, 1, 64);
                const int oi = __shfl_xor(bi, 1, 64);
                if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
                const int row = m0 + wm * C::WTM + i * 32 + rr;
                if (half == 0 && row < M) {
                    const long long p = (long long)row * epi.n_tiles + (n0 + wn * 64) / 64;
                    epi.amax_val[p] = bv;
                    epi.amax_idx[p] = bi;
                }
            }
#pragma unroll
            for (int sidx = 0; sidx < 8; ++sidx) {
                if (!epi.out) break;
                const int f = lane + 64 * sidx, rr = f >> 4, c4 = f & 15;
                const int row = m0 + wm * C::WTM + i * 32 + rr;
                const int col = n0 + wn * 64 + c4 * 4;
                if (row >= M || col >= N) continue;
                float4 v = *(const float4*)(ep + rr * EP + c4 * 4);
                v.x *= epi.alpha; v.y *= epi.alpha; v.z *= epi.alpha; v.w *= epi.alpha;
                if (epi.bias) {
                    const float4 bb = *(const float4*)(epi.bias + col);
                    v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
                }
                if (epi.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
                if (epi.res0) {
                    float4 r0;
                    if (epi.res0_bf16) {
                        const bf16x4 rb = *(const bf16x4*)((const bf16*)epi.res0 + (long long)row * epi.ld_res0 + col);
                        r0 = make_float4(bf2f(rb[0]), bf2f(rb[1]), bf2f(rb[2]), bf2f(rb[3]));
                    } else {
                        r0 = *(const float4*)(epi.res0 + (long long)row * epi.ld_res0 + col);
                    }
                    v.x += r0.x; v.y += r0.y; v.z += r0.z; v.w += r0.w;
                }
                if (epi.res1) {
                    const float4 r1 = *(const float4*)(epi.res1 + (long long)row * epi.ld_res1 + col);
                    v.x += r1.x; v.y += r1.y; v.z += r1.z; v.w += r1.w;
                }
                const long long ob = epi.out_map.off(row) + col;
                if (f32o) *(float4*)((float*)epi.out + ob) = v;
                else {
                    bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                    *(bf16x4*)((bf16*)epi.out + ob) = t;
                }
                if (epi.out2) {
                    bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
                    *(bf16x4*)((bf16*)epi.out2 + epi.out2_map.off(row) + col) = t;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        return;
    }
    // scalar fallback epilogue (odd N / strides): straight from the accumulators
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + wm * C::WTM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
            if (row >= M) continue;
            const long long ob = epi.out_map.off(row);
#pragma unroll
            for (int j = 0; j < NI; ++j) {
                const int col = n0 + wn * C::WTN + j * 32 + fr;
                if (col >= N) continue;
                float v = acc[i][j][e] * epi.alpha;
                if (epi.bias) v += epi.bias[col];
                if (epi.relu) v = fmaxf(v, 0.f);
                if (epi.res0) v += epi.res0_bf16 ? bf2f(((const bf16*)epi.res0)[(long long)row * epi.ld_res0 + col])
                                                 : epi.res0[(long long)row * epi.ld_res0 + col];
                if (epi.res1) v += epi.res1[(long long)row * epi.ld_res1 + col];
                if (epi.out_dtype == DT_F32) ((float*)epi.out)[ob + col] = v;
                else ((bf16*)epi.out)[ob + col] = f2bf(v);
                if (epi.out2) ((bf16*)epi.out2)[epi.out2_map.off(row) + col] = f2bf(v);
            }
        }
    }
}

// tile configurations (PFM_GEMM_CFG selects one per launch for A/B runs; 0 = automatic)
using C1 = Cfg<256, 256, 2, 4, 64, 2>;   // 128 KiB LDS, 8 waves, wave 128x64, 1 block/CU
using C2 = Cfg<256, 128, 4, 2, 32, 3>;   // 72 KiB, 8 waves, wave 64x64, 2 blocks/CU
using C3 = Cfg<128, 128, 2, 2, 64, 2>;   // 64 KiB, 4 waves, wave 64x64, 2 blocks/CU
using C4 = Cfg<128, 256, 2, 4, 32, 3>;   // 72 KiB, 8 waves, wave 64x64, 2 blocks/CU
using C5 = Cfg<256, 256, 2, 4, 32, 4>;   // 128 KiB, BK 32 x 4 stages

template <class C>
hipError_t launch(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K, const GemmEpi& e2,
                  hipStream_t st) {
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    }
    const int tiles_m = (M + C::BM - 1) / C::BM, tiles_n = (N + C::BN - 1) / C::BN;
    hipLaunchKernelGGL(gemm_bf16_kernel<C>, dim3(tiles_m * tiles_n), dim3(C::NT), C::LDS, st, (const bf16*)A, amap,
                       (const bf16*)W, ldw, M, N, K, tiles_n, e2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int pick_cfg(int M, int N) {
    const char* e = getenv("PFM_GEMM_CFG");   // read per launch: lets one process A/B configurations
    const int f = e ? atoi(e) : 0;
    if (f >= 1 && f <= 5) return f;
    // 256x256 when the grid has >= 2 tiles per CU, else 128x256 (64x64 wave tiles, 2 blocks / CU)
    const long long big = (long long)((M + 255) / 256) * ((N + 255) / 256);
    return big >= 512 ? 1 : 4;
}

}  // namespace

bool pfm_gemm_bf16_256_ok(RowMap amap, long long ldw, int K) {
    return K % 64 == 0 && ldw % 8 == 0 && amap.ld % 8 == 0 && (amap.rows_per_seg <= 0 || amap.seg_stride % 8 == 0);
}

// argmax partials: one per (row, 64-column block), row stride rounded up to 256 columns
int pfm_gemm_bf16_256_amax_tiles(int N) { return (N + 255) / 256 * 4; }

hipError_t pfm_gemm_bf16_256(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                             const GemmEpi& epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (!pfm_gemm_bf16_256_ok(amap, ldw, K)) return hipErrorInvalidValue;
    GemmEpi e2 = epi;
    e2.vec_ok = epi_vec_ok(epi, N);
    switch (pick_cfg(M, N)) {
        case 2: return launch<C2>(A, amap, W, ldw, M, N, K, e2, st);
        case 3: return launch<C3>(A, amap, W, ldw, M, N, K, e2, st);
        case 4: return launch<C4>(A, amap, W, ldw, M, N, K, e2, st);
        case 5: return launch<C5>(A, amap, W, ldw, M, N, K, e2, st);
        default: return launch<C1>(A, amap, W, ldw, M, N, K, e2, st);
    }
}
