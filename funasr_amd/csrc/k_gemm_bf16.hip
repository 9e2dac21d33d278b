// bf16 MFMA GEMM, 256x256 block tile, for the FAST-mode projections (gfx950).
//
//   C[M,N] = epi( A[M,K] . W[N,K]^T ),  A/W bf16 K-contiguous rows, f32 accumulate.
//
// Geometry: 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 output tile =
// 4x2 blocks of v_mfma_f32_32x32x16_bf16 (128 accumulator registers). K-step 64 (one 128-B
// row segment per operand row); arithmetic intensity 128 FLOP per staged byte.
// Staging: global_load_lds_dwordx4 straight into LDS (no register round trip), two 64 KiB
// stages (A and W tiles, 256 rows x 128 B each). An LDS-DMA writes lane-linear 1 KiB pieces
// (8 rows), so the bank swizzle is applied on the SOURCE address: LDS slot s of row r holds
// logical 16-B chunk s ^ ((r >> 1) & 7), which makes every ds_read_b128 fragment read (16
// distinct rows per lane group, same chunk) bank-conflict free.
// Pipeline (2-phase): at K-step k the DMA of step k+1 is issued first, then the 32 MFMAs of
// step k run from LDS, then vmcnt(0) + barrier.
// Requirements (checked by the launcher): K % 64 == 0, row strides % 8 == 0 (16-B aligned
// rows). Rows beyond M / N are clamped (valid memory) and dropped in the epilogue.
#include <stdlib.h>

#include "pfm_common.h"

namespace {

constexpr int BM = 256, BN = 256;

// Geometry of one variant: BK (K per stage, bf16 elements) and NS (LDS ring stages).
template <int BK_, int NS_> struct Geo {
    static constexpr int BK = BK_, NS = NS_;
    static constexpr int ROWB = BK * 2;              // bytes per tile row per stage (128 or 64)
    static constexpr int CPR = ROWB / 16;            // 16-B chunks per row (8 or 4)
    static constexpr int TILE = BM * ROWB;           // A tile bytes (W tile the same)
    static constexpr int STAGE = 2 * TILE;
    static constexpr int PIECES = TILE / 1024 / 8;   // 1-KiB DMA pieces per wave per operand
    static constexpr int LDS = NS * STAGE;
    // bank swizzle of 16-B slot within a row: conflict-free ds_read_b128 of 16 distinct rows
    __device__ static inline int swz(int row) { return CPR == 8 ? ((row >> 1) & 7) : ((row >> 2) & 3); }
};

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

template <int Vb, int Vs> __device__ __forceinline__ void wait_stage(int rem) {
    // wait until at most `rem` later stages (each 2*PIECES DMA instructions per thread) are in flight
    constexpr int P = 2 * Geo<Vb, Vs>::PIECES;
    if (rem >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * P) : "memory");
    else if (rem == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
    else if (rem == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BK_, int NS_>
__global__ __launch_bounds__(512) void gemm_bf16_256_kernel(const bf16* __restrict__ A, RowMap amap,
                                                            const bf16* __restrict__ W, long long ldw, int M, int N,
                                                            int K, int tiles_n, GemmEpi epi) {
    using G = Geo<BK_, NS_>;
    constexpr int BK = G::BK, ROWB = G::ROWB, TILE = G::TILE, STAGE = G::STAGE, PIECES = G::PIECES, NS = G::NS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 2, wn = wid & 3;

    // ---- DMA source addresses: wave w, piece j covers rows (PIECES*w + j) * RPP .. +RPP-1
    constexpr int RPP = 1024 / ROWB;   // rows per 1-KiB piece
    const bf16* ga[PIECES];
    const bf16* gw[PIECES];
    {
        const int sub = lane / G::CPR, slot = lane % G::CPR;
#pragma unroll
        for (int j = 0; j < PIECES; ++j) {
            const int row = RPP * (PIECES * wid + j) + sub;
            const int chunk = slot ^ G::swz(row);
            const int am = min(m0 + row, M - 1), wr = min(n0 + row, N - 1);
            ga[j] = A + amap.off(am) + chunk * 8;
            gw[j] = W + (long long)wr * ldw + chunk * 8;
        }
    }
    auto stage = [&](int k0, int s) {
        unsigned char* base = smem + s * STAGE;
#pragma unroll
        for (int j = 0; j < PIECES; ++j) {
            const int piece = PIECES * wid + j;
            __builtin_amdgcn_global_load_lds((gbl_void*)(ga[j] + k0), (lds_void*)(base + piece * 1024), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gbl_void*)(gw[j] + k0), (lds_void*)(base + TILE + piece * 1024), 16, 0,
                                             0);
        }
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int fr = lane & 31, fh = lane >> 5;
    // per-lane read offsets (row part) for the A and W fragments
    int aoff[4], woff[2], asw[4], wsw[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = wm * 128 + i * 32 + fr;
        aoff[i] = row * ROWB;
        asw[i] = G::swz(row);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int row = wn * 64 + j * 32 + fr;
        woff[j] = TILE + row * ROWB;
        wsw[j] = G::swz(row);
    }

    const int nk = K / BK;
    // prologue: NS-1 stages in flight
#pragma unroll
    for (int sidx = 0; sidx < NS - 1; ++sidx)
        if (sidx < nk) stage(sidx * BK, sidx);
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed for this wave's DMAs (later stages may stay in flight), then the barrier
        // makes every wave's pieces visible and frees slot (kt-1) % NS for re-staging
        wait_stage<BK_, NS_>(min(NS - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + NS - 1 < nk) stage((kt + NS - 1) * BK, (kt + NS - 1) % NS);
        const unsigned char* sb = smem + (kt % NS) * STAGE;
#pragma unroll
        for (int kq = 0; kq < BK / 16; ++kq) {
            const int c = 2 * kq + fh;
            bf16x8 af[4], bfr[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(sb + aoff[i] + ((c ^ asw[i]) << 4));
#pragma unroll
            for (int j = 0; j < 2; ++j) bfr[j] = *(const bf16x8*)(sb + woff[j] + ((c ^ wsw[j]) << 4));
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- epilogue (C/D map: col = lane&31, row = (e&3) + 8(e>>2) + 4(lane>>5))
    if (epi.vec_ok || epi.amax_val) {
        // LDS-staged epilogue: each wave re-lays its 32x64 sub-tiles row-major in its own 8.5 KiB
        // LDS slice, then every lane handles float4 column groups of whole rows: 16-B bias /
        // residual loads and 16-B (f32) or 8-B (bf16) stores, 256 contiguous bytes per 16 lanes.
        constexpr int EP = 68;                              // floats per staged row (64 + 4 pad)
        float* ep = (float*)(smem + wid * (32 * EP * 4));
        const bool f32o = epi.out_dtype == DT_F32;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
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
                const int row = m0 + wm * 128 + i * 32 + rr;
                if (half == 0 && row < M) {
                    const long long p = (long long)row * epi.n_tiles + (tn * 4 + wn);
                    epi.amax_val[p] = bv;
                    epi.amax_idx[p] = bi;
                }
            }
#pragma unroll
            for (int sidx = 0; sidx < 8; ++sidx) {
                if (!epi.out) break;
                const int f = lane + 64 * sidx, rr = f >> 4, c4 = f & 15;
                const int row = m0 + wm * 128 + i * 32 + rr;
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
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + wm * 128 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
            if (row >= M) continue;
            const long long ob = epi.out_map.off(row);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = n0 + wn * 64 + j * 32 + fr;
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

int gemm_variant() {   // PFM_GEMM_VARIANT: 0 = BK64 x 2 stages, 1 = BK32 x 4, 2 = BK32 x 5, 3 = BK64 x 2 (alias)
    static int v = -1;
    if (v < 0) { const char* e = getenv("PFM_GEMM_VARIANT"); v = e ? atoi(e) : 0; }
    return v;
}

template <int BK_, int NS_>
hipError_t launch_variant(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                          const GemmEpi& e2, hipStream_t st) {
    using G = Geo<BK_, NS_>;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)gemm_bf16_256_kernel<BK_, NS_>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
    }
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    hipLaunchKernelGGL((gemm_bf16_256_kernel<BK_, NS_>), dim3(tiles_m * tiles_n), dim3(512), G::LDS, st,
                       (const bf16*)A, amap, (const bf16*)W, ldw, M, N, K, tiles_n, e2);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace


bool pfm_gemm_bf16_256_ok(RowMap amap, long long ldw, int K) {
    return K % 64 == 0 && ldw % 8 == 0 && amap.ld % 8 == 0 && (amap.rows_per_seg <= 0 || amap.seg_stride % 8 == 0);
}

int pfm_gemm_bf16_256_amax_tiles(int N) { return ((N + BN - 1) / BN) * (BN / 64); }

hipError_t pfm_gemm_bf16_256(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                             const GemmEpi& epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (!pfm_gemm_bf16_256_ok(amap, ldw, K)) return hipErrorInvalidValue;
    GemmEpi e2 = epi;
    e2.vec_ok = epi_vec_ok(epi, N);
    switch (gemm_variant()) {
        case 1: return launch_variant<32, 4>(A, amap, W, ldw, M, N, K, e2, st);
        case 2: return launch_variant<32, 5>(A, amap, W, ldw, M, N, K, e2, st);
        default: return launch_variant<64, 2>(A, amap, W, ldw, M, N, K, e2, st);
    }
}
