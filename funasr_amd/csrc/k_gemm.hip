// MFMA GEMM for every dense projection on the Paraformer path (gfx950).
//
//   C[M,N] = epi( alpha * A[M,K] . W[N,K]^T )
//
// W is the torch nn.Linear weight as stored in the state_dict ([out, in], K-contiguous),
// so both operands stream K-contiguous rows ("NT" GEMM) and no weight transpose is needed.
// Replaces the ATen addmm calls behind nn.Linear in funasr/models/sanm/attention.py:193,240,
// transformer/positionwise_feed_forward.py:32-34, sanm/positionwise_feed_forward.py:26-33,
// paraformer/decoder.py:406 and the k=3 conv of paraformer/cif_predictor.py:214 (as a GEMM
// over three adjacent encoder rows).
//
// Two precisions share one tiling:
//   float : v_mfma_f32_32x32x2_f32  (exact f32 FMA chain; "exact" mode, token-ID parity)
//   bf16  : v_mfma_f32_32x32x16_bf16 (f32 accumulate; "fast" mode)
// Block tile 128x128, 4 waves (2x2), each wave a 64x64 tile = 2x2 MFMA 32x32 blocks.
// K-step = 128 bytes of each row (32 f32 / 64 bf16); LDS rows padded to 144 B so the
// ds_read_b128 fragment reads (16 rows x one 16-B slot per lane group) are conflict-free.
// Register-staged double buffer: the next K-step's global loads are in flight while the
// current one is consumed from LDS; one barrier per K-step.
#include "pfm_common.h"

namespace {

constexpr int BM = 128, BN = 128;
constexpr int ROWB = 128;          // bytes of K per row per K-step
constexpr int PITCH = 144;         // padded LDS row pitch (bytes)
constexpr int TILE_BYTES = BM * PITCH;
constexpr int LDS_BYTES = 2 /*stages*/ * 2 /*A,W*/ * TILE_BYTES;

template <typename T> struct Mf;
template <> struct Mf<float> {
    static constexpr int KSTEP = ROWB / 4;   // 32
    // lane holds float4 of k = kq*8 + 4h + c, c = 0..3  -> 4 MFMAs (K=2 each, halves give k and k+4)
    __device__ static inline void mma(const uint4& a, const uint4& b, f32x16& acc) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
    }
};
template <> struct Mf<bf16> {
    static constexpr int KSTEP = ROWB / 2;   // 64
    // lane holds bf16x8 of k = kq*16 + 8h + j -> one 32x32x16 MFMA
    __device__ static inline void mma(const uint4& a, const uint4& b, f32x16& acc) {
        bf16x8 av, bv;
        __builtin_memcpy(&av, &a, 16);
        __builtin_memcpy(&bv, &b, 16);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
};

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
    return v > bv || (v == bv && i < bi);
}

template <typename T>
__global__ __launch_bounds__(256) void gemm_nt_kernel(const T* __restrict__ A, RowMap amap,
                                                      const T* __restrict__ W, long long ldw,
                                                      int M, int N, int K, int tiles_n, GemmEpi epi) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int EPC = 16 / sizeof(T);      // elements per 16-B chunk
    constexpr int KS = Mf<T>::KSTEP;

    // XCD-aware bijective remap of the linear block id: consecutive logical tiles (same
    // A row-panel, neighbouring W panels) land on one XCD's L2.
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int tm = wg / tiles_n, tn = wg % tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;

    // global->register staging: 4 chunks of A and 4 of W per thread
    const T* ga[4];
    const T* gw[4];
    bool va[4], vw[4];
    int lrow[4], lch[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = tid + 256 * i;
        lrow[i] = c >> 3;
        lch[i] = c & 7;
        const int am = m0 + lrow[i], wn_ = n0 + lrow[i];
        va[i] = am < M;
        vw[i] = wn_ < N;
        ga[i] = A + (va[i] ? amap.off(am) : 0) + lch[i] * EPC;
        gw[i] = W + (vw[i] ? (long long)wn_ * ldw : 0) + lch[i] * EPC;
    }
    uint4 ra[4], rw[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool kin = (k0 + lch[i] * EPC) < K;
            ra[i] = (va[i] && kin) ? *(const uint4*)(ga[i] + k0) : make_uint4(0, 0, 0, 0);
            rw[i] = (vw[i] && kin) ? *(const uint4*)(gw[i] + k0) : make_uint4(0, 0, 0, 0);
        }
    };
    auto sstore = [&](int s) {
        unsigned char* As = smem + s * 2 * TILE_BYTES;
        unsigned char* Ws = As + TILE_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *(uint4*)(As + lrow[i] * PITCH + lch[i] * 16) = ra[i];
            *(uint4*)(Ws + lrow[i] * PITCH + lch[i] * 16) = rw[i];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int nk = (K + KS - 1) / KS;
    gload(0);
    sstore(0);
    __syncthreads();

    const int fr = lane & 31, fh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * KS);
        const unsigned char* As = smem + cur * 2 * TILE_BYTES;
        const unsigned char* Ws = As + TILE_BYTES;
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
            uint4 af[2], bfv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                af[i] = *(const uint4*)(As + (wm * 64 + i * 32 + fr) * PITCH + kq * 32 + fh * 16);
                bfv[i] = *(const uint4*)(Ws + (wn * 64 + i * 32 + fr) * PITCH + kq * 32 + fh * 16);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) Mf<T>::mma(af[i], bfv[j], acc[i][j]);
        }
        if (kt + 1 < nk) sstore(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    if (epi.amax_val) {
        // fused row-argmax over this wave's 64 columns (output layer; logits never hit HBM)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                float bv = -INFINITY;
                int bi = 0x7fffffff;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int col = n0 + wn * 64 + j * 32 + fr;
                    if (col < N) {
                        float v = acc[i][j][e] * epi.alpha + (epi.bias ? epi.bias[col] : 0.f);
                        if (better(v, col, bv, bi)) { bv = v; bi = col; }
                    }
                }
#pragma unroll
                for (int o = 1; o < 32; o <<= 1) {
                    const float ov = __shfl_xor(bv, o, 64);
                    const int oi = __shfl_xor(bi, o, 64);
                    if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
                }
                if (fr == 0 && row < M) {
                    const long long p = (long long)row * epi.n_tiles + (tn * 2 + wn);
                    epi.amax_val[p] = bv;
                    epi.amax_idx[p] = bi;
                }
            }
        }
        if (!epi.out) return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
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

}  // namespace

// Host launcher. A rows via amap, W [N, ldw]. dtype = DT_F32 (exact) or DT_BF16 (fast).
hipError_t pfm_gemm(int dtype, const void* A, RowMap amap, const void* W, long long ldw, int M, int N,
                    int K, const GemmEpi& epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const int epc = dtype == DT_F32 ? 4 : 8;
    if (K % epc != 0 || ldw % epc != 0) return hipErrorInvalidValue;
    static bool attr_done = false;
    if (!attr_done) {
        attr_done = true;
        (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
        (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<bf16>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    }
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    dim3 grid(tiles_m * tiles_n), block(256);
    if (dtype == DT_F32)
        hipLaunchKernelGGL(gemm_nt_kernel<float>, grid, block, LDS_BYTES, st, (const float*)A, amap,
                           (const float*)W, ldw, M, N, K, tiles_n, epi);
    else
        hipLaunchKernelGGL(gemm_nt_kernel<bf16>, grid, block, LDS_BYTES, st, (const bf16*)A, amap,
                           (const bf16*)W, ldw, M, N, K, tiles_n, epi);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

int pfm_gemm_amax_tiles(int N) { return 2 * ((N + BN - 1) / BN); }
