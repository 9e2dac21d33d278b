// Skinny-M bf16 GEMM: C[M, N] = epi(alpha * A[M, K] . W[N, K]^T) for M <= 64 (and the few-tile shapes
// above it: 64-row blocks on grid.y).
//
// The streaming chunk path (paraformer_streaming, pfm_stream_step) projects 5 + 10 window rows per
// stream through every encoder layer and 1..~10 token rows through every decoder layer. The tiled
// 128x256 / 256x256 kernels (k_gemm_bf16.hip) give such a GEMM 2-8 workgroups, so 2-8 CUs stream the
// whole weight matrix over K (measured 12-24 us per projection). Here the weight matrix is the only
// real traffic (N x K bf16, each byte read once), so the grid is laid out over it:
//   * one workgroup per 16 output columns (N = 512 -> 32 workgroups, 2048 -> 128), 8 waves;
//   * the K axis is cut into 32-wide steps dealt round-robin to the 8 waves, so one round of the
//     workgroup reads 512 contiguous bytes of each of its 16 weight rows (16-B fragments per lane,
//     straight from HBM into v_mfma_f32_16x16x32_bf16 B operands; no LDS staging);
//   * A fragments (rows m of 16-row blocks, <= 4 blocks) come from L2 (A is 15..64 rows);
//   * the 8 waves' 16x16 partials are summed through LDS in wave order (deterministic), then the
//     GemmEpi epilogue of the tiled kernels is applied per element (bias, alpha, relu, residuals,
//     f32 / bf16 output, optional bf16 second output).
// Fragment layout (as k_gemm_bf16.hip, MF == 1): lane (r = lane & 15, g = lane >> 4) holds row r,
// K chunk g (8 contiguous bf16) of a 16 x 32 operand; the accumulator element e of lane l is
// row 4 (l >> 4) + e, column l & 15.
#include "pfm_common.h"
#include "pfm_stream.h"

namespace {

constexpr int SK_WAVES = 8;
constexpr int SK_UNROLL = 4;   // 32-wide K steps whose fragments are in flight per wave (K <= 1024: one round)
// K = 2048 (FFN w2): 8 steps in flight per wave, so all 64 steps of a workgroup are one round of loads instead of two
// dependent ones (the accumulation order per wave is the same: steps w, w + 8, ..., w + 56)
constexpr int SK_UNROLL_WIDE = 8;

// The epilogue operands (bias, residuals) of the <= MT*256/512 elements a thread finishes, loaded at kernel start
// so their memory round trip overlaps the operand loads instead of following the K loop (these launches are
// latency-bound: each serial HBM / L2 round trip is a visible share of a 4-6 us kernel). Same values, same order.
template <int MT>
struct SkEpiPre {
    static constexpr int EPT = (MT * 256 + 511) / 512;
    float b[EPT], r0[EPT], r1[EPT];
    __device__ __forceinline__ void load(const GemmEpi& e, int mb, int n0, int M, int N) {
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int idx = threadIdx.x + j * 512;
            const int t = idx >> 8, rc = idx & 255;
            const int row = mb + t * 16 + (rc >> 4), col = n0 + (rc & 15);
            b[j] = 0.f; r0[j] = 0.f; r1[j] = 0.f;
            if (idx >= MT * 256 || row >= M || col >= N) continue;
            if (e.bias) b[j] = e.bias[col];
            if (e.res0) r0[j] = e.res0_bf16 ? bf2f(((const bf16*)e.res0)[(long long)row * e.ld_res0 + col])
                                            : e.res0[(long long)row * e.ld_res0 + col];
            if (e.res1) r1[j] = e.res1[(long long)row * e.ld_res1 + col];
        }
    }
};

template <int MT, int UNR = SK_UNROLL>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const bf16* __restrict__ A, RowMap amap,
                                                          const bf16* __restrict__ W, long long ldw, int M, int N,
                                                          int K, GemmEpi e) {
    __shared__ float red[SK_WAVES][MT][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r16 = lane & 15, g = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int n = n0 + r16;
    const int mb = blockIdx.y * 64;   // row block of this workgroup (M > 64: grid.y = ceil(M / 64))
    const bool nok = n < N;
    const bf16* wrow = W + (long long)(nok ? n : 0) * ldw + g * 8;
    const bf16* arow[MT];
    bool mok[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = mb + t * 16 + r16;
        mok[t] = m < M;
        arow[t] = A + amap.off(mok[t] ? m : 0) + g * 8;
    }
    SkEpiPre<MT> pre;
    pre.load(e, mb, n0, M, N);
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16x8 zero8 = {};
    const int nsteps = K / 32;
    for (int s0 = w; s0 < nsteps; s0 += SK_WAVES * UNR) {
        bf16x8 bw[UNR], ba[UNR][MT];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int s = s0 + u * SK_WAVES;
            const bool sok = s < nsteps;
            bw[u] = (sok && nok) ? *(const bf16x8*)(wrow + s * 32) : zero8;
#pragma unroll
            for (int t = 0; t < MT; ++t) ba[u][t] = (sok && mok[t]) ? *(const bf16x8*)(arow[t] + s * 32) : zero8;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba[u][t], bw[u], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[w][t][(4 * g + q) * 16 + r16] = acc[t][q];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SkEpiPre<MT>::EPT; ++j) {
        const int idx = threadIdx.x + j * 512;
        const int t = idx >> 8, rc = idx & 255;
        const int row = mb + t * 16 + (rc >> 4), col = n0 + (rc & 15);
        if (idx >= MT * 256 || row >= M || col >= N) continue;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < SK_WAVES; ++ww) v += red[ww][t][rc];
        v *= e.alpha;
        if (e.bias) v += pre.b[j];
        if (e.relu) v = fmaxf(v, 0.f);
        if (e.res0) v += pre.r0[j];
        if (e.res1) v += pre.r1[j];
        const long long ob = e.out_map.off(row);
        if (e.out_dtype == DT_F32) ((float*)e.out)[ob + col] = v;
        else ((bf16*)e.out)[ob + col] = f2bf(v);
        if (e.out2) ((bf16*)e.out2)[e.out2_map.off(row) + col] = f2bf(v);
    }
}

// The same GEMM with the LayerNorm of its A rows in front (streaming: LN1 -> QKV, LN2 -> FFN w1, decoder LN -> w1 / q):
// A = bf16(LN(X) g + b) for f32 rows X [M, K = 512]; every workgroup normalises the <= 64 rows of its row block into
// LDS (one wave per row, the statistics of layernorm_v8_kernel: f64 sums in the same order, f32 affine), so the
// LayerNorm's own launch and its bf16 round trip through HBM go away. Rows padded by 8 elements in LDS (conflict-free
// 16-B fragment reads across the 16 rows of a tile).
// VPL 512-wide segments per row (K = 512 VPL): f32 rows (the encoder / decoder inputs, VPL 1) or bf16 rows (the
// decoder FFN's 2048-wide hidden before w2, VPL 4, M <= 16); lane l holds elements 512 i + 8 l .. + 7 of segment i,
// summed in the order of layernorm_v8_kernel<VPL> (bit-identical LayerNorm output)
template <typename TIN>
__device__ __forceinline__ void ln_load8(const TIN* p, float4& a, float4& b) {
    if constexpr (sizeof(TIN) == 4) {
        a = *(const float4*)p;
        b = *(const float4*)(p + 4);
    } else {
        const bf16x8 t = *(const bf16x8*)p;
        a = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
        b = make_float4(bf2f(t[4]), bf2f(t[5]), bf2f(t[6]), bf2f(t[7]));
    }
}
// Streaming encoder layer (SQ): the LN1 -> QKV launch also builds the attention's key buffer and the window's FSMN
// memory block, the work of kv_gather_fsmn_kernel, because both are per column over all rows of one stream and a
// workgroup holds all M <= 64 rows of its 16 columns: K|V columns go to their buffer rows [cl, cl + tw) of each stream
// with the cached rows [0, cl) and zero rows [cl + tw, Tk) beside them (kv_gather_row), and the V columns' bf16 values
// (what QKVb holds) feed fsmn_win_body<11, bf16, 5>'s arithmetic from LDS.
struct SkQkv {
    const SPrm* prm;
    const bf16* cache;   // this layer's [slots][C][2d]
    bf16* buf;           // [n][Tk][2d]
    const float* wT;     // FSMN taps [11][d]
    bf16* fout;          // FSMN block output, [n Tw][d]
    int Tw, Tk, C, D;
};
constexpr int SQ_K = 11, SQ_LEFT = 5;

template <int MT, int VPL, typename TIN, bool SQ = false>
__global__ __launch_bounds__(512) void gemm_skinny_ln_kernel(const TIN* __restrict__ X, RowMap xmap,
                                                             const float* __restrict__ g, const float* __restrict__ bta,
                                                             float eps, const bf16* __restrict__ W, long long ldw, int M,
                                                             int N, GemmEpi e, SkQkv sq) {
    constexpr int LNK = 512 * VPL, LNP = LNK + 8;
    constexpr int UNR = VPL >= 4 ? SK_UNROLL_WIDE : SK_UNROLL;
    __shared__ float red[SK_WAVES][MT][256];
    __shared__ __attribute__((aligned(16))) bf16 As[MT * 16][LNP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int mb = blockIdx.y * 64;
    const int r16 = lane & 15, gq = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int n = n0 + r16;
    const bool nok = n < N;
    const bf16* wrow = W + (long long)(nok ? n : 0) * ldw + gq * 8;
    const bf16x8 zero8 = {};
    constexpr int nsteps = LNK / 32;
    // the first K round's weight fragments and the epilogue operands go out before the LayerNorm prologue: neither
    // depends on it, so their round trips overlap the X row loads
    bf16x8 bw[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
        const int st = w + u * SK_WAVES;
        bw[u] = (st < nsteps && nok) ? *(const bf16x8*)(wrow + st * 32) : zero8;
    }
    SkEpiPre<MT> pre;
    pre.load(e, mb, n0, M, N);
    // SQ: per-stream parameters into LDS (read by the epilogue after the prologue's barrier), and the work the tail
    // would otherwise start with a round trip — this workgroup's cached key rows and FSMN taps — loaded now
    __shared__ int4 sqp[SQ ? 64 : 1];   // slot, cle, tw per stream (M <= 64 rows)
    constexpr int SQC = 2;              // cached-row chunks (16 B) per thread prefetched
    uint4 sqc[SQC];
    float tap[SQ_K];
    if constexpr (SQ) {
        const int D = sq.D, ns = M / sq.Tw;
        if ((int)threadIdx.x < ns) {
            const SPrm p = sq.prm[threadIdx.x];
            sqp[threadIdx.x] = make_int4(p.slot, p.cle, p.tw, 0);
        }
#pragma unroll
        for (int u = 0; u < SQC; ++u) {
            sqc[u] = make_uint4(0, 0, 0, 0);
            const int idx = threadIdx.x + u * 512;
            if (n0 < D || idx >= ns * sq.Tk * 2) continue;
            const int hh = idx & 1, ir = idx >> 1, i = ir / sq.Tk, r = ir - i * sq.Tk;
            const SPrm p = sq.prm[i];
            if (r < p.cle) sqc[u] = *(const uint4*)(sq.cache + ((long long)p.slot * sq.C + r) * 2 * D + n0 - D + 8 * hh);
        }
#pragma unroll
        for (int k = 0; k < SQ_K; ++k) tap[k] = n0 >= 2 * D ? sq.wT[k * D + n0 - 2 * D + (threadIdx.x & 15)] : 0.f;
    }
    for (int rr = w; rr < MT * 16; rr += SK_WAVES) {   // LN of the block's rows (wave w: rows w, w + 8, ...)
        const int row = mb + rr;
        if (row < M) {
            const TIN* xr = X + xmap.off(row);
            float4 v[VPL][2];
#pragma unroll
            for (int i = 0; i < VPL; ++i) ln_load8(xr + i * 512 + lane * 8, v[i][0], v[i][1]);
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < VPL; ++i)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
                    s += (double)v[i][hh].x + (double)v[i][hh].y + (double)v[i][hh].z + (double)v[i][hh].w;
            const double mean = wave_sum_d(s) / LNK;
            double q = 0.0;
#pragma unroll
            for (int i = 0; i < VPL; ++i)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const double a0 = v[i][hh].x - mean, a1 = v[i][hh].y - mean, a2 = v[i][hh].z - mean,
                                 a3 = v[i][hh].w - mean;
                    q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
                }
            const double rstd = 1.0 / sqrt(wave_sum_d(q) / LNK + (double)eps);
#pragma unroll
            for (int i = 0; i < VPL; ++i) {
                const int c = i * 512 + lane * 8;
                const float4 g0 = *(const float4*)(g + c), g1 = *(const float4*)(g + c + 4);
                const float4 b0 = *(const float4*)(bta + c), b1 = *(const float4*)(bta + c + 4);
                float y[8];
                y[0] = (float)((v[i][0].x - mean) * rstd) * g0.x + b0.x;
                y[1] = (float)((v[i][0].y - mean) * rstd) * g0.y + b0.y;
                y[2] = (float)((v[i][0].z - mean) * rstd) * g0.z + b0.z;
                y[3] = (float)((v[i][0].w - mean) * rstd) * g0.w + b0.w;
                y[4] = (float)((v[i][1].x - mean) * rstd) * g1.x + b1.x;
                y[5] = (float)((v[i][1].y - mean) * rstd) * g1.y + b1.y;
                y[6] = (float)((v[i][1].z - mean) * rstd) * g1.z + b1.z;
                y[7] = (float)((v[i][1].w - mean) * rstd) * g1.w + b1.w;
                bf16x8 o;
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = f2bf(y[j]);
                *(bf16x8*)&As[rr][c] = o;
            }
        } else {
#pragma unroll
            for (int i = 0; i < VPL; ++i) *(bf16x8*)&As[rr][i * 512 + lane * 8] = bf16x8{};   // rows beyond M: zeros
        }
    }
    __syncthreads();
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s0 = w; s0 < nsteps; s0 += SK_WAVES * UNR) {
        bf16x8 ba[UNR][MT];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int st = s0 + u * SK_WAVES;
            const bool sok = st < nsteps;
            if (s0 != w) bw[u] = (sok && nok) ? *(const bf16x8*)(wrow + st * 32) : zero8;
#pragma unroll
            for (int t = 0; t < MT; ++t) ba[u][t] = sok ? *(const bf16x8*)&As[t * 16 + r16][st * 32 + gq * 8] : zero8;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ba[u][t], bw[u], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[w][t][(4 * gq + q) * 16 + r16] = acc[t][q];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SkEpiPre<MT>::EPT; ++j) {
        const int idx = threadIdx.x + j * 512;
        const int t = idx >> 8, rc = idx & 255;
        const int row = mb + t * 16 + (rc >> 4), col = n0 + (rc & 15);
        if (idx >= MT * 256 || row >= M || col >= N) continue;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < SK_WAVES; ++ww) v += red[ww][t][rc];
        v *= e.alpha;
        if (e.bias) v += pre.b[j];
        if (e.relu) v = fmaxf(v, 0.f);
        if (e.res0) v += pre.r0[j];
        if (e.res1) v += pre.r1[j];
        const long long ob = e.out_map.off(row);
        if (e.out_dtype == DT_F32) ((float*)e.out)[ob + col] = v;
        else ((bf16*)e.out)[ob + col] = f2bf(v);
        if (e.out2) ((bf16*)e.out2)[e.out2_map.off(row) + col] = f2bf(v);
        if constexpr (SQ) {
            const int i = row / sq.Tw, t = row - i * sq.Tw;
            if (n0 >= sq.D) {   // window K|V row t of stream i -> key row cl + t
                const int4 p = sqp[i];
                if (t < p.z) sq.buf[((long long)i * sq.Tk + p.y + t) * 2 * sq.D + (col - sq.D)] = f2bf(v);
            }
            // the V columns' bf16 values (what QKVb holds), for the FSMN below; As is free once the K loop is done
            if (n0 >= 2 * sq.D) ((float*)&As[0][0])[row * 16 + (rc & 15)] = bf2f(f2bf(v));
        }
    }
    if constexpr (SQ) {
        const int D = sq.D, n = M / sq.Tw;
        if (n0 >= D) {   // the cached rows [0, cl) and the zero rows [cl + tw, Tk) of this workgroup's 16 columns
#pragma unroll
            for (int u = 0; u < SQC + 1; ++u)
                for (int idx = threadIdx.x + u * 512; idx < n * sq.Tk * 2; idx += (u < SQC ? n * sq.Tk * 2 : 512)) {
                    const int hh = idx & 1, ir = idx >> 1, i = ir / sq.Tk, r = ir - i * sq.Tk;
                    const int4 p = sqp[i];
                    if (r >= p.y && r < p.y + p.z) continue;
                    const int c8 = n0 - D + 8 * hh;
                    uint4 val = make_uint4(0, 0, 0, 0);
                    if (u < SQC) val = sqc[u];
                    else if (r < p.y) val = *(const uint4*)(sq.cache + ((long long)p.x * sq.C + r) * 2 * D + c8);
                    *(uint4*)(sq.buf + ((long long)i * sq.Tk + r) * 2 * D + c8) = val;
                }
        }
        if (n0 >= 2 * D) {   // FSMN over each stream's tw window rows, as fsmn_win_body<11, bf16, 5> (lens = tw)
            __syncthreads();
            const float* vs = (const float*)&As[0][0];
            for (int idx = threadIdx.x; idx < M * 16; idx += 512) {
                const int row = idx >> 4, cc = idx & 15, c = n0 - 2 * D + cc;
                const int i = row / sq.Tw, t = row - i * sq.Tw;
                const int L = min(sqp[i].z, sq.Tw);
                float y = 0.f;
                if (t < L) {
                    float acc = 0.f;
#pragma unroll
                    for (int k = 0; k < SQ_K; ++k) {
                        const int tt = t - SQ_LEFT + k;
                        const float x = (tt >= 0 && tt < L) ? vs[(i * sq.Tw + tt) * 16 + cc] : 0.f;
                        acc = fmaf(tap[k], x, acc);
                    }
                    y = acc + vs[row * 16 + cc];
                }
                sq.fout[(long long)row * D + c] = f2bf(y);
            }
        }
    }
}

}  // namespace

// LN-fused form: X f32 rows of K = 512 (16-B aligned), LN(X) g + b as the bf16 A operand; M <= 64 per row block (any M,
// grid.y = ceil(M / 64)); the same epilogue contract as pfm_gemm_skinny
bool pfm_gemm_skinny_ln_ok(const float* X, RowMap xmap, const void* W, long long ldw, int M, int N, int K,
                           const GemmEpi& e) {
    if (K != 512 || M < 1 || M > 64 || ldw % 8 != 0 || xmap.ld % 4 != 0) return false;
    if (xmap.rows_per_seg > 0 && xmap.seg_stride % 4 != 0) return false;
    if (((uintptr_t)X | (uintptr_t)W) % 16 != 0) return false;
    if (!e.out || e.amax_val) return false;
    return pfm_knobs().gemm_skinny && pfm_knobs().gemm_cfg == 0;
}

hipError_t pfm_gemm_skinny_ln(const float* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                              long long ldw, int M, int N, const GemmEpi& e, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((N + 15) / 16, (M + 63) / 64), block(512);
    const bf16* wt = (const bf16*)W;
    switch ((M + 15) / 16) {
        case 1: hipLaunchKernelGGL((gemm_skinny_ln_kernel<1, 1, float>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, SkQkv{}); break;
        case 2: hipLaunchKernelGGL((gemm_skinny_ln_kernel<2, 1, float>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, SkQkv{}); break;
        case 3: hipLaunchKernelGGL((gemm_skinny_ln_kernel<3, 1, float>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, SkQkv{}); break;
        case 4: hipLaunchKernelGGL((gemm_skinny_ln_kernel<4, 1, float>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, SkQkv{}); break;
        default: return hipErrorInvalidValue;
    }
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// ... and for bf16 rows of K = 2048 (the decoder FFN's hidden before w2, streaming: <= 16 token rows)
bool pfm_gemm_skinny_ln2048_ok(const bf16* X, RowMap xmap, const void* W, long long ldw, int M, int N, int K,
                               const GemmEpi& e) {
    if (K != 2048 || M < 1 || M > 16 || ldw % 8 != 0 || xmap.ld % 8 != 0) return false;
    if (xmap.rows_per_seg > 0 && xmap.seg_stride % 8 != 0) return false;
    if (((uintptr_t)X | (uintptr_t)W) % 16 != 0) return false;
    if (!e.out || e.amax_val) return false;
    return pfm_knobs().gemm_skinny && pfm_knobs().gemm_cfg == 0;
}
hipError_t pfm_gemm_skinny_ln2048(const bf16* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                                  long long ldw, int M, int N, const GemmEpi& e, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (M > 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_skinny_ln_kernel<1, 4, bf16>), dim3((N + 15) / 16, 1), dim3(512), 0, st, X, xmap, g, b, eps,
                       (const bf16*)W, ldw, M, N, e, SkQkv{});
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// Shapes this kernel takes: bf16 operands, M <= 64 or few 128x256 tiles, K % 32 == 0, 16-B aligned rows, and an epilogue
// without the fused argmax / LayerNorm-statistics features of the tiled kernels.
bool pfm_gemm_skinny_ok(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                        const GemmEpi& e) {
    if (M < 1 || K % 32 != 0 || ldw % 8 != 0 || amap.ld % 8 != 0) return false;
    if (amap.rows_per_seg > 0 && amap.seg_stride % 8 != 0) return false;
    if (((uintptr_t)A | (uintptr_t)W) % 16 != 0) return false;
    if (!e.out || e.amax_val) return false;
    if (!pfm_knobs().gemm_skinny) return false;    // PFM_GEMM_SKINNY=0: tiled kernels for every M (A/B)
    if (pfm_knobs().gemm_cfg != 0) return false;   // a forced tile configuration wins (tile-config tests / A/B)
    // beyond 64 rows: only while the tiled kernels would launch fewer than ~64 128x256 tiles (the
    // multi-stream chunk batches, M = 15 x streams), i.e. where they leave most CUs idle
    return M <= 64 || (long long)((M + 127) / 128) * ((N + 255) / 256) < 64;
}

hipError_t pfm_gemm_skinny(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                           const GemmEpi& e, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const dim3 grid((N + 15) / 16, (M + 63) / 64), block(512);
    const bf16* a = (const bf16*)A;
    const bf16* wt = (const bf16*)W;
    switch (M > 64 ? 4 : (M + 15) / 16) {
        case 1:
            if (K > 32 * SK_WAVES * SK_UNROLL) hipLaunchKernelGGL((gemm_skinny_kernel<1, SK_UNROLL_WIDE>), grid, block, 0, st, a, amap, wt, ldw, M, N, K, e);
            else hipLaunchKernelGGL(gemm_skinny_kernel<1>, grid, block, 0, st, a, amap, wt, ldw, M, N, K, e);
            break;
        case 2:
            if (K > 32 * SK_WAVES * SK_UNROLL) hipLaunchKernelGGL((gemm_skinny_kernel<2, SK_UNROLL_WIDE>), grid, block, 0, st, a, amap, wt, ldw, M, N, K, e);
            else hipLaunchKernelGGL(gemm_skinny_kernel<2>, grid, block, 0, st, a, amap, wt, ldw, M, N, K, e);
            break;
        case 3: hipLaunchKernelGGL(gemm_skinny_kernel<3>, grid, block, 0, st, a, amap, wt, ldw, M, N, K, e); break;
        case 4: hipLaunchKernelGGL(gemm_skinny_kernel<4>, grid, block, 0, st, a, amap, wt, ldw, M, N, K, e); break;
        default: return hipErrorInvalidValue;
    }
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// Streaming encoder layer: LN1 -> QKV as above (M <= 64 rows = n streams x Tw window rows, K = 512, N = 3d, d % 16 == 0,
// bf16 q|k|v rows) that also writes the attention's key buffer [n][Tk][2d] from this layer's K/V cache and the window's
// FSMN memory block (11 taps, left 5, lens = tw): pfm_kv_gather_fsmn's two outputs, bit-identical, without its launch.
// hipErrorNotSupported (nothing launched) for any other shape.
hipError_t pfm_gemm_skinny_ln_qkv(const float* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                                  long long ldw, int M, int N, const GemmEpi& e, const SPrm* prm, int n, int Tw,
                                  const bf16* cache, int C, bf16* buf, int Tk, const float* wT, bf16* fout, int D,
                                  hipStream_t st) {
    if (!pfm_gemm_skinny_ln_ok(X, xmap, W, ldw, M, N, 512, e)) return hipErrorNotSupported;
    if (n < 1 || Tw < 1 || M != n * Tw || N != 3 * D || D % 16 || e.out_dtype != DT_BF16 || Tk < Tw)
        return hipErrorNotSupported;
    if (((uintptr_t)cache | (uintptr_t)buf) % 16 != 0 || !prm || !wT || !fout) return hipErrorNotSupported;
    const SkQkv sq{prm, cache, buf, wT, fout, Tw, Tk, C, D};
    const dim3 grid(N / 16, 1), block(512);
    const bf16* wt = (const bf16*)W;
    switch ((M + 15) / 16) {
        case 1: hipLaunchKernelGGL((gemm_skinny_ln_kernel<1, 1, float, true>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, sq); break;
        case 2: hipLaunchKernelGGL((gemm_skinny_ln_kernel<2, 1, float, true>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, sq); break;
        case 3: hipLaunchKernelGGL((gemm_skinny_ln_kernel<3, 1, float, true>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, sq); break;
        case 4: hipLaunchKernelGGL((gemm_skinny_ln_kernel<4, 1, float, true>), grid, block, 0, st, X, xmap, g, b, eps, wt, ldw, M, N, e, sq); break;
        default: return hipErrorNotSupported;
    }
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
