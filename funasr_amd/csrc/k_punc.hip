// CT-Transformer punctuation kernels (funasr/models/ct_transformer/model.py:81-93):
// the word-embedding input of the SANMEncoder, attention for its 32-wide heads, and the punctuation head.
//
//   punc_embed_kernel   X[b,t] = embed[ids[b,t]] * sqrt(d) + PE[t]   (Embedding -> SANMEncoder input
//                       scaling + SinusoidalPositionEncoder, sanm/encoder.py:378-379; the product is
//                       rounded before the add, as torch evaluates it)
//   attn_small_kernel   softmax(q k^T * d_k^-0.5, -inf on keys >= klen) v for head widths 32 / 64 (the
//                       Paraformer kernels in k_attn.hip are built for d_k = 128): 16 lanes per query
//                       row, each with an online softmax in f32 over every 16th key of 64-key K/V tiles
//                       staged in LDS, merged by shuffles. Sequences are mini-sentences (<= ~220 words), so
//                       the kernel is latency-bound (serial key chains), not MFMA-bound
//   punc_head_kernel    logits = after_norm(x) . W^T + b over the punctuation classes, argmax (first index
//                       on ties, topk(1)); one wave per word, lanes over the d columns
#include <math.h>

#include "pfm_common.h"

namespace {

__global__ __launch_bounds__(256) void punc_embed_kernel(const int* __restrict__ ids, const int* __restrict__ lens,
                                                         int T, const float* __restrict__ embed, int n_embed,
                                                         const float* __restrict__ pe, int D, float scale,
                                                         float* __restrict__ X) {
    const int row = blockIdx.x, b = row / T, t = row % T;
    int id = t < lens[b] ? ids[row] : 0;
    id = id < 0 ? 0 : (id >= n_embed ? n_embed - 1 : id);
    const float4* er = (const float4*)(embed + (long long)id * D);
    const float4* pr = (const float4*)(pe + (long long)t * D);
    float4* xr = (float4*)(X + (long long)row * D);
    for (int c = threadIdx.x; c < D / 4; c += 256) {
        const float4 e = er[c], p = pr[c];
        xr[c] = make_float4(__fadd_rn(__fmul_rn(e.x, scale), p.x), __fadd_rn(__fmul_rn(e.y, scale), p.y),
                            __fadd_rn(__fmul_rn(e.z, scale), p.z), __fadd_rn(__fmul_rn(e.w, scale), p.w));
    }
}

template <typename T> __device__ __forceinline__ float ld1(const T* p);
template <> __device__ __forceinline__ float ld1<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld1<bf16>(const bf16* p) { return bf2f(*p); }

constexpr int AS_KT = 64;   // keys per LDS tile
constexpr int AS_QR = 16;   // query rows per workgroup
constexpr int AS_KL = 16;   // key lanes per query row: a row's keys are split over 16 lanes, merged at the end

// Workgroup = 16 query rows x 16 key lanes (256 threads; a wave holds 4 rows). Lane kl of a row runs an online
// softmax over keys kl, kl + 16, kl + 32, ... of each 64-key LDS tile: its four scores per tile are independent
// FMA chains, and the running maximum is rescaled once per tile, not per key. The 16 partial (max, sum, acc) of
// a row are merged with xor shuffles inside the 16-lane group. K and V rows sit in LDS with a one-float pad, so
// the 16 rows read at once fall in distinct banks.
template <typename T, int DKS>
__global__ __launch_bounds__(256) void attn_small_kernel(const T* __restrict__ q, RowMap qmap, const T* __restrict__ k,
                                                         RowMap kmap, const T* __restrict__ v, RowMap vmap,
                                                         float* __restrict__ o, bf16* __restrict__ o2, long long ldo,
                                                         const int* __restrict__ klen, int Tq, int Tk, float scale) {
    constexpr int LD = DKS + 1;
    __shared__ float ks[AS_KT * LD], vs[AS_KT * LD];
    const int b = blockIdx.z, h = blockIdx.y;
    const int qi = threadIdx.x / AS_KL, kl = threadIdx.x % AS_KL;
    const int t = blockIdx.x * AS_QR + qi;
    const bool qok = t < Tq;
    const int nk = min(klen[b], Tk);
    float qv[DKS], acc[DKS];
    const T* qr = q + qmap.off((long long)b * Tq + (qok ? t : 0)) + h * DKS;
#pragma unroll
    for (int c = 0; c < DKS; ++c) {
        qv[c] = ld1(qr + c) * scale;   // q * d_k^-0.5 before the product (attention.py:251)
        acc[c] = 0.f;
    }
    float mx = -INFINITY, den = 0.f;
    for (int k0 = 0; k0 < nk; k0 += AS_KT) {
        const int kn = min(AS_KT, nk - k0);
        __syncthreads();
        for (int i = threadIdx.x; i < AS_KT * DKS; i += 256) {   // rows >= kn zero: p = 0 must not meet a NaN
            const int r = i / DKS, c = i % DKS;
            const long long m = (long long)b * Tk + k0 + r;
            ks[r * LD + c] = r < kn ? ld1(k + kmap.off(m) + h * DKS + c) : 0.f;
            vs[r * LD + c] = r < kn ? ld1(v + vmap.off(m) + h * DKS + c) : 0.f;
        }
        __syncthreads();
        float s[AS_KT / AS_KL];
#pragma unroll
        for (int j = 0; j < AS_KT / AS_KL; ++j) s[j] = 0.f;
#pragma unroll
        for (int c = 0; c < DKS; ++c)
#pragma unroll
            for (int j = 0; j < AS_KT / AS_KL; ++j) s[j] = fmaf(qv[c], ks[(kl + j * AS_KL) * LD + c], s[j]);
        float tm = -INFINITY;
#pragma unroll
        for (int j = 0; j < AS_KT / AS_KL; ++j) {
            if (kl + j * AS_KL >= kn) s[j] = -INFINITY;   // keys >= klen: masked (attention.py:254-262)
            tm = fmaxf(tm, s[j]);
        }
        if (tm > mx) {   // rescale the running sums to the new maximum (exp(-inf) = 0 on the first tile)
            const float f = expf(mx - tm);
            den *= f;
#pragma unroll
            for (int c = 0; c < DKS; ++c) acc[c] *= f;
            mx = tm;
        }
#pragma unroll
        for (int j = 0; j < AS_KT / AS_KL; ++j) {
            const float p = kl + j * AS_KL < kn ? expf(s[j] - mx) : 0.f;
            den += p;
#pragma unroll
            for (int c = 0; c < DKS; ++c) acc[c] = fmaf(p, vs[(kl + j * AS_KL) * LD + c], acc[c]);
        }
    }
    // merge the 16 key lanes of the row: (m, l, a) (+) (m', l', a') = (M, l e^(m-M) + l' e^(m'-M), ...)
#pragma unroll
    for (int off = AS_KL / 2; off >= 1; off >>= 1) {
        const float mo = __shfl_xor(mx, off, 64), dno = __shfl_xor(den, off, 64);
        const float mn = fmaxf(mx, mo);
        const float f = mx == -INFINITY ? 0.f : expf(mx - mn);   // a lane without keys carries nothing
        const float fo = mo == -INFINITY ? 0.f : expf(mo - mn);
        den = den * f + dno * fo;
#pragma unroll
        for (int c = 0; c < DKS; ++c) acc[c] = acc[c] * f + __shfl_xor(acc[c], off, 64) * fo;
        mx = mn;
    }
    if (!qok || kl) return;
    const float inv = nk > 0 ? 1.f / den : 0.f;   // no valid key: the reference's masked_fill(0) row
    const long long ob = ((long long)b * Tq + t) * ldo + h * DKS;
#pragma unroll
    for (int c = 0; c < DKS; ++c) {
        const float y = acc[c] * inv;
        if (o) o[ob + c] = y;
        if (o2) o2[ob + c] = f2bf(y);
    }
}

__global__ __launch_bounds__(256) void punc_head_kernel(const float* __restrict__ x, int M, int T,
                                                        const int* __restrict__ lens, const float* __restrict__ W,
                                                        const float* __restrict__ bias, int NP, int D,
                                                        int* __restrict__ punc, float* __restrict__ logits) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int b = row / T, t = row % T;
    const float* xr = x + (long long)row * D;
    float best = -INFINITY;
    int bi = 0;
    for (int c = 0; c < NP; ++c) {
        float s = 0.f;
        for (int j = lane; j < D; j += 64) s = fmaf(xr[j], W[(long long)c * D + j], s);
        s = wave_sum(s) + bias[c];
        if (logits && lane == 0) logits[(long long)row * NP + c] = s;
        if (s > best) { best = s; bi = c; }   // strict: the first index wins ties
    }
    if (lane == 0) punc[row] = t < lens[b] ? bi : -1;
}

}  // namespace

hipError_t pfm_punc_embed(const int* ids, const int* lens, int B, int T, const float* embed, int n_embed,
                          const float* pe, int D, float scale, float* X, hipStream_t st) {
    if (B <= 0 || T <= 0) return hipSuccess;
    if (D % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(punc_embed_kernel, dim3(B * T), dim3(256), 0, st, ids, lens, T, embed, n_embed, pe, D, scale, X);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// Attention for head widths other than the k_attn.hip kernels' 128 (o: f32 rows, o2: bf16 rows, both ldo).
hipError_t pfm_attention_small(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                               RowMap vmap, float* o, void* o2, long long ldo, const int* klen, int B, int Tq, int Tk,
                               int heads, int dk, float scale, hipStream_t st) {
    if (B <= 0 || Tq <= 0) return hipSuccess;
    const dim3 grid((Tq + AS_QR - 1) / AS_QR, heads, B), block(256);
#define PFM_AS_LAUNCH(TT, DD)                                                                                 \
    hipLaunchKernelGGL((attn_small_kernel<TT, DD>), grid, block, 0, st, (const TT*)q, qmap, (const TT*)k, kmap, \
                       (const TT*)v, vmap, o, (bf16*)o2, ldo, klen, Tq, Tk, scale)
    if (dtype == DT_F32 && dk == 32) PFM_AS_LAUNCH(float, 32);
    else if (dtype == DT_F32 && dk == 64) PFM_AS_LAUNCH(float, 64);
    else if (dtype == DT_BF16 && dk == 32) PFM_AS_LAUNCH(bf16, 32);
    else if (dtype == DT_BF16 && dk == 64) PFM_AS_LAUNCH(bf16, 64);
    else return hipErrorInvalidValue;
#undef PFM_AS_LAUNCH
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_punc_head(const float* x, int B, int T, const int* lens, const float* W, const float* bias, int NP,
                         int D, int* punc, float* logits, hipStream_t st) {
    const int M = B * T;
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(punc_head_kernel, dim3((M + 3) / 4), dim3(256), 0, st, x, M, T, lens, W, bias, NP, D, punc,
                       logits);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
