// Streaming Paraformer chunk kernels (paraformer_streaming/model.py:468-554): the per-stream caches of
// SANMEncoderChunkOpt / CifPredictorV2.forward_chunk / ParaformerSANMDecoder.forward_chunk live in HBM,
// indexed by slot, and every kernel here advances a batch of n streams by one chunk.
#include "pfm_common.h"
#include "pfm_stream.h"

namespace {

// ------------------------------------------------------------------------------------------
// Encoder input window (scama/encoder.py:456-473 + embedding.py:436-444):
//   non-tail: x = [fcache(C0 rows) ; feats * sqrt(d) + PE(start + 1 ..)]         tw = C0 + nfeat
//   tail:     x = fcache * sqrt(d)  (forward_chunk scales cache["feats"] in place)  tw = C0
// rows t >= tw are zero. One 256-thread block per (stream, row), float4 columns (I % 4 == 0).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void stream_window_kernel(const float* __restrict__ feats, int Tn,
                                                            const SPrm* __restrict__ prm, const float* __restrict__ fcache,
                                                            const float* __restrict__ pe, int I, int C0, int Tw,
                                                            float scale, float* __restrict__ x) {
    const int i = blockIdx.y, t = blockIdx.x;
    const SPrm p = prm[i];
    float4* xr = (float4*)(x + ((long long)i * Tw + t) * I);
    const bool tail = p.nfeat == 0;
    for (int c = threadIdx.x; c < I / 4; c += 256) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t < p.tw) {
            if (t < C0) {
                v = ((const float4*)(fcache + ((long long)p.slot * C0 + t) * I))[c];
                if (tail) v = make_float4(__fmul_rn(v.x, scale), __fmul_rn(v.y, scale), __fmul_rn(v.z, scale),
                                          __fmul_rn(v.w, scale));
            } else {
                const float4 f = ((const float4*)(feats + ((long long)i * Tn + (t - C0)) * I))[c];
                const float4 e = ((const float4*)(pe + (long long)(p.start + t - C0) * I))[c];
                v = make_float4(__fadd_rn(__fmul_rn(f.x, scale), e.x), __fadd_rn(__fmul_rn(f.y, scale), e.y),
                                __fadd_rn(__fmul_rn(f.z, scale), e.z), __fadd_rn(__fmul_rn(f.w, scale), e.w));
            }
        }
        xr[c] = v;
    }
}

// cache["feats"] = window[-C0:] for non-tail streams (encoder.py:448-454)
__global__ __launch_bounds__(256) void stream_fcache_kernel(const float* __restrict__ x, const SPrm* __restrict__ prm,
                                                            int I, int C0, int Tw, float* __restrict__ fcache) {
    const int i = blockIdx.y, r = blockIdx.x;
    const SPrm p = prm[i];
    if (p.nfeat == 0) return;
    const float4* src = (const float4*)(x + ((long long)i * Tw + p.tw - C0 + r) * I);
    float4* dst = (float4*)(fcache + ((long long)p.slot * C0 + r) * I);
    for (int c = threadIdx.x; c < I / 4; c += 256) dst[c] = src[c];
}

// Attention keys of one layer (kv_gather_row, pfm_stream.h): one block per (stream, key row)
template <typename T>
__global__ __launch_bounds__(128) void kv_gather_kernel(const T* __restrict__ cache, long long cache_ls, int C,
                                                        const SPrm* __restrict__ prm, int dec, const T* __restrict__ src,
                                                        long long src_ls, long long src_ld, int Tw, T* __restrict__ buf,
                                                        long long buf_ls, int Tk, int W) {
    const int i = blockIdx.y, r = blockIdx.x, l = blockIdx.z;   // grid.z: layers (strides in elements)
    kv_gather_row(cache + l * cache_ls, C, prm[i], dec, src + l * src_ls, src_ld, Tw, buf + l * buf_ls, Tk, W, i, r,
                  (int)threadIdx.x, 128);
}

// New cache = the last min(C, cl + tw - drop) rows of buf[i][0 .. cl + tw - drop): drop = chunk_size[2]
// look-ahead rows for the encoder (attention.py:329-334), 0 for the decoder (:733-737). Decoder caches
// only move for streams whose decoder ran (ntok > 0, model.py:494-495).
template <typename T>
__global__ __launch_bounds__(128) void kv_retain_kernel(const T* __restrict__ buf, int Tk, const SPrm* __restrict__ prm,
                                                        int dec, int drop, const int* __restrict__ ntok,
                                                        T* __restrict__ cache, int C, int W) {
    const int i = blockIdx.y, j = blockIdx.x;
    const SPrm p = prm[i];
    if (dec && ntok[i] < 1) return;
    const int len0 = (dec ? p.cld : p.cle) + p.tw - drop;
    const int ncl = min(C, len0);
    if (j >= ncl) return;
    constexpr int V = 16 / sizeof(T);
    const uint4* s = (const uint4*)(buf + ((long long)i * Tk + (len0 - ncl + j)) * W);
    uint4* d = (uint4*)(cache + ((long long)p.slot * C + j) * W);
    for (int c = threadIdx.x; c < W / V; c += 128) d[c] = s[c];
}

// Zero the window rows t >= tw of the after_norm output in its [n][Tw+2][D] layout (row 0 / Tw+1 are
// the conv padding, cleared by the host): the predictor's conv1d sees exactly the stream's frames.
__global__ __launch_bounds__(256) void stream_mask_rows_kernel(float* __restrict__ encp, bf16* __restrict__ encpb,
                                                               const SPrm* __restrict__ prm, int Tw, int D) {
    const int i = blockIdx.y, t = blockIdx.x;
    if (t < prm[i].tw) return;
    const long long row = (long long)i * (Tw + 2) + t + 1;
    for (int c = threadIdx.x; c < D; c += 256) {
        encp[row * D + c] = 0.f;
        if (encpb) encpb[row * D + c] = f2bf(0.f);
    }
}

// ------------------------------------------------------------------------------------------
// CifPredictorV2.forward_chunk (cif_predictor.py:255-344) for one stream per block:
//   alpha[t] = relu(sigmoid(w . hc[t] + b) * smooth - noise), t < tw; 0 for t < cs0 and, unless final,
//   for t >= cs0 + cs1; sequence = [carry (cif_hidden, cif_alphas)] ++ frames ++ [tail (0, 0.45) if final];
//   the reference's scalar integrate-and-fire loop in f32 (no contraction), fired frames -> emb;
//   carry = (integrate, frames / integrate) (or frames when integrate <= 0).
// ------------------------------------------------------------------------------------------
constexpr int CIF_CH = 4;   // channels per thread (D <= 1024)
__global__ __launch_bounds__(256) void cif_chunk_kernel(const float* __restrict__ hc, const float* __restrict__ wout,
                                                        const float* __restrict__ bout, const float* __restrict__ encp,
                                                        const SPrm* __restrict__ prm, int Tw, int D, int cs0, int keep,
                                                        float smooth, float noise, float tail, float thr,
                                                        float* __restrict__ chid, float* __restrict__ calpha,
                                                        float* __restrict__ emb, int Lcap, int* __restrict__ ntok,
                                                        float* __restrict__ alphas_out, int stage) {
    __shared__ float al[64];
    extern __shared__ __attribute__((aligned(16))) float ers[];   // staged window rows [tw][D] (stage != 0)
    const int i = blockIdx.x;
    const SPrm p = prm[i];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the integrate loop below is sequential over the rows: with the rows read from global memory inside it, every row
    // was a dependent round trip; they are staged into LDS up front (one parallel copy), as are 4 rows per wave of the
    // alpha dot products (same per-row summation order)
    const float* erow0 = encp + ((long long)i * (Tw + 2) + 1) * D;   // padded rows 1 .. tw == frames 0 .. tw - 1
    if (stage)
        for (int q = threadIdx.x; q < p.tw * D / 4; q += 256) ((float4*)ers)[q] = ((const float4*)erow0)[q];
    constexpr int RW = 4;
    for (int t0 = wv; t0 < p.tw; t0 += 4 * RW) {
        double s[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) s[r] = 0.0;
        for (int c = lane; c < D; c += 64) {
            const double wc = (double)wout[c];
#pragma unroll
            for (int r = 0; r < RW; ++r) {
                const int t = t0 + 4 * r;
                if (t < p.tw) s[r] += (double)hc[((long long)i * Tw + t) * D + c] * wc;
            }
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int t = t0 + 4 * r;
            if (t >= p.tw) break;
            const double sr = wave_sum_d(s[r]);
            if (lane == 0) {
                const float z = (float)(sr + (double)bout[0]);
                const float sg = (float)(1.0 / (1.0 + exp(-(double)z)));
                float a = fmaxf(sg * smooth - noise, 0.f);
                if (t < cs0 || (!p.fin && t >= keep)) a = 0.f;
                al[t] = a;
                if (alphas_out) alphas_out[(long long)i * Tw + t] = a;
            }
        }
    }
    __syncthreads();
    float fr[CIF_CH], cache_h[CIF_CH];
    const float* hrow = chid + (long long)p.slot * D;
#pragma unroll
    for (int k = 0; k < CIF_CH; ++k) {
        const int c = threadIdx.x + k * 256;
        fr[k] = 0.f;
        cache_h[k] = c < D ? hrow[c] : 0.f;
    }
    float integ = 0.f;
    int nf = 0;
    const int nseq = 1 + p.tw + (p.fin ? 1 : 0);
    for (int s = 0; s < nseq; ++s) {
        float a;
        float hv[CIF_CH];
        if (s == 0) {
            a = calpha[p.slot];
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) hv[k] = cache_h[k];
        } else if (s <= p.tw) {
            a = al[s - 1];
            const float* er = (stage ? (const float*)ers : erow0) + (long long)(s - 1) * D;   // frame s - 1
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) {
                const int c = threadIdx.x + k * 256;
                hv[k] = c < D ? er[c] : 0.f;
            }
        } else {
            a = tail;
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) hv[k] = 0.f;
        }
        if (__fadd_rn(a, integ) < thr) {
            integ = __fadd_rn(integ, a);
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) fr[k] = __fadd_rn(fr[k], __fmul_rn(a, hv[k]));
        } else {
            const float r = __fsub_rn(thr, integ);
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) {
                fr[k] = __fadd_rn(fr[k], __fmul_rn(r, hv[k]));
                const int c = threadIdx.x + k * 256;
                if (c < D && nf < Lcap) emb[((long long)i * Lcap + nf) * D + c] = fr[k];
            }
            ++nf;
            integ = __fadd_rn(integ, a);
            integ = __fsub_rn(integ, thr);
#pragma unroll
            for (int k = 0; k < CIF_CH; ++k) fr[k] = __fmul_rn(integ, hv[k]);
        }
    }
    float* hw = chid + (long long)p.slot * D;
#pragma unroll
    for (int k = 0; k < CIF_CH; ++k) {
        const int c = threadIdx.x + k * 256;
        if (c < D) {
            hw[c] = integ > 0.f ? __fdiv_rn(fr[k], integ) : fr[k];
            for (int j = nf; j < Lcap; ++j) emb[((long long)i * Lcap + j) * D + c] = 0.f;
        }
    }
    if (threadIdx.x == 0) {
        calpha[p.slot] = integ;
        ntok[i] = min(nf, Lcap);
    }
}

// ------------------------------------------------------------------------------------------
// Decoder FSMN with its chunk cache (sanm/attention.py:499-547, sanm_shfit 5 -> left pad K-1): causal over
// the stream's token history, whose last K-1 rows are the cache (zeros before the first chunk):
//   x[t] += sum_k w[k] hist[t + k]  +  v[t],   hist = [state (K-1 rows) ; v[0 .. ntok)]
// state <- last K-1 rows of hist when the decoder ran (ntok > 0). Thread per (stream, channel).
// ------------------------------------------------------------------------------------------
template <typename TIN, int K>
__global__ __launch_bounds__(256) void dec_fsmn_stream_kernel(const TIN* __restrict__ v, const float* __restrict__ wT,
                                                              float* __restrict__ state, const SPrm* __restrict__ prm,
                                                              const int* __restrict__ ntok, int L, int D,
                                                              float* __restrict__ x) {
    const int i = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= D) return;
    const int nt = min(ntok[i], L);
    if (nt < 1) return;
    const SPrm p = prm[i];
    float* st = state + (long long)p.slot * (K - 1) * D + c;
    float hist[K], w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = wT[(long long)k * D + c];
#pragma unroll
    for (int k = 0; k < K - 1; ++k) hist[k] = st[(long long)k * D];
    for (int t = 0; t < nt; ++t) {
        const long long row = (long long)i * L + t;
        const float vt = to_f<TIN>(v[row * D + c]);
        hist[K - 1] = vt;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fmaf(w[k], hist[k], acc);
        x[row * D + c] = x[row * D + c] + (acc + vt);
#pragma unroll
        for (int k = 0; k < K - 1; ++k) hist[k] = hist[k + 1];
    }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) st[(long long)k * D] = hist[k];
}

// The same FSMN with the decoder layer's norm2 in front (fast mode): v = bf16(LN(t) g + b) of the FFN output rows t
// (f32, [n][L][512]), the arithmetic of layernorm_v8_kernel<1, R> (f64 sums in its order, f32 affine, bf16 out), then
// dec_fsmn_stream_kernel<bf16> on those rows: one 512-thread block per stream, the normalised rows in LDS (one wave per
// row), a thread per channel for the causal FSMN. Replaces a LayerNorm launch and its bf16 round trip per layer.
template <int K>
__global__ __launch_bounds__(512) void dec_fsmn_ln_stream_kernel(const float* __restrict__ tin, const float* __restrict__ g,
                                                                 const float* __restrict__ bta, float eps,
                                                                 const float* __restrict__ wT, float* __restrict__ state,
                                                                 const SPrm* __restrict__ prm, const int* __restrict__ ntok,
                                                                 int L, float* __restrict__ x) {
    constexpr int D = 512;
    extern __shared__ __attribute__((aligned(16))) bf16 vn[];   // [nt][512]
    const int i = blockIdx.x;
    const int nt = min(ntok[i], L);
    if (nt < 1) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    {
        const int c = lane * 8;
        const float4 g0 = *(const float4*)(g + c), g1 = *(const float4*)(g + c + 4);
        const float4 b0 = *(const float4*)(bta + c), b1 = *(const float4*)(bta + c + 4);
        for (int t = w; t < nt; t += 8) {
            const float* xr = tin + ((long long)i * L + t) * D;
            const float4 v0 = *(const float4*)(xr + c), v1 = *(const float4*)(xr + c + 4);
            double s = 0.0;
            s += (double)v0.x + (double)v0.y + (double)v0.z + (double)v0.w;
            s += (double)v1.x + (double)v1.y + (double)v1.z + (double)v1.w;
            const double mean = wave_sum_d(s) / D;
            double q = 0.0;
            {
                const double a0 = v0.x - mean, a1 = v0.y - mean, a2 = v0.z - mean, a3 = v0.w - mean;
                q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
            }
            {
                const double a0 = v1.x - mean, a1 = v1.y - mean, a2 = v1.z - mean, a3 = v1.w - mean;
                q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
            }
            const double rstd = 1.0 / sqrt(wave_sum_d(q) / D + (double)eps);
            bf16x8 o;
            o[0] = f2bf((float)((v0.x - mean) * rstd) * g0.x + b0.x);
            o[1] = f2bf((float)((v0.y - mean) * rstd) * g0.y + b0.y);
            o[2] = f2bf((float)((v0.z - mean) * rstd) * g0.z + b0.z);
            o[3] = f2bf((float)((v0.w - mean) * rstd) * g0.w + b0.w);
            o[4] = f2bf((float)((v1.x - mean) * rstd) * g1.x + b1.x);
            o[5] = f2bf((float)((v1.y - mean) * rstd) * g1.y + b1.y);
            o[6] = f2bf((float)((v1.z - mean) * rstd) * g1.z + b1.z);
            o[7] = f2bf((float)((v1.w - mean) * rstd) * g1.w + b1.w);
            *(bf16x8*)&vn[t * D + c] = o;
        }
    }
    __syncthreads();
    const int c = threadIdx.x;
    const SPrm p = prm[i];
    float* st = state + (long long)p.slot * (K - 1) * D + c;
    float hist[K], wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = wT[(long long)k * D + c];
#pragma unroll
    for (int k = 0; k < K - 1; ++k) hist[k] = st[(long long)k * D];
    for (int t = 0; t < nt; ++t) {
        const long long row = (long long)i * L + t;
        const float vt = bf2f(vn[t * D + c]);
        hist[K - 1] = vt;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fmaf(wk[k], hist[k], acc);
        x[row * D + c] = x[row * D + c] + (acc + vt);
#pragma unroll
        for (int k = 0; k < K - 1; ++k) hist[k] = hist[k + 1];
    }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) st[(long long)k * D] = hist[k];
}

}  // namespace

hipError_t pfm_dec_fsmn_ln_stream(const float* tin, const float* g, const float* b, float eps, const float* wT, int K,
                                  float* state, const SPrm* prm, const int* ntok, int n, int L, int D, float* x,
                                  hipStream_t st) {
    if (n <= 0 || L <= 0) return hipSuccess;
    if (K != 11 || D != 512 || L > 64 || ((uintptr_t)tin % 16) || ((uintptr_t)g % 16) || ((uintptr_t)b % 16))
        return hipErrorNotSupported;
    hipLaunchKernelGGL((dec_fsmn_ln_stream_kernel<11>), dim3(n), dim3(512), (size_t)L * D * 2, st, tin, g, b, eps, wT,
                       state, prm, ntok, L, x);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_stream_window(const float* feats, int Tn, const SPrm* prm, int n, const float* fcache, const float* pe,
                             int I, int C0, int Tw, float scale, float* x, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (I % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(stream_window_kernel, dim3(Tw, n), dim3(256), 0, st, feats, Tn, prm, fcache, pe, I, C0, Tw,
                       scale, x);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_stream_fcache(const float* x, const SPrm* prm, int n, int I, int C0, int Tw, float* fcache,
                             hipStream_t st) {
    if (n <= 0 || C0 <= 0) return hipSuccess;
    hipLaunchKernelGGL(stream_fcache_kernel, dim3(C0, n), dim3(256), 0, st, x, prm, I, C0, Tw, fcache);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_kv_gather_layers(int dtype, const void* cache, long long cache_ls, int C, const SPrm* prm, int n, int dec,
                                const void* src, long long src_ls, long long src_ld, int Tw, void* buf, long long buf_ls,
                                int Tk, int W, int layers, hipStream_t st) {
    if (n <= 0 || Tk <= 0 || layers <= 0) return hipSuccess;
    const int es = dtype == DT_F32 ? 4 : 2;
    if ((W * es) % 16 || (src_ld * es) % 16 || ((uintptr_t)src % 16) || ((uintptr_t)buf % 16) ||
        ((uintptr_t)cache % 16) || (cache_ls * es) % 16 || (src_ls * es) % 16 || (buf_ls * es) % 16)
        return hipErrorInvalidValue;
    const dim3 grid(Tk, n, layers);
    if (dtype == DT_F32)
        hipLaunchKernelGGL(kv_gather_kernel<float>, grid, dim3(128), 0, st, (const float*)cache, cache_ls, C, prm, dec,
                           (const float*)src, src_ls, src_ld, Tw, (float*)buf, buf_ls, Tk, W);
    else
        hipLaunchKernelGGL(kv_gather_kernel<bf16>, grid, dim3(128), 0, st, (const bf16*)cache, cache_ls, C, prm, dec,
                           (const bf16*)src, src_ls, src_ld, Tw, (bf16*)buf, buf_ls, Tk, W);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_kv_gather(int dtype, const void* cache, int C, const SPrm* prm, int n, int dec, const void* src,
                         long long src_ld, int Tw, void* buf, int Tk, int W, hipStream_t st) {
    return pfm_kv_gather_layers(dtype, cache, 0, C, prm, n, dec, src, 0, src_ld, Tw, buf, 0, Tk, W, 1, st);
}

hipError_t pfm_kv_retain(int dtype, const void* buf, int Tk, const SPrm* prm, int n, int dec, int drop, const int* ntok,
                         void* cache, int C, int W, hipStream_t st) {
    if (n <= 0 || C <= 0) return hipSuccess;
    if (dtype == DT_F32)
        hipLaunchKernelGGL(kv_retain_kernel<float>, dim3(C, n), dim3(128), 0, st, (const float*)buf, Tk, prm, dec, drop,
                           ntok, (float*)cache, C, W);
    else
        hipLaunchKernelGGL(kv_retain_kernel<bf16>, dim3(C, n), dim3(128), 0, st, (const bf16*)buf, Tk, prm, dec, drop,
                           ntok, (bf16*)cache, C, W);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_stream_mask_rows(float* encp, bf16* encpb, const SPrm* prm, int n, int Tw, int D, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(stream_mask_rows_kernel, dim3(Tw, n), dim3(256), 0, st, encp, encpb, prm, Tw, D);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_cif_chunk(const float* hc, const float* wout, const float* bout, const float* encp, const SPrm* prm,
                         int n, int Tw, int D, int cs0, int keep, float smooth, float noise, float tail, float thr,
                         float* chid, float* calpha, float* emb, int Lcap, int* ntok, float* alphas_out,
                         hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (D > 256 * CIF_CH || Tw > 64) return hipErrorInvalidValue;
    const size_t lds = (size_t)Tw * D * 4;
    const int stage = (lds <= 48 * 1024 && D % 4 == 0 && ((uintptr_t)encp % 16) == 0) ? 1 : 0;
    hipLaunchKernelGGL(cif_chunk_kernel, dim3(n), dim3(256), stage ? lds : 0, st, hc, wout, bout, encp, prm, Tw, D, cs0, keep,
                       smooth, noise, tail, thr, chid, calpha, emb, Lcap, ntok, alphas_out, stage);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_dec_fsmn_stream(int dtype, const void* v, const float* wT, int K, float* state, const SPrm* prm,
                               const int* ntok, int n, int L, int D, float* x, hipStream_t st) {
    if (n <= 0 || L <= 0) return hipSuccess;
    if (K != 11) return hipErrorInvalidValue;
    dim3 grid((D + 255) / 256, n);
    if (dtype == DT_F32)
        hipLaunchKernelGGL((dec_fsmn_stream_kernel<float, 11>), grid, dim3(256), 0, st, (const float*)v, wT, state, prm,
                           ntok, L, D, x);
    else
        hipLaunchKernelGGL((dec_fsmn_stream_kernel<bf16, 11>), grid, dim3(256), 0, st, (const bf16*)v, wT, state, prm,
                           ntok, L, D, x);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// ------------------------------------------------------------------------------------------
// Plain kernels for the two layout fixes of a step (kept as kernel nodes in the step graphs):
//   pad rows: rows 0 and Tw+1 of each stream's [Tw+2][D] encoder image are zero (CIF conv padding)
//   row copy: dst[r][0..w) = src[r][0..w), w floats (decoder input <- the CIF embeds)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pad_rows_zero_kernel(float* __restrict__ encp, bf16* __restrict__ encpb, int Tw,
                                                            int D) {
    const long long row = (long long)blockIdx.x * (Tw + 2) + (blockIdx.y ? Tw + 1 : 0);
    for (int c = threadIdx.x; c < D; c += 256) {
        encp[row * D + c] = 0.f;
        if (encpb) encpb[row * D + c] = f2bf(0.f);
    }
}

__global__ __launch_bounds__(256) void rows_copy_kernel(float* __restrict__ dst, long long dld,
                                                        const float* __restrict__ src, long long sld, int w4) {
    const int r = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < w4) ((float4*)(dst + r * dld))[c] = ((const float4*)(src + r * sld))[c];
}

hipError_t pfm_pad_rows_zero(float* encp, bf16* encpb, int n, int Tw, int D, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(pad_rows_zero_kernel, dim3(n, 2), dim3(256), 0, st, encp, encpb, Tw, D);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_rows_copy(float* dst, long long dld, const float* src, long long sld, int w, int rows, hipStream_t st) {
    if (rows <= 0 || w <= 0) return hipSuccess;
    if (w % 4 || dld % 4 || sld % 4) return hipErrorInvalidValue;
    const int w4 = w / 4;
    hipLaunchKernelGGL(rows_copy_kernel, dim3((w4 + 255) / 256, rows), dim3(256), 0, st, dst, dld, src, sld, w4);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
