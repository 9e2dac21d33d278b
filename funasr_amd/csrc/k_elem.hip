// HBM-bound kernels of the Paraformer path: LayerNorm (+ embedding prologue), FSMN memory
// block, CIF predictor head + integrate-and-fire, and the row-argmax reduction.
#include <stdint.h>
#include <stdlib.h>

#include "pfm_common.h"
#include "pfm_stream.h"

namespace {

// ------------------------------------------------------------------------------------------
// LayerNorm over the last dim (funasr/models/transformer/layer_norm.py:13-39, eps 1e-12).
// One wave per row, float4 loads; mean/var in f64 (rows are <= 2048 wide) so the result is the
// correctly-rounded normalisation the CPU reference approximates to ~1 ulp.
// Optional prologue (encoder input, sanm/encoder.py:377-397):  x = in * in_scale + pe[t].
// ------------------------------------------------------------------------------------------
constexpr int LN_MAXV = 8;   // float4 per lane -> D <= 2048

// Streaming form for D = 512 * VPL (the path's 512- and 2048-wide rows): lane owns 8 contiguous
// columns per 512-column slab (two float4 loads, one 16-B store), R rows per wave with every row
// load and gamma / beta issued before the first store (vmcnt retires in order, so a load behind a
// store waits for it). Same f64 statistics as layernorm_kernel.
template <int VPL, int R, typename TIN = float>   // TIN bf16: fast-mode FFN hidden (one 16-B load per 8 columns)
__global__ __launch_bounds__(256) void layernorm_v8_kernel(const TIN* __restrict__ x, RowMap xmap, int M,
                                                           const float* __restrict__ g, const float* __restrict__ bta,
                                                           float eps, void* out, RowMap omap, int odt, void* out2,
                                                           RowMap o2map, int o2dt) {
    constexpr int D = 512 * VPL;
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
    if (row0 >= M) return;
    float4 v[R][VPL][2];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const TIN* xr = x + xmap.off(min(row0 + r, M - 1));
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            const int c = i * 512 + lane * 8;
            if constexpr (sizeof(TIN) == 4) {
                v[r][i][0] = *(const float4*)(xr + c);
                v[r][i][1] = *(const float4*)(xr + c + 4);
            } else {
                const bf16x8 t = *(const bf16x8*)(xr + c);
                v[r][i][0] = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
                v[r][i][1] = make_float4(bf2f(t[4]), bf2f(t[5]), bf2f(t[6]), bf2f(t[7]));
            }
        }
    }
    float4 gg[VPL][2], bb[VPL][2];
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
        const int c = i * 512 + lane * 8;
        gg[i][0] = *(const float4*)(g + c); gg[i][1] = *(const float4*)(g + c + 4);
        bb[i][0] = *(const float4*)(bta + c); bb[i][1] = *(const float4*)(bta + c + 4);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        if (row >= M) break;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < VPL; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                s += (double)v[r][i][h].x + (double)v[r][i][h].y + (double)v[r][i][h].z + (double)v[r][i][h].w;
        const double mean = wave_sum_d(s) / D;
        double q = 0.0;
#pragma unroll
        for (int i = 0; i < VPL; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const double a0 = v[r][i][h].x - mean, a1 = v[r][i][h].y - mean, a2 = v[r][i][h].z - mean,
                             a3 = v[r][i][h].w - mean;
                q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
            }
        const double rstd = 1.0 / sqrt(wave_sum_d(q) / D + (double)eps);
        const long long ob = omap.off(row), ob2 = out2 ? o2map.off(row) : 0;
#pragma unroll
        for (int i = 0; i < VPL; ++i) {
            const int c = i * 512 + lane * 8;
            float y[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float4 t = v[r][i][h], ga = gg[i][h], be = bb[i][h];
                y[4 * h + 0] = (float)((t.x - mean) * rstd) * ga.x + be.x;
                y[4 * h + 1] = (float)((t.y - mean) * rstd) * ga.y + be.y;
                y[4 * h + 2] = (float)((t.z - mean) * rstd) * ga.z + be.z;
                y[4 * h + 3] = (float)((t.w - mean) * rstd) * ga.w + be.w;
            }
            if (odt == DT_F32) {
                *(float4*)((float*)out + ob + c) = make_float4(y[0], y[1], y[2], y[3]);
                *(float4*)((float*)out + ob + c + 4) = make_float4(y[4], y[5], y[6], y[7]);
            } else if (odt == DT_X3) {   // EXACT-mode split operand: planes D apart within the 3D-wide row
                bf16x8 p0, p1, p2;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    bf16 u, w, z;
                    split3_bf16(y[e], u, w, z);
                    p0[e] = u; p1[e] = w; p2[e] = z;
                }
                *(bf16x8*)((bf16*)out + ob + c) = p0;
                *(bf16x8*)((bf16*)out + ob + D + c) = p1;
                *(bf16x8*)((bf16*)out + ob + 2 * D + c) = p2;
            } else {
                bf16x8 t = {f2bf(y[0]), f2bf(y[1]), f2bf(y[2]), f2bf(y[3]), f2bf(y[4]), f2bf(y[5]), f2bf(y[6]), f2bf(y[7])};
                *(bf16x8*)((bf16*)out + ob + c) = t;
            }
            if (out2) {
                if (o2dt == DT_F32) {
                    *(float4*)((float*)out2 + ob2 + c) = make_float4(y[0], y[1], y[2], y[3]);
                    *(float4*)((float*)out2 + ob2 + c + 4) = make_float4(y[4], y[5], y[6], y[7]);
                } else {
                    bf16x8 t = {f2bf(y[0]), f2bf(y[1]), f2bf(y[2]), f2bf(y[3]), f2bf(y[4]), f2bf(y[5]), f2bf(y[6]), f2bf(y[7])};
                    *(bf16x8*)((bf16*)out2 + ob2 + c) = t;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, RowMap xmap, int M, int D,
                                                        const float* __restrict__ g, const float* __restrict__ bta,
                                                        float eps, const float* __restrict__ pe, int pe_T,
                                                        float in_scale, void* out, RowMap omap, int odt,
                                                        void* out2, RowMap o2map, int o2dt) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float* xr = x + xmap.off(row);
    const float* per = pe ? pe + (long long)(row % pe_T) * D : nullptr;
    float4 v[LN_MAXV];
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int c = (lane + 64 * i) * 4;
        if (c < D) {
            float4 t = *(const float4*)(xr + c);
            if (per) {
                const float4 p = *(const float4*)(per + c);
                t.x = t.x * in_scale + p.x; t.y = t.y * in_scale + p.y;
                t.z = t.z * in_scale + p.z; t.w = t.w * in_scale + p.w;
            }
            v[i] = t;
            s += (double)t.x + (double)t.y + (double)t.z + (double)t.w;
        }
    }
    s = wave_sum_d(s);
    const double mean = s / D;
    double q = 0.0;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int c = (lane + 64 * i) * 4;
        if (c < D) {
            const double a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
            q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
        }
    }
    q = wave_sum_d(q);
    const double rstd = 1.0 / sqrt(q / D + (double)eps);
    const long long ob = omap.off(row), ob2 = out2 ? o2map.off(row) : 0;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int c = (lane + 64 * i) * 4;
        if (c < D) {
            const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(bta + c);
            float4 y;
            y.x = (float)((v[i].x - mean) * rstd) * gg.x + bb.x;
            y.y = (float)((v[i].y - mean) * rstd) * gg.y + bb.y;
            y.z = (float)((v[i].z - mean) * rstd) * gg.z + bb.z;
            y.w = (float)((v[i].w - mean) * rstd) * gg.w + bb.w;
            if (odt == DT_F32) *(float4*)((float*)out + ob + c) = y;
            else {
                bf16x4 t = {f2bf(y.x), f2bf(y.y), f2bf(y.z), f2bf(y.w)};
                *(bf16x4*)((bf16*)out + ob + c) = t;
            }
            if (out2) {
                if (o2dt == DT_F32) *(float4*)((float*)out2 + ob2 + c) = y;
                else {
                    bf16x4 t = {f2bf(y.x), f2bf(y.y), f2bf(y.z), f2bf(y.w)};
                    *(bf16x4*)((bf16*)out2 + ob2 + c) = t;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// FSMN memory block (sanm/attention.py:207-223 encoder; :499-547 decoder):
//   y[t,c] = m[t] * ( sum_k w[c,k] * m[t+k-left] v[t+k-left,c] + m[t] v[t,c] )  (+ res[t,c])
// depthwise Conv1d(groups=D, no bias) over the masked sequence with (left, K-1-left) zero pad.
// One thread per (row, 4 channels); the K-row window is served from L1/L2.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fsmn_kernel(const float* __restrict__ v, RowMap vmap,
                                                   const int* __restrict__ len, int B, int T, int D,
                                                   const float* __restrict__ w, int K, int left,
                                                   const float* __restrict__ res, float* __restrict__ out,
                                                   bf16* __restrict__ out_bf) {
    const int qpr = D / 4;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)B * T * qpr) return;
    const int c = (int)(gid % qpr) * 4;
    const long long row = gid / qpr;
    const int b = (int)(row / T), t = (int)(row % T);
    const int L = min(len[b], T);
    float4 acc = make_float4(0, 0, 0, 0);
    float4 self = make_float4(0, 0, 0, 0);
    const bool valid = t < L;
    if (valid) {
        for (int k = 0; k < K; ++k) {
            const int tt = t + k - left;
            if (tt < 0 || tt >= L) continue;
            const float4 x = *(const float4*)(v + vmap.off((long long)b * T + tt) + c);
            const float4 wk = *(const float4*)(w + (long long)k * D + c);
            acc.x = fmaf(wk.x, x.x, acc.x);
            acc.y = fmaf(wk.y, x.y, acc.y);
            acc.z = fmaf(wk.z, x.z, acc.z);
            acc.w = fmaf(wk.w, x.w, acc.w);
        }
        self = *(const float4*)(v + vmap.off(row) + c);
    }
    float4 y;
    y.x = valid ? acc.x + self.x : 0.f;
    y.y = valid ? acc.y + self.y : 0.f;
    y.z = valid ? acc.z + self.z : 0.f;
    y.w = valid ? acc.w + self.w : 0.f;
    if (res) {
        const float4 r = *(const float4*)(res + row * D + c);
        y.x = r.x + y.x; y.y = r.y + y.y; y.z = r.z + y.z; y.w = r.w + y.w;
    }
    *(float4*)(out + row * D + c) = y;
    if (out_bf) {
        bf16x4 tb = {f2bf(y.x), f2bf(y.y), f2bf(y.z), f2bf(y.w)};
        *(bf16x4*)(out_bf + row * D + c) = tb;
    }
}

// Register-window FSMN: one thread = 4 channels x FR consecutive frames of one utterance.
// The (FR + K - 1)-frame window of masked inputs lives in registers (each input float4 is
// loaded once per window instead of K times) and the taps come from the transposed weight
// wT[K][D] as float4 (coalesced). Same arithmetic order as fsmn_kernel.
constexpr int FR = 8;
template <typename T> __device__ __forceinline__ float4 load4(const T* p);
template <> __device__ __forceinline__ float4 load4<float>(const float* p) { return *(const float4*)p; }
template <> __device__ __forceinline__ float4 load4<bf16>(const bf16* p) {
    const bf16x4 b = *(const bf16x4*)p;
    return make_float4(bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3]));
}

template <int KK, typename TIN, int LEFT = -1>   // LEFT >= 0: compile-time offset (static window index)
__device__ __forceinline__ void fsmn_win_body(long long gid, const TIN* __restrict__ v, RowMap vmap,
                                              const int* __restrict__ len, int B, int T, int D,
                                              const float* __restrict__ wT, int left_rt,
                                              const float* __restrict__ res, float* __restrict__ out,
                                              bf16* __restrict__ out_bf) {
    const int left = LEFT >= 0 ? LEFT : left_rt;
    const int qpr = D / 4;
    const int nblk = (T + FR - 1) / FR;
    if (gid >= (long long)B * nblk * qpr) return;
    const int c = (int)(gid % qpr) * 4;
    const long long rb = gid / qpr;
    const int b = (int)(rb / nblk), t0 = (int)(rb % nblk) * FR;
    const int L = min(len[b], T);
    float4 w[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) w[k] = *(const float4*)(wT + (long long)k * D + c);
    // rows of one utterance are contiguous (plain map, or one segment per utterance: host-checked), so
    // the window is ubase + tt*ld. Loads are unconditional from a clamped row and masked afterwards:
    // all FR+KK-1 loads are in flight together instead of one branch + vmcnt(0) round trip per row.
    const long long ubase = vmap.rows_per_seg > 0 ? (long long)b * vmap.seg_stride : (long long)b * T * vmap.ld;
    float4 x[FR + KK - 1];
#pragma unroll
    for (int i = 0; i < FR + KK - 1; ++i) {
        const int tt = t0 - left + i;
        const int tc = min(max(tt, 0), T - 1);
        x[i] = load4<TIN>(v + ubase + (long long)tc * vmap.ld + c);
    }
#pragma unroll
    for (int i = 0; i < FR + KK - 1; ++i) {
        const int tt = t0 - left + i;
        if (!(tt >= 0 && tt < L)) x[i] = make_float4(0, 0, 0, 0);
    }
    // residual rows are read before any store: vmcnt retires in order, so a load issued after a
    // store would wait for that store
    float4 rv[FR];
    if (res) {
#pragma unroll
        for (int i = 0; i < FR; ++i)
            rv[i] = *(const float4*)(res + ((long long)b * T + min(t0 + i, T - 1)) * D + c);
    }
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        const int t = t0 + i;
        if (t >= T) break;
        const long long row = (long long)b * T + t;
        float4 y = make_float4(0, 0, 0, 0);
        if (t < L) {
            float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                acc.x = fmaf(w[k].x, x[i + k].x, acc.x);
                acc.y = fmaf(w[k].y, x[i + k].y, acc.y);
                acc.z = fmaf(w[k].z, x[i + k].z, acc.z);
                acc.w = fmaf(w[k].w, x[i + k].w, acc.w);
            }
            const float4 self = x[i + left];
            y = make_float4(acc.x + self.x, acc.y + self.y, acc.z + self.z, acc.w + self.w);
        }
        if (res) {
            const float4 r = rv[i];
            y.x = r.x + y.x; y.y = r.y + y.y; y.z = r.z + y.z; y.w = r.w + y.w;
        }
        if (out) *(float4*)(out + row * D + c) = y;
        if (out_bf) {
            bf16x4 tb = {f2bf(y.x), f2bf(y.y), f2bf(y.z), f2bf(y.w)};
            *(bf16x4*)(out_bf + row * D + c) = tb;
        }
    }
}
template <int KK, typename TIN, int LEFT = -1>
__global__ __launch_bounds__(256) void fsmn_win_kernel(const TIN* __restrict__ v, RowMap vmap,
                                                       const int* __restrict__ len, int B, int T, int D,
                                                       const float* __restrict__ wT, int left_rt,
                                                       const float* __restrict__ res, float* __restrict__ out,
                                                       bf16* __restrict__ out_bf) {
    fsmn_win_body<KK, TIN, LEFT>((long long)blockIdx.x * blockDim.x + threadIdx.x, v, vmap, len, B, T, D, wT, left_rt,
                                 res, out, out_bf);
}

// streaming encoder layer: blocks [0, nf) run the window's FSMN (fsmn_win_kernel<11, bf16, 5>, lens = tw), blocks
// nf + (i Tk + r) gather key row r of stream i (kv_gather_row): two independent launches of the chunk step as one
__global__ __launch_bounds__(256) void kv_gather_fsmn_kernel(int nf, const bf16* __restrict__ cache, int C,
                                                             const SPrm* __restrict__ prm, const bf16* __restrict__ src,
                                                             long long src_ld, int Tw, bf16* __restrict__ buf, int Tk,
                                                             int W, const bf16* __restrict__ v, RowMap vmap,
                                                             const int* __restrict__ len, int B, int D,
                                                             const float* __restrict__ wT, bf16* __restrict__ out_bf) {
    if ((int)blockIdx.x < nf) {
        fsmn_win_body<11, bf16, 5>((long long)blockIdx.x * blockDim.x + threadIdx.x, v, vmap, len, B, Tw, D, wT, 5,
                                   nullptr, nullptr, out_bf);
        return;
    }
    const int g = (int)blockIdx.x - nf, i = g / Tk, r = g - i * Tk;
    kv_gather_row(cache, C, prm[i], 0, src, src_ld, Tw, buf, Tk, W, i, r, (int)threadIdx.x, 256);
}

// fsmn_win_kernel<11, TIN, 5> with the following LayerNorm fused (D = 512: a 256-thread block is two
// 8-row blocks x all 128 channel quads): y = res + FSMN(v) as there -> out (f32); then per row
// mean / centred variance over the 512 channels (wave sums, the row's two waves joined through LDS)
// -> ln_out = bf16(LN(y) * g + b). Used by the fast decoder: x += FSMN(LN2(t)) then LN3(x) (decoder.py:104-110).
template <typename TIN>
__global__ __launch_bounds__(256) void fsmn_ln_kernel(const TIN* __restrict__ v, RowMap vmap, const int* __restrict__ len,
                                                      int B, int T, const float* __restrict__ wT,
                                                      const float* __restrict__ res, float* __restrict__ out,
                                                      const float* __restrict__ g, const float* __restrict__ bb,
                                                      float eps, bf16* __restrict__ ln_out) {
    constexpr int KK = 11, LEFT = 5, D = 512, QPR = D / 4;
    __shared__ float red[2][2][FR];   // [row block][wave of the row block][row]
    const int nblk = (T + FR - 1) / FR;
    const long long rbg = (long long)blockIdx.x * 2 + (threadIdx.x >> 7);   // global row block
    const bool valid = rbg < (long long)B * nblk;
    const int q = threadIdx.x & (QPR - 1), c = q * 4;
    const int half = threadIdx.x >> 7, wv = (threadIdx.x >> 6) & 1;
    const int b = valid ? (int)(rbg / nblk) : 0, t0 = valid ? (int)(rbg % nblk) * FR : 0;
    const int L = min(len[b], T);
    float4 w[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) w[k] = *(const float4*)(wT + (long long)k * D + c);
    const long long ubase = vmap.rows_per_seg > 0 ? (long long)b * vmap.seg_stride : (long long)b * T * vmap.ld;
    float4 x[FR + KK - 1];
#pragma unroll
    for (int i = 0; i < FR + KK - 1; ++i) {
        const int tc = min(max(t0 - LEFT + i, 0), T - 1);
        x[i] = load4<TIN>(v + ubase + (long long)tc * vmap.ld + c);
    }
#pragma unroll
    for (int i = 0; i < FR + KK - 1; ++i) {
        const int tt = t0 - LEFT + i;
        if (!(tt >= 0 && tt < L)) x[i] = make_float4(0, 0, 0, 0);
    }
    float4 rv[FR];
#pragma unroll
    for (int i = 0; i < FR; ++i) rv[i] = *(const float4*)(res + ((long long)b * T + min(t0 + i, T - 1)) * D + c);
    float4 y[FR];
    float ps[FR];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        const int t = t0 + i;
        float4 f = make_float4(0, 0, 0, 0);
        if (t < L) {
            float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                acc.x = fmaf(w[k].x, x[i + k].x, acc.x);
                acc.y = fmaf(w[k].y, x[i + k].y, acc.y);
                acc.z = fmaf(w[k].z, x[i + k].z, acc.z);
                acc.w = fmaf(w[k].w, x[i + k].w, acc.w);
            }
            const float4 self = x[i + LEFT];
            f = make_float4(acc.x + self.x, acc.y + self.y, acc.z + self.z, acc.w + self.w);
        }
        const float4 r = rv[i];
        y[i] = make_float4(r.x + f.x, r.y + f.y, r.z + f.z, r.w + f.w);
        ps[i] = (y[i].x + y[i].y) + (y[i].z + y[i].w);
        if (valid && t < T) *(float4*)(out + ((long long)b * T + t) * D + c) = y[i];
    }
    // row means: 64-lane sums, then the row block's two waves
#pragma unroll
    for (int i = 0; i < FR; ++i) ps[i] = wave_sum(ps[i]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int i = 0; i < FR; ++i) red[half][wv][i] = ps[i];
    __syncthreads();
    float mean[FR], pq[FR];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        mean[i] = (red[half][0][i] + red[half][1][i]) * (1.f / D);
        const float dx = y[i].x - mean[i], dy = y[i].y - mean[i], dz = y[i].z - mean[i], dw = y[i].w - mean[i];
        pq[i] = (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
    __syncthreads();   // every thread read red[] before it is reused
#pragma unroll
    for (int i = 0; i < FR; ++i) pq[i] = wave_sum(pq[i]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int i = 0; i < FR; ++i) red[half][wv][i] = pq[i];
    __syncthreads();
    const float4 gg = *(const float4*)(g + c), be = *(const float4*)(bb + c);
#pragma unroll
    for (int i = 0; i < FR; ++i) {
        const int t = t0 + i;
        const float rstd = 1.f / sqrtf((red[half][0][i] + red[half][1][i]) * (1.f / D) + eps);
        bf16x4 o = {f2bf((y[i].x - mean[i]) * rstd * gg.x + be.x), f2bf((y[i].y - mean[i]) * rstd * gg.y + be.y),
                    f2bf((y[i].z - mean[i]) * rstd * gg.z + be.z), f2bf((y[i].w - mean[i]) * rstd * gg.w + be.w)};
        if (valid && t < T) *(bf16x4*)(ln_out + ((long long)b * T + t) * D + c) = o;
    }
}

// ------------------------------------------------------------------------------------------
// CIF predictor head (cif_predictor.py:214-242, 346-370):
//   alpha[t] = relu(sigmoid(w . relu(conv)[t] + b) * smooth - noise) * mask[t],  t < T
//   alpha[T] = 0;  alpha[len] += tail_threshold   (tail_process_fn with mask)
// One wave per (utterance, frame); dot product in f64.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cif_alpha_kernel(const float* __restrict__ hc, int D,
                                                        const float* __restrict__ wout, const float* __restrict__ bout,
                                                        const int* __restrict__ len, int B, int T, float smooth,
                                                        float noise, float tail, float* __restrict__ alphas) {
    const int lane = threadIdx.x & 63;
    const long long item = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= (long long)B * (T + 1)) return;
    const int b = (int)(item / (T + 1)), t = (int)(item % (T + 1));
    const int L = min(len[b], T);
    float a = 0.f;
    if (t < T) {
        const float* hr = hc + ((long long)b * T + t) * D;
        double s = 0.0;
        for (int c = lane * 4; c < D; c += 256) {
            const float4 x = *(const float4*)(hr + c), ww = *(const float4*)(wout + c);
            s += (double)x.x * ww.x + (double)x.y * ww.y + (double)x.z * ww.z + (double)x.w * ww.w;
        }
        s = wave_sum_d(s);
        const float z = (float)(s + (double)bout[0]);
        const float sg = (float)(1.0 / (1.0 + exp(-(double)z)));
        a = fmaxf(sg * smooth - noise, 0.f);
        if (t >= L) a = 0.f;
    }
    if (t == L) a = a + tail;
    if (lane == 0) alphas[(long long)b * (T + 1) + t] = a;
}

// ------------------------------------------------------------------------------------------
// Continuous integrate-and-fire (cif_wo_hidden_v1 / cif_v1, cif_predictor.py:668-735).
// One workgroup per utterance; every thread walks the T+1 frames (fire decisions are uniform).
//   P_t  = f32( sum_{s<=t} f64(alpha_s) )            fire_t = floor(P_t) > floor(P_{t-1}), floor(P_-1)=0
//   fires_t = fire_t + (P_t - floor(P_t))  (f32)      rem_t = fires_t - floor(fires_t)
//   PH_t = f32( sum_{s<=t} f64(f32(alpha_s * h_s)) )  (torch CPU cumsum accumulates f32 in f64)
//   emb_k = ((PH_tk - PH_tk-1) + rem_tk-1 h_tk-1) - rem_tk h_tk,    rows >= n_fire are zero
// token_num = floor(sum_t alpha_t) (f64 sum; the reference sums in f32 — see DESIGN.md).
// h rows via RowMap; row T of each utterance must be the zero row appended by tail_process_fn.
// ------------------------------------------------------------------------------------------
// Grid (D/64 channel slabs, B): one wave per (slab, utterance), one channel per lane. Every wave
// recomputes the (uniform) fire schedule, so each channel's operations and their order are those of
// the sequential reference loop; h rows are prefetched CIF_PF frames ahead of the recurrence.
#ifndef CIF_PF_N
#define CIF_PF_N 32
#endif
constexpr int CIF_PF = CIF_PF_N;   // frames per batch; the next batch is in flight while one is scanned
__global__ __launch_bounds__(64) void cif_fire_kernel(const float* __restrict__ alphas, const float* __restrict__ h,
                                                      RowMap hmap, int T, int D, int Lcap,
                                                      float* __restrict__ emb, float* __restrict__ peaks,
                                                      int* __restrict__ n_fire, int* __restrict__ ntok) {
    const int b = blockIdx.y;
    const int c = blockIdx.x * 64 + threadIdx.x;
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    const bool act = c < D;
    const int cc = act ? c : D - 1;
    const float* al = alphas + (long long)b * (T + 1);
    double ph = 0.0, P = 0.0;
    float pph = 0.f, prh = 0.f, prevfl = 0.f;
    int k = 0;
    // an utterance's T + 1 rows are ld apart within one segment (plain map or one segment per utterance:
    // launcher check), so the row address is a base plus t * ld (no per-frame RowMap division)
    const float* hb = h + hmap.off((long long)b * (T + 1)) + cc;
    const long long hld = hmap.ld;
    auto fetch = [&](int t0, float (&hv)[CIF_PF], float (&av)[CIF_PF]) {
#pragma unroll
        for (int i = 0; i < CIF_PF; ++i) {
            const int t = min(t0 + i, T);
            av[i] = al[t];
            hv[i] = hb[(long long)t * hld];
        }
    };
    auto scan = [&](int t0, const float (&hv)[CIF_PF], const float (&av)[CIF_PF]) {
#pragma unroll
        for (int i = 0; i < CIF_PF; ++i) {
            const int t = t0 + i;
            if (t > T) break;
            const float a = av[i];
            P += (double)a;
            const float Pf = (float)P;
            const float fl = floorf(Pf);
            const bool fire = (fl - prevfl) > 0.f;
            prevfl = fl;
            const float fires = (fire ? 1.f : 0.f) + (Pf - fl);
            if (lead && peaks) peaks[(long long)b * (T + 1) + t] = fires;
            const float rem = fires - floorf(fires);
            ph += (double)(a * hv[i]);
            if (fire) {
                const float phf = (float)ph;
                const float rh = rem * hv[i];
                if (act && k < Lcap) emb[((long long)b * Lcap + k) * D + c] = ((phf - pph) + prh) - rh;
                pph = phf;
                prh = rh;
                ++k;
            }
        }
    };
    // two named batches: batch n+1 is loading while batch n is scanned (arrays stay in registers)
    float hA[CIF_PF], aA[CIF_PF], hB[CIF_PF], aB[CIF_PF];
    fetch(0, hA, aA);
    for (int t0 = 0; t0 <= T; t0 += 2 * CIF_PF) {
        if (t0 + CIF_PF <= T) fetch(t0 + CIF_PF, hB, aB);
        scan(t0, hA, aA);
        if (t0 + CIF_PF > T) break;
        if (t0 + 2 * CIF_PF <= T) fetch(t0 + 2 * CIF_PF, hA, aA);
        scan(t0 + CIF_PF, hB, aB);
    }
    if (act)
        for (int kk = k; kk < Lcap; ++kk) emb[((long long)b * Lcap + kk) * D + c] = 0.f;
    if (lead) {   // P is the f64 running sum of alpha[0..T] in order: token_num = floor(sum(alphas))
        n_fire[b] = k;
        ntok[b] = (int)floor(P);
    }
}

// ------------------------------------------------------------------------------------------
// Row argmax over the GEMM's per-(row, 64-column block) partial maxima; first index on ties
// (torch.argmax). argmax(log_softmax(x)) == argmax(x), so logits never reach HBM.
// tokens[b, l] for l < ntok[b], -1 elsewhere (paraformer/model.py:527-536).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void argmax_reduce_kernel(const float* __restrict__ val, const int* __restrict__ idx,
                                                            int ntiles, int ncount, int B, int L, const int* __restrict__ ntok,
                                                            int Lcap, int* __restrict__ tokens, float* __restrict__ score) {
    const int lane = threadIdx.x & 63;
    const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= (long long)B * L) return;
    const int b = (int)(row / L), l = (int)(row % L);
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = lane; i < ncount; i += 64) {
        const float v = val[row * ntiles + i];
        const int ii = idx[row * ntiles + i];
        if (v > bv || (v == bv && ii < bi)) { bv = v; bi = ii; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0 && l < Lcap) {
        tokens[(long long)b * Lcap + l] = (l < ntok[b]) ? bi : -1;
        if (score) score[(long long)b * Lcap + l] = bv;
    }
}

__global__ void fill_i32_kernel(int* p, long long n, int v) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
    const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i + 3 < n) {
        const float4 v = *(const float4*)(x + i);
        bf16x4 t = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
        *(bf16x4*)(y + i) = t;
    } else {
        for (long long j = i; j < n; ++j) y[j] = f2bf(x[j]);
    }
}

// ------------------------------------------------------------------------------------------
// SenseVoiceSmall input (sense_voice/model.py:851-876): every utterance gets the four query
// embeddings [language, event, emotion, text-norm] in front of its frames; lengths grow by nq.
//   x[b, t] = t < nq ? embed[qid[t]] : feats[b, t - nq]      x: [B, T + nq, I]
// One wave per output row, float4 copies (I % 4 == 0).
// ------------------------------------------------------------------------------------------
struct QueryIds { int id[4]; };
__global__ __launch_bounds__(256) void sv_input_kernel(const float* __restrict__ feats, const int* __restrict__ lens,
                                                       const float* __restrict__ embed, QueryIds q, int nq, int B,
                                                       int T, int I, float* __restrict__ x, int* __restrict__ olen) {
    const int lane = threadIdx.x & 63;
    const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int Tq = T + nq;
    if (row >= (long long)B * Tq) return;
    const int b = (int)(row / Tq), t = (int)(row % Tq);
    const float* src = t < nq ? embed + (long long)q.id[t] * I : feats + ((long long)b * T + (t - nq)) * I;
    float* dst = x + row * I;
    for (int c = lane * 4; c < I; c += 256) *(float4*)(dst + c) = *(const float4*)(src + c);
    // clamp like every other length consumer: the collapse kernel reads [0, olen) of a [T + nq] row
    if (t == 0 && lane == 0) olen[b] = min(max(lens[b], 0), T) + nq;
}

// ------------------------------------------------------------------------------------------
// Greedy CTC collapse (sense_voice/model.py:893-906; ctc/model.py greedy): per utterance,
// unique_consecutive over the frame argmax ids [0, olen), then drop blank. One wave per
// utterance walks 64-frame chunks: keep[t] = id[t] != blank && (t == 0 || id[t] != id[t-1]);
// ballot + popcount give each kept frame its output slot. tokens [B, Lcap] (-1 beyond ntok).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ctc_collapse_kernel(const int* __restrict__ ids, long long ld, const int* __restrict__ olen,
                                                          int blank, int Lcap, int* __restrict__ tokens,
                                                          int* __restrict__ ntok) {
    const int lane = threadIdx.x;
    const int b = blockIdx.x;
    const int n = (int)min((long long)max(olen[b], 0), ld);   // never past the utterance's id row
    const int* r = ids + (long long)b * ld;
    int* out = tokens + (long long)b * Lcap;
    int cnt = 0;
    for (int base = 0; base < n; base += 64) {
        const int t = base + lane;
        const int v = t < n ? r[t] : blank;
        const int pv = (t > 0 && t - 1 < n) ? r[t - 1] : -2;
        const bool keep = t < n && v != blank && v != pv;
        const unsigned long long m = __ballot(keep);
        const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
        if (keep && pos < Lcap) out[pos] = v;
        cnt += __popcll(m);
    }
    for (int i = cnt + lane; i < Lcap; i += 64) out[i] = -1;
    if (lane == 0) ntok[b] = cnt;
}


// ------------------------------------------------------------------------------------------
// [A][Bd][C] -> [A][C][Bd] (weight re-layout of device-resident state_dict tensors: Conv1d [O][I][k] -> [O][k][I],
// depthwise taps [D][1][K] -> [K][D]); one thread per output element, coalesced stores
__global__ void swap_last2_kernel(const float* __restrict__ x, float* __restrict__ y, long long A, long long Bd,
                                  long long C) {
    const long long i = blockIdx.x * 256LL + threadIdx.x, n = A * Bd * C;
    if (i >= n) return;
    const long long b = i % Bd, c = (i / Bd) % C, a = i / (Bd * C);
    y[i] = x[(a * Bd + b) * C + c];
}

}  // namespace

hipError_t pfm_sv_input(const float* feats, const int* lens, const float* embed, const int* qid, int nq, int B, int T,
                        int I, float* x, int* olen, hipStream_t st) {
    if (nq < 0 || nq > 4 || I % 4) return hipErrorInvalidValue;
    QueryIds q = {{0, 0, 0, 0}};
    for (int i = 0; i < nq; ++i) q.id[i] = qid[i];
    const long long rows = (long long)B * (T + nq);
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(sv_input_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, feats, lens, embed, q, nq,
                       B, T, I, x, olen);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_ctc_collapse(const int* ids, long long ld, const int* olen, int B, int blank, int Lcap, int* tokens,
                            int* ntok, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(ctc_collapse_kernel, dim3((unsigned)B), dim3(64), 0, st, ids, ld, olen, blank, Lcap, tokens,
                       ntok);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_layernorm(const float* x, RowMap xmap, int M, int D, const float* g, const float* b, float eps,
                         const float* pe, int pe_T, float in_scale, void* out, RowMap omap, int odt, void* out2,
                         RowMap o2map, int o2dt, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (D % 4 != 0 || D > 4 * 64 * LN_MAXV) return hipErrorInvalidValue;
    // streaming kernel: no prologue, D in {512, 1024, 2048}, 16-B aligned rows (8-element multiples)
    auto al8 = [](const RowMap& m, const void* p, int dt) {
        const int q = dt == DT_F32 ? 4 : 8;
        return m.ld % q == 0 && (m.rows_per_seg <= 0 || m.seg_stride % q == 0) && ((uintptr_t)p % 16) == 0;
    };
    if (!pe && (D == 512 || D == 1024 || D == 2048) && al8(xmap, x, DT_F32) && al8(omap, out, odt) &&
        (!out2 || al8(o2map, out2, o2dt))) {
        constexpr int R = 2;
        const unsigned blocks = (unsigned)(((M + R - 1) / R + 3) / 4);
        const unsigned blocks1 = (unsigned)((M + 3) / 4);   // 2048-wide rows: one row per wave (register budget)
        if (D == 512)
            hipLaunchKernelGGL((layernorm_v8_kernel<1, R>), dim3(blocks), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                               omap, odt, out2, o2map, o2dt);
        else if (D == 1024)
            hipLaunchKernelGGL((layernorm_v8_kernel<2, R>), dim3(blocks), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                               omap, odt, out2, o2map, o2dt);
        else
            hipLaunchKernelGGL((layernorm_v8_kernel<4, 1>), dim3(blocks1), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                               omap, odt, out2, o2map, o2dt);
        PFM_LAUNCH_CHECK();
        return hipSuccess;
    }
    if (odt == DT_X3 || o2dt == DT_X3) return hipErrorInvalidValue;   // split output: streaming kernel only
    hipLaunchKernelGGL(layernorm_kernel, dim3((M + 3) / 4), dim3(256), 0, st, x, xmap, M, D, g, b, eps, pe,
                       pe_T > 0 ? pe_T : 1, in_scale, out, omap, odt, out2, o2map, o2dt);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// bf16-input LayerNorm (fast mode; D in {512, 1024, 2048}, 16-B aligned rows)
hipError_t pfm_layernorm_bf16in(const bf16* x, RowMap xmap, int M, int D, const float* g, const float* b, float eps,
                                void* out, RowMap omap, int odt, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (!(D == 512 || D == 1024 || D == 2048) || xmap.ld % 8 || (xmap.rows_per_seg > 0 && xmap.seg_stride % 8) ||
        ((uintptr_t)x % 16) || ((uintptr_t)out % 16) || omap.ld % 8)
        return hipErrorInvalidValue;
    const unsigned blocks2 = (unsigned)(((M + 1) / 2 + 3) / 4), blocks1 = (unsigned)((M + 3) / 4);
    if (D == 512)
        hipLaunchKernelGGL((layernorm_v8_kernel<1, 2, bf16>), dim3(blocks2), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                           omap, odt, nullptr, rowmap_plain(0), 0);
    else if (D == 1024)
        hipLaunchKernelGGL((layernorm_v8_kernel<2, 2, bf16>), dim3(blocks2), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                           omap, odt, nullptr, rowmap_plain(0), 0);
    else
        hipLaunchKernelGGL((layernorm_v8_kernel<4, 1, bf16>), dim3(blocks1), dim3(256), 0, st, x, xmap, M, g, b, eps, out,
                           omap, odt, nullptr, rowmap_plain(0), 0);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// wT: taps transposed [K][D] (the registry stores fsmn_block.weight [D,1,K] that way).
hipError_t pfm_fsmn(const float* v, RowMap vmap, const int* len, int B, int T, int D, const float* wT, int K,
                    int left, const float* res, float* out, bf16* out_bf, hipStream_t st) {
    if (B <= 0 || T <= 0) return hipSuccess;
    if (D % 4 != 0 || left < 0 || left >= K) return hipErrorInvalidValue;
    if (K == 11 && (vmap.rows_per_seg <= 0 || vmap.rows_per_seg == T)) {
        const long long n = (long long)B * ((T + FR - 1) / FR) * (D / 4);
        if (left == 5)
            hipLaunchKernelGGL((fsmn_win_kernel<11, float, 5>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v,
                               vmap, len, B, T, D, wT, left, res, out, out_bf);
        else
            hipLaunchKernelGGL((fsmn_win_kernel<11, float>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v,
                               vmap, len, B, T, D, wT, left, res, out, out_bf);
        PFM_LAUNCH_CHECK();
        return hipSuccess;
    }
    const long long n = (long long)B * T * (D / 4);
    hipLaunchKernelGGL(fsmn_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v, vmap, len, B, T, D, wT,
                       K, left, res, out, out_bf);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// bf16 input V (fast mode): out_bf only (f32 out optional)
// x_out = res + FSMN(v) (K 11, left 5, D 512; f32) and ln_out = bf16(LayerNorm(x_out) g + b) in one pass
hipError_t pfm_fsmn_ln_bf16in(const bf16* v, RowMap vmap, const int* len, int B, int T, int D, const float* wT,
                              int K, int left, const float* res, float* out, const float* g, const float* b, float eps,
                              bf16* ln_out, hipStream_t st) {
    if (B <= 0 || T <= 0) return hipSuccess;
    if (D != 512 || K != 11 || left != 5 || !res || !out || !ln_out) return hipErrorInvalidValue;
    if (vmap.rows_per_seg > 0 && vmap.rows_per_seg != T) return hipErrorInvalidValue;
    const long long nrb = (long long)B * ((T + FR - 1) / FR);
    hipLaunchKernelGGL(fsmn_ln_kernel<bf16>, dim3((unsigned)((nrb + 1) / 2)), dim3(256), 0, st, v, vmap, len, B, T, wT,
                       res, out, g, b, eps, ln_out);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_fsmn_bf16in(const bf16* v, RowMap vmap, const int* len, int B, int T, int D, const float* wT, int K,
                           int left, const float* res, float* out, bf16* out_bf, hipStream_t st) {
    if (B <= 0 || T <= 0) return hipSuccess;
    if (D % 4 != 0 || K != 11 || left < 0 || left >= K) return hipErrorInvalidValue;
    if (vmap.rows_per_seg > 0 && vmap.rows_per_seg != T) return hipErrorInvalidValue;
    const long long n = (long long)B * ((T + FR - 1) / FR) * (D / 4);
    if (left == 5)
        hipLaunchKernelGGL((fsmn_win_kernel<11, bf16, 5>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v, vmap,
                           len, B, T, D, wT, left, res, out, out_bf);
    else
        hipLaunchKernelGGL((fsmn_win_kernel<11, bf16>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, v, vmap,
                           len, B, T, D, wT, left, res, out, out_bf);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_kv_gather_fsmn(const bf16* cache, int C, const SPrm* prm, int n, const bf16* src, long long src_ld, int Tw,
                              bf16* buf, int Tk, int W, const bf16* v, RowMap vmap, const int* len, int D, const float* wT,
                              bf16* out_bf, hipStream_t st) {
    if (n <= 0 || Tk <= 0 || Tw <= 0) return hipSuccess;
    if (D % 4 || (W * 2) % 16 || (src_ld * 2) % 16 || ((uintptr_t)src % 16) || ((uintptr_t)buf % 16) ||
        ((uintptr_t)cache % 16) || (vmap.rows_per_seg > 0 && vmap.rows_per_seg != Tw))
        return hipErrorInvalidValue;
    const long long nfl = ((long long)n * ((Tw + FR - 1) / FR) * (D / 4) + 255) / 256;
    const long long ng = (long long)n * Tk;
    if (nfl + ng >= (1LL << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kv_gather_fsmn_kernel, dim3((unsigned)(nfl + ng)), dim3(256), 0, st, (int)nfl, cache, C, prm, src,
                       src_ld, Tw, buf, Tk, W, v, vmap, len, n, D, wT, out_bf);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_cif_alpha(const float* hc, int D, const float* wout, const float* bout, const int* len, int B,
                         int T, float smooth, float noise, float tail, float* alphas, hipStream_t st) {
    const long long n = (long long)B * (T + 1);
    hipLaunchKernelGGL(cif_alpha_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, hc, D, wout, bout, len,
                       B, T, smooth, noise, tail, alphas);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_cif_fire(const float* alphas, const float* h, RowMap hmap, int B, int T, int D, int Lcap,
                        float* emb, float* peaks, int* n_fire, int* ntok, hipStream_t st) {
    if (B <= 0 || D <= 0) return hipSuccess;
    if (hmap.rows_per_seg > 0 && hmap.rows_per_seg != T + 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cif_fire_kernel, dim3((D + 63) / 64, B), dim3(64), 0, st, alphas, h, hmap, T, D, Lcap, emb,
                       peaks, n_fire, ntok);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// ntiles: row stride of the partial buffers; ncount: valid 64-column blocks (ceil(N/64))
hipError_t pfm_argmax_reduce(const float* val, const int* idx, int ntiles, int ncount, int B, int L, const int* ntok,
                             int Lcap, int* tokens, float* score, hipStream_t st) {
    const long long n = (long long)B * L;
    if (n <= 0) return hipSuccess;
    if (ncount > ntiles) return hipErrorInvalidValue;
    hipLaunchKernelGGL(argmax_reduce_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, val, idx, ntiles, ncount,
                       B, L, ntok, Lcap, tokens, score);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_fill_i32(int* p, long long n, int v, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_i32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, n, v);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// ------------------------------------------------------------------------------------------
// Three-way bf16 split of f32 operands for the split-bf16 emulation of EXACT-mode GEMMs:
//   x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)  =>  x0 + x1 + x2 == x exactly (normal range;
// each residual is exact in f32 and has <= 8 significant bits left for x2). With these,
//   a.w ~= a0w0 + a0w1 + a1w0 + a0w2 + a1w1 + a2w0   (dropped terms <= 2^-25 |a w|; bf16 products exact)
// so six bf16 MFMAs with f32 accumulation reproduce the f32 product to f32 rounding.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void split3(float x, bf16& a, bf16& b, bf16& c) {
    a = f2bf(x);
    const float r1 = x - bf2f(a);
    b = f2bf(r1);
    c = f2bf(r1 - bf2f(b));
}

// rows of x (RowMap, K columns) -> out [M][3 Kp] = [x0 | x1 | x2], segments zero-padded to Kp >= K columns;
// 4 columns per thread
__global__ __launch_bounds__(256) void split3_rows_kernel(const float* __restrict__ x, RowMap xm, int M, int K, int Kp,
                                                          bf16* __restrict__ out) {
    const int k4 = Kp >> 2;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)M * k4) return;
    const long long row = i / k4;
    const int c = (int)(i - row * k4) * 4;
    const float4 v = c < K ? *(const float4*)(x + xm.off(row) + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float xv[4] = {v.x, v.y, v.z, v.w};
    bf16x4 p0, p1, p2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        bf16 a, b, cc;
        split3(xv[e], a, b, cc);
        p0[e] = a;
        p1[e] = b;
        p2[e] = cc;
    }
    bf16* o = out + row * 3 * Kp + c;
    *(bf16x4*)o = p0;
    *(bf16x4*)(o + Kp) = p1;
    *(bf16x4*)(o + 2 * Kp) = p2;
}

// n contiguous f32 -> planes p, p + plane, p + 2 plane (weights: plane stride = the arena size)
__global__ __launch_bounds__(256) void split3_planes_kernel(const float* __restrict__ x, bf16* __restrict__ p,
                                                            long long plane, long long n) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    bf16 a, b, c;
    split3(x[i], a, b, c);
    p[i] = a;
    p[plane + i] = b;
    p[2 * plane + i] = c;
}

hipError_t pfm_split3_rows(const float* x, RowMap xm, int M, int K, int Kp, bf16* out, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (K % 4 || Kp % 4 || Kp < K || !rowmap_vec4(xm) || ((uintptr_t)x % 16) || ((uintptr_t)out % 8))
        return hipErrorInvalidValue;
    const long long n = (long long)M * (Kp / 4);
    hipLaunchKernelGGL(split3_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, xm, M, K, Kp, out);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_split3_planes(const float* x, bf16* p, long long plane, long long n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(split3_planes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, p, plane, n);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_f32_to_bf16(const float* x, bf16* y, long long n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const long long nt = (n + 3) / 4;
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, x, y, n);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_swap_last2(const float* x, float* y, long long A, long long Bd, long long C, hipStream_t st) {
    const long long n = A * Bd * C;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(swap_last2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, y, A, Bd, C);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
