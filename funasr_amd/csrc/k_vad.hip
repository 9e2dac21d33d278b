// FSMN-VAD encoder kernels (funasr/models/fsmn_vad_streaming/encoder.py:12-279): the per-frame speech /
// silence posteriors that the VAD state machine (fsmn_vad_streaming/model.py:493-546, host side) consumes.
//
//   vad_dense_kernel   Y[t, n] = act(X[t, :] . W[n, :] + b[n]) for the Affine / Linear transforms
//                      (K = 400, 140, 250, 128: any K; f32 FMA chain per output in k order, 64 x 64
//                      LDS-tiled, the weight matrices (<= 56k floats) stay L2-resident)
//   vad_fsmn_kernel    causal memory block (FSMNBlock.forward with its cache, rorder 0): y[t] = x[t] +
//                      sum_j w[c][j] * x[t - (L-1) + j], rows before the chunk from the per-layer cache
//                      (zeros at the start of a stream); the cache then keeps the chunk's last L-1 rows
//   vad_softmax_kernel softmax over the output pdfs per frame (one wave per frame); writes p[t][0] (the
//                      silence pdf, sil_pdf_ids = [0]) and optionally every posterior
#include <math.h>

#include "pfm_common.h"

namespace {

// 64 x 64 output tile per 256-thread block, 4 x 4 outputs per thread, K staged through LDS 16 at a time
// (X and W tiles stored k-major so a thread's 4 rows / 4 columns are contiguous). Every output keeps the
// plain serial chain s = fma(x[k], w[k], s) for k = 0..K-1 (the k loop never pads), then + b, then ReLU,
// so the result is bit-identical to a one-thread-per-output dot product; the tiling only removes the
// K-strided weight reads and re-reads of X.
constexpr int VD_TM = 64, VD_TN = 64, VD_TK = 16;
__global__ __launch_bounds__(256) void vad_dense_kernel(const float* __restrict__ X, int ldx, int M, int K,
                                                        const float* __restrict__ W, const float* __restrict__ b,
                                                        int N, int relu, float* __restrict__ Y, int ldy) {
    __shared__ float Xs[VD_TK][VD_TM + 4];
    __shared__ float Ws[VD_TK][VD_TN + 4];
    const int tid = threadIdx.x;
    const int tx = tid % 16, ty = tid / 16;          // 16 x 16 threads, each 4 cols x 4 rows
    const int m0 = blockIdx.y * VD_TM, n0 = blockIdx.x * VD_TN;
    const int lr = tid / 4, lk = (tid % 4) * 4;      // loader: row lr of the tile, k lk..lk+3
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    for (int k0 = 0; k0 < K; k0 += VD_TK) {
        const int kn = min(VD_TK, K - k0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = k0 + lk + q;
            const int m = m0 + lr, n = n0 + lr;
            Xs[lk + q][lr] = (k < K && m < M) ? X[(long long)m * ldx + k] : 0.f;
            Ws[lk + q][lr] = (k < K && n < N) ? W[(long long)n * K + k] : 0.f;
        }
        __syncthreads();
        for (int kk = 0; kk < kn; ++kk) {
            float a[4], w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = Xs[kk][ty * 4 + i];
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = Ws[kk][tx * 4 + j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], w[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty * 4 + i;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx * 4 + j;
            if (n >= N) continue;
            float s = acc[i][j];
            if (b) s += b[n];
            if (relu) s = fmaxf(s, 0.f);
            Y[(long long)m * ldy + n] = s;
        }
    }
}

// x [T, D] (this chunk), cache [L-1, D] (previous rows), w [D, L] (conv_left taps, tap j multiplies row
// t - (L-1) + j). One thread per (row, channel). The cache update runs in a second launch (rows must be
// read before they are replaced).
__global__ __launch_bounds__(256) void vad_fsmn_kernel(const float* __restrict__ x, int T, int D,
                                                       const float* __restrict__ cache, const float* __restrict__ w,
                                                       int L, float* __restrict__ y) {
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= (long long)T * D) return;
    const int c = (int)(gid % D);
    const int t = (int)(gid / D);
    float s = 0.f;
    for (int j = 0; j < L; ++j) {
        const int r = t - (L - 1) + j;   // row of the chunk; < 0 -> cache row L-1+r
        const float v = r >= 0 ? x[(long long)r * D + c] : cache[(long long)(L - 1 + r) * D + c];
        s = fmaf(w[c * L + j], v, s);
    }
    y[(long long)t * D + c] = x[(long long)t * D + c] + s;
}

// new cache = last L-1 rows of [cache ; x]
__global__ __launch_bounds__(256) void vad_fsmn_cache_kernel(const float* __restrict__ x, int T, int D,
                                                             const float* __restrict__ cache_old, int L,
                                                             float* __restrict__ cache_new) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (L - 1) * D) return;
    const int r = i / D, c = i % D;
    const int src = T - (L - 1) + r;   // row index into [cache ; x] minus (L-1)
    cache_new[i] = src >= 0 ? x[(long long)src * D + c] : cache_old[(long long)(L - 1 + src) * D + c];
}

__global__ __launch_bounds__(256) void vad_softmax_kernel(const float* __restrict__ logits, int M, int N,
                                                          float* __restrict__ p_sil, float* __restrict__ probs) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float* l = logits + (long long)row * N;
    float mx = -INFINITY;
    for (int j = lane; j < N; j += 64) mx = fmaxf(mx, l[j]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int j = lane; j < N; j += 64) s += expf(l[j] - mx);
    s = wave_sum(s);
    if (probs)
        for (int j = lane; j < N; j += 64) probs[(long long)row * N + j] = expf(l[j] - mx) / s;
    if (lane == 0) p_sil[row] = expf(l[0] - mx) / s;
}

// ComputeDecibel's frame energy (fsmn_vad_streaming/model.py:326-348: 10 log10(sum(frame^2) + 1e-6) over numpy float32
// frames) -- the sum exactly as numpy's float32 add.reduce forms it along a contiguous row: pairwise_sum (blocks of
// <= 128 elements summed by 8 interleaved accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), the tail added in
// order; longer runs split at n/2 rounded down to a multiple of 8), starting from 0, each square rounded before its add
// (contraction off). The log10 stays on the host in numpy (the values it sees are then the reference's bit for bit).
#pragma clang fp contract(off)
__device__ float vad_pw_leaf(const float* x, int n) {
    if (n < 8) {
        float res = 0.f;
        for (int i = 0; i < n; ++i) {
            const float q = x[i] * x[i];
            res = res + q;
        }
        return res;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[j] * x[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float q = x[i + j] * x[i + j];
            r[j] = r[j] + q;
        }
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) {
        const float q = x[i] * x[i];
        res = res + q;
    }
    return res;
}
template <int D> __device__ float vad_pw(const float* x, int n) {
    if (n <= 128) return vad_pw_leaf(x, n);
    if constexpr (D == 0) {
        return __builtin_nanf("");   // deeper than the launcher allows (frame_len <= 2048)
    } else {
        int n2 = n / 2;
        n2 -= n2 % 8;
        const float a = vad_pw<D - 1>(x, n2);
        const float b = vad_pw<D - 1>(x + n2, n - n2);
        return a + b;
    }
}
__global__ __launch_bounds__(256) void vad_frame_energy_kernel(const float* __restrict__ w, int nframes, int fl, int fs,
                                                               float* __restrict__ e) {
    const int f = blockIdx.x * 256 + threadIdx.x;
    if (f < nframes) e[f] = vad_pw<4>(w + (long long)f * fs, fl);
}
#pragma clang fp contract(on)

}  // namespace

hipError_t pfm_vad_frame_energy(const float* wav, int nframes, int fl, int fs, float* e, hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    if (fl < 1 || fl > 2048 || fs < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(vad_frame_energy_kernel, dim3((nframes + 255) / 256), dim3(256), 0, st, wav, nframes, fl, fs, e);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_vad_dense(const float* X, int ldx, int M, int K, const float* W, const float* b, int N, int relu,
                         float* Y, int ldy, hipStream_t st) {
    const long long n = (long long)M * N;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(vad_dense_kernel, dim3((unsigned)((N + VD_TN - 1) / VD_TN), (unsigned)((M + VD_TM - 1) / VD_TM)),
                       dim3(256), 0, st, X, ldx, M, K, W, b, N, relu, Y, ldy);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t pfm_vad_fsmn(const float* x, int T, int D, float* cache, float* cache_tmp, const float* w, int L, float* y,
                        hipStream_t st) {
    if (T <= 0) return hipSuccess;
    const long long n = (long long)T * D;
    hipLaunchKernelGGL(vad_fsmn_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, T, D, cache, w, L, y);
    PFM_LAUNCH_CHECK();
    if (L > 1) {
        const int nc = (L - 1) * D;
        hipLaunchKernelGGL(vad_fsmn_cache_kernel, dim3((nc + 255) / 256), dim3(256), 0, st, x, T, D, cache, L,
                           cache_tmp);
        PFM_LAUNCH_CHECK();
        const hipError_t e = hipMemcpyAsync(cache, cache_tmp, (size_t)nc * 4, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t pfm_vad_softmax(const float* logits, int M, int N, float* p_sil, float* probs, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(vad_softmax_kernel, dim3((M + 3) / 4), dim3(256), 0, st, logits, M, N, p_sil, probs);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
