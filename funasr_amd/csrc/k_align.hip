// SenseVoice timestamps on the device: the CTC forced alignment of the greedy transcript
// (funasr/models/sense_voice/model.py:917-928 with ctc_forced_align, funasr/models/sense_voice/utils/
// ctc_alignment.py:2-60).
//
// The reference aligns against the softmax PROBABILITIES of the CTC head (self.ctc.softmax), with the blank
// probability set to 0 on frames whose argmax is the blank, summed along the path in f32 as if they were
// log-probabilities. Per utterance (the reference runs one at a time):
//   ext      = [blank, y1, blank, y2, ..., yL, blank]                       (S = 2L + 1 states)
//   best_0   = (emis[0][blank], emis[0][y1], -inf, ...)
//   best_t[s]= emis[t][ext[s]] + max(best[s], best[s-1], ext[s] != ext[s-2] ? best[s-2] : -inf)
//              (ties to the first of stay / previous / skip, as torch.max(dim=0) on the stacked candidates)
//   end      = 2L - 1 + argmax(best[2L-1], best[2L])   (first on a tie), then back-pointers down to frame 0
// Output: the label id of each frame's state.
#include <hip/hip_runtime.h>

#include "pfm_common.h"

namespace {

constexpr int NT_ST = 256;
constexpr int NT_AL = 1024;

// one workgroup per frame row: row max, first argmax, 1 / sum exp(x - max) (softmax = exp(x - max) * inv)
__global__ __launch_bounds__(NT_ST) void emis_stats_kernel(const float* __restrict__ logits, int V,
                                                         float* __restrict__ mx, float* __restrict__ inv,
                                                         int* __restrict__ amax) {
    const long long r = blockIdx.x;
    const float* row = logits + r * V;
    __shared__ float sv[NT_ST];
    __shared__ int si[NT_ST];
    __shared__ double ss[NT_ST];
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = threadIdx.x; v < V; v += NT_ST) {
        const float x = row[v];
        if (x > bv) { bv = x; bi = v; }   // ascending v per thread: first maximum kept
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int s = NT_ST / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            const float ov = sv[threadIdx.x + s];
            const int oi = si[threadIdx.x + s];
            if (ov > sv[threadIdx.x] || (ov == sv[threadIdx.x] && oi < si[threadIdx.x])) {
                sv[threadIdx.x] = ov;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    const float m = sv[0];
    double sum = 0.0;
    for (int v = threadIdx.x; v < V; v += NT_ST) sum += (double)expf(row[v] - m);
    ss[threadIdx.x] = sum;
    __syncthreads();
    for (int s = NT_ST / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) ss[threadIdx.x] += ss[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        mx[r] = m;
        inv[r] = 1.f / (float)ss[0];
        amax[r] = si[0] == 0x7fffffff ? 0 : si[0];
    }
}

struct AlignArgs {
    const float* logits;   // [B * Tf][V] rows of the speech frames (frame t of utterance b at row b * Tf + t)
    const float* mx;
    const float* inv;
    const int* amax;
    int Tf, V, blank;
    const int* olen;       // [B] encoder_out_lens (query rows + speech frames): speech frames = olen - 4
    const int* tg;         // [B][Lmax] target ids (token_int[4:])
    const int* tlen;       // [B]
    int Lmax;
    unsigned char* bp;     // [B][Tf][2 Lmax + 1] back-pointers
    int* align;            // [B][Tf] out (-1 beyond the utterance's frames)
};

__device__ __forceinline__ float emis(const AlignArgs& a, long long row, int tok) {
    if (tok == a.blank && a.amax[row] == a.blank) return 0.f;   // logits_speech[pred == blank, blank] = 0
    return expf(a.logits[row * a.V + tok] - a.mx[row]) * a.inv[row];
}

__global__ __launch_bounds__(NT_AL) void ctc_align_kernel(AlignArgs a) {
#pragma clang fp contract(off)
    extern __shared__ float sm[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int Tp = min(a.olen[b] - 4, a.Tf), L = a.Lmax > 0 ? min(a.tlen[b], a.Lmax) : 0, S = 2 * L + 1;
    const int Smax = 2 * a.Lmax + 1;
    const int* tg = a.tg + (long long)b * a.Lmax;
    int* out = a.align + (long long)b * a.Tf;
    for (int t = tid; t < a.Tf; t += NT_AL) out[t] = -1;
    if (Tp <= 0) return;
    float* cur = sm;                 // padded scores: cur[2 + s] = state s, cur[0..1] = -inf
    float* nxt = sm + Smax + 2;
    auto ext = [&](int s) { return (s & 1) ? tg[s >> 1] : a.blank; };
    const long long row0 = (long long)b * a.Tf;
    for (int s = tid; s < S + 2; s += NT_AL) {
        float v = -INFINITY;
        if (s == 2) v = emis(a, row0, a.blank);
        if (s == 3 && S > 1) v = emis(a, row0, ext(1));
        cur[s] = v;
        nxt[s] = -INFINITY;
    }
    __syncthreads();
    unsigned char* bp = a.bp + (long long)b * a.Tf * Smax;
    for (int t = 1; t < Tp; ++t) {
        const long long row = row0 + t;
        for (int s = tid; s < S; s += NT_AL) {
            const float c0 = cur[2 + s], c1 = cur[1 + s];
            const float c2 = (s >= 2 && ext(s) != ext(s - 2)) ? cur[s] : -INFINITY;
            float v = c0;
            int idx = 0;
            if (c1 > v) { v = c1; idx = 1; }
            if (c2 > v) { v = c2; idx = 2; }
            nxt[2 + s] = emis(a, row, ext(s)) + v;
            bp[(long long)t * Smax + s] = (unsigned char)idx;
        }
        __syncthreads();
        float* tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    if (tid == 0) {
        // end state (padded coordinates): the last label (2L - 1) or the final blank (2L), first on a tie
        const float l1 = 2 * L - 1 >= 0 ? cur[2 + 2 * L - 1] : -INFINITY, l2 = cur[2 + 2 * L];
        int p = 2 + 2 * L - 1 + (l2 > l1 ? 1 : 0);
        out[Tp - 1] = ext(max(p - 2, 0));
        for (int t = Tp - 1; t > 0; --t) {
            const int s = p - 2;
            p -= s >= 0 ? (int)bp[(long long)t * Smax + s] : 0;
            out[t - 1] = ext(max(p - 2, 0));
        }
    }
}

}  // namespace

hipError_t pfm_emis_stats(const float* logits, long long rows, int V, float* mx, float* inv, int* amax, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(emis_stats_kernel, dim3((unsigned)rows), dim3(NT_ST), 0, st, logits, V, mx, inv, amax);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// logits [B * Tf][V]; scratch bp of B * Tf * (2 Lmax + 1) bytes
hipError_t pfm_ctc_align_run(const float* logits, const float* mx, const float* inv, const int* amax, int B, int Tf,
                             int V, int blank, const int* olen, const int* tg, const int* tlen, int Lmax,
                             unsigned char* bp, int* align, hipStream_t st) {
    if (B <= 0 || Tf <= 0) return hipSuccess;
    const size_t lds = (size_t)2 * (2 * Lmax + 3) * sizeof(float);
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    AlignArgs a;
    a.logits = logits; a.mx = mx; a.inv = inv; a.amax = amax; a.Tf = Tf; a.V = V; a.blank = blank; a.olen = olen;
    a.tg = tg; a.tlen = tlen; a.Lmax = Lmax; a.bp = bp; a.align = align;
    hipLaunchKernelGGL(ctc_align_kernel, dim3(B), dim3(NT_AL), lds, st, a);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
