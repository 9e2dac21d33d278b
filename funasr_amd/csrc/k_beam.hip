// Joint decoder / CTC prefix beam search of Paraformer (BeamSearchPara, funasr/models/paraformer/search.py:35-451,
// with the CTCPrefixScorer of transformer/scorers/ctc.py:10-80 over CTCPrefixScore,
// transformer/scorers/ctc_prefix_score.py:255-337, and the LengthBonus full scorer), run on the device: one
// workgroup per utterance walks the decoder positions, all of its hypotheses and candidates in parallel.
//
// Per position i (search.py:281-333) for every running hypothesis h (score s_h, CTC state r_h[T][2], CTC prefix
// score p_h):
//   ws0[v]   = am[i][v] (+ penalty)                  the decoder log-probs (+ LengthBonus)
//   cands    = top-P of ws0 (P = int(1.5 beam), the same set for every h: pre-beam key "full")
//   psi[h,c] = CTC prefix log-probability of h + c (Algorithm 2 of the hybrid CTC/attention paper, as
//              CTCPrefixScore.__call__: forward variables r^n, r^b over the utterance's frames)
//   ws[h,c]  = (ws0[c] + w_ctc (psi[h,c] - p_h)) + s_h        (f32, the reference's operation order)
//   the best `beam` candidates of each h, appended in hypothesis order, are stable-sorted by ws and pruned to
//   `beam`; at the last position <eos> is appended; hypotheses ending in <eos> move to the ended list;
//   end detection (metrics/common.py:18-46, M = 3, D_end = -10) stops the search.
// The n-best ended hypotheses (stable order for equal scores) are written as token ids without sos / eos /
// blank (paraformer/model.py:553-565).
//
// All arithmetic is f32 like the reference (numpy float32 state arrays, torch f32 scores); logaddexp follows
// numpy's float32 npy_logaddexpf (equal operands -> x + ln 2, else max + log1p(exp(-|d|))).
#include "pfm_common.h"

#include <hip/hip_runtime.h>

namespace {

constexpr float LOGZERO = -10000000000.0f;   // CTCPrefixScore.logzero
constexpr float D_END = -10.0f;              // end_detect D_end = log(1 * exp(-10))
constexpr int NT = 256;
constexpr int MAXK = 16;                     // beam
constexpr int MAXP = 64;                     // pre-beam candidates (int(1.5 beam), or the vocabulary without pre-beam)
constexpr int MAXN = 16;                     // n-best

__device__ __forceinline__ float lae(float a, float b) {
#pragma clang fp contract(off)
    if (a == b) return a + 0.693147180559945309417232121458176568f;
    const float d = a - b;
    if (d > 0.f) return a + log1pf(expf(-d));
    if (d <= 0.f) return b + log1pf(expf(d));
    return d;   // nan
}

// row-wise log_softmax in place: x[r][0..V) -> x - max - log(sum exp(x - max)) (sum in f64)
__global__ __launch_bounds__(256) void logsoftmax_rows_kernel(float* __restrict__ x, long long ld, int V) {
#pragma clang fp contract(off)
    float* row = x + (long long)blockIdx.x * ld;
    __shared__ float smx[256];
    __shared__ double ssm[256];
    float mx = -INFINITY;
    for (int v = threadIdx.x; v < V; v += 256) mx = fmaxf(mx, row[v]);
    smx[threadIdx.x] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + s]);
        __syncthreads();
    }
    mx = smx[0];
    double sm = 0.0;
    for (int v = threadIdx.x; v < V; v += 256) sm += exp((double)row[v] - (double)mx);
    ssm[threadIdx.x] = sm;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) ssm[threadIdx.x] += ssm[threadIdx.x + s];
        __syncthreads();
    }
    const float lse = (float)log(ssm[0]);
    for (int v = threadIdx.x; v < V; v += 256) row[v] = (row[v] - mx) - lse;
}

struct BeamArgs {
    const float* am;     // [B][L][V] decoder log-probs
    int L;
    const float* x;      // [B][T][V] CTC log-probs
    int T;
    const int* lens;     // [B] frames of each utterance (encoder_out_lens)
    const int* ntok;     // [B] decoder positions (pre_token_length)
    int V, K, P, nbest;
    float wctc, pen;
    int use_pen, end_detect;
    int sos, eos, blank;
    float* fs;           // per-utterance float scratch (fstride floats)
    int* is;             // per-utterance int scratch (istride ints)
    long long fstride, istride;
    int* tokens;         // [B][nbest][Lcap]
    int Lcap;
    int* olen;           // [B][nbest] token count of each n-best hypothesis, -1 = none
    float* oscore;       // [B][nbest]
};

__global__ __launch_bounds__(NT) void ctc_beam_kernel(BeamArgs a) {
#pragma clang fp contract(off)   // every product rounded before its sum, as the reference's numpy / torch ops
    const int b = blockIdx.x, tid = threadIdx.x;
    const int V = a.V, K = a.K, P = a.P, Tb = min(a.lens[b], a.T), maxlen = min(a.ntok[b], a.L);
    const int S = a.L + 2;   // yseq capacity: sos + L tokens + eos
    const float* am = a.am + (long long)b * a.L * V;
    const float* x = a.x + (long long)b * a.T * V;
    // scratch layout (floats): Rcur [K][T][2] | Rnew [K][P][T][2] | xs [T][P] | xb [T] | best_by_len [S + 1]
    float* Rcur = a.fs + b * a.fstride;
    float* Rnew = Rcur + (long long)K * a.T * 2;
    float* xs = Rnew + (long long)K * P * a.T * 2;
    float* xb = xs + (long long)a.T * P;
    float* bylen = xb + a.T;
    // (ints): ycur [K][S] | ynew [K][S] | yend [nbest][S] | has_len [S + 1] (ended lengths reach S)
    int* ycur = a.is + b * a.istride;
    int* ynew = ycur + K * S;
    int* yend = ynew + K * S;
    int* haslen = yend + a.nbest * S;

    __shared__ int cs[MAXP];
    __shared__ float ws0c[MAXP];
    __shared__ float psi[MAXK][MAXP];
    __shared__ float hscore[MAXK], hprev[MAXK];
    __shared__ int hlen[MAXK], nlen[MAXK];
    __shared__ float nscore[MAXK], nprev[MAXK];
    __shared__ int nsrc[MAXK], ntokn[MAXK];            // new hypothesis: source (k * P + j), appended token
    __shared__ float cscore[MAXK * MAXK];
    __shared__ int cidx[MAXK * MAXK];
    __shared__ float escore[MAXN];
    __shared__ int elen[MAXN];
    __shared__ int nrun, nend, stop;
    __shared__ float best_end;
    __shared__ float redv[NT];
    __shared__ int redi[NT];

    for (int s = tid; s <= S; s += NT) haslen[s] = 0;
    if (tid == 0) {
        nrun = 1; nend = 0; stop = maxlen < 1; best_end = -INFINITY;
        hscore[0] = 0.f; hprev[0] = 0.f; hlen[0] = 1;
        ycur[0] = a.sos;
        // CTCPrefixScore.initial_state: r^n = logzero, r^b = cumulative blank log-probs
        float rb = 0.f;
        for (int t = 0; t < Tb; ++t) {
            rb = t == 0 ? x[a.blank] : rb + x[(long long)t * V + a.blank];
            Rcur[2 * t] = LOGZERO;
            Rcur[2 * t + 1] = rb;
        }
    }
    for (int t = tid; t < Tb; t += NT) xb[t] = x[(long long)t * V + a.blank];
    __syncthreads();

    for (int i = 0; i < maxlen && !stop; ++i) {
        const float* ami = am + (long long)i * V;
        // ---- pre-beam: top-P of ws0 (descending; equal values: lower id first)
        for (int r = 0; r < P; ++r) {
            float bv = -INFINITY;
            int bi = 0x7fffffff;
            if (P == V) {   // no pre-beam: the candidates are the whole vocabulary in id order
                if (tid == 0) { cs[r] = r; ws0c[r] = a.use_pen ? ami[r] + a.pen : ami[r]; }
                continue;
            }
            for (int v = tid; v < V; v += NT) {
                bool taken = false;
                for (int q = 0; q < r; ++q) taken |= cs[q] == v;
                const float w = a.use_pen ? ami[v] + a.pen : ami[v];
                if (!taken && (w > bv || (w == bv && v < bi))) { bv = w; bi = v; }
            }
            redv[tid] = bv;
            redi[tid] = bi;
            __syncthreads();
            for (int s = NT / 2; s > 0; s >>= 1) {
                if (tid < s) {
                    const float ov = redv[tid + s];
                    const int oi = redi[tid + s];
                    if (ov > redv[tid] || (ov == redv[tid] && oi < redi[tid])) { redv[tid] = ov; redi[tid] = oi; }
                }
                __syncthreads();
            }
            if (tid == 0) { cs[r] = redi[0]; ws0c[r] = redv[0]; }
            __syncthreads();
        }
        __syncthreads();
        // ---- the candidates' CTC log-probs over the frames, gathered once per position
        for (int e = tid; e < Tb * P; e += NT) {
            const int t = e / P, j = e - t * P;
            xs[e] = x[(long long)t * V + cs[j]];
        }
        __syncthreads();
        // ---- CTC prefix scores: one thread per (hypothesis, candidate)
        for (int w = tid; w < nrun * P; w += NT) {
            const int k = w / P, j = w - k * P;
            const int c = cs[j];
            const int ol = hlen[k] - 1;                 // output_length (sos ignored)
            const int last = ycur[k * S + hlen[k] - 1];
            const bool phi_b = ol > 0 && c == last;     // log_phi = r^b(g) for a repeated label
            const float* rp = Rcur + (long long)k * a.T * 2;
            float* rn = Rnew + ((long long)k * P + j) * a.T * 2;
            float r0, r1, lpsi;
            const int start = max(ol, 1);
            if (ol == 0) {
                r0 = xs[j];
                r1 = LOGZERO;
                if (Tb > 0) { rn[0] = r0; rn[1] = r1; }
            } else {
                r0 = LOGZERO;
                r1 = LOGZERO;
                if (ol - 1 < Tb) { rn[2 * (ol - 1)] = r0; rn[2 * (ol - 1) + 1] = r1; }
            }
            lpsi = r0;   // r[start - 1, 0]
            for (int t = start; t < Tb; ++t) {
                const float pn = rp[2 * (t - 1)], pb = rp[2 * (t - 1) + 1];
                const float phi = phi_b ? pb : lae(pn, pb);
                const float xt = xs[t * P + j];
                const float n0 = lae(r0, phi) + xt;
                const float n1 = lae(r0, r1) + xb[t];
                lpsi = lae(lpsi, phi + xt);
                r0 = n0;
                r1 = n1;
                rn[2 * t] = r0;
                rn[2 * t + 1] = r1;
            }
            if (c == a.eos) lpsi = Tb > 0 ? lae(rp[2 * (Tb - 1)], rp[2 * (Tb - 1) + 1]) : LOGZERO;   // r_sum[-1]
            if (c == a.blank) lpsi = LOGZERO;
            psi[k][j] = lpsi;
        }
        __syncthreads();
        // ---- scores, per-hypothesis beam, stable global prune (thread 0: at most beam x beam candidates)
        if (tid == 0) {
            int nc = 0;
            for (int k = 0; k < nrun; ++k) {
                float ws[MAXP];
                for (int j = 0; j < P; ++j) {
                    const float ts = psi[k][j] - hprev[k];
                    ws[j] = (ws0c[j] + a.wctc * ts) + hscore[k];
                }
                bool used[MAXP];
                for (int j = 0; j < P; ++j) used[j] = false;
                const int kk = min(K, P);
                for (int r = 0; r < kk; ++r) {   // top-beam of this hypothesis, descending
                    int bj = -1;
                    for (int j = 0; j < P; ++j)
                        if (!used[j] && (bj < 0 || ws[j] > ws[bj])) bj = j;   // equal: lower pre-beam rank
                    used[bj] = true;
                    // stable insertion into the running candidate list (sorted descending)
                    int pos = nc;
                    while (pos > 0 && cscore[pos - 1] < ws[bj]) {
                        cscore[pos] = cscore[pos - 1];
                        cidx[pos] = cidx[pos - 1];
                        --pos;
                    }
                    cscore[pos] = ws[bj];
                    cidx[pos] = k * P + bj;
                    ++nc;
                }
                if (nc > K) nc = K;   // search.py:330-332: sort and prune after each hypothesis
            }
            for (int s = 0; s < nc; ++s) {
                const int k = cidx[s] / P, j = cidx[s] - k * P;
                nscore[s] = cscore[s];
                nprev[s] = psi[k][j];
                nsrc[s] = cidx[s];
                ntokn[s] = cs[j];
                nlen[s] = hlen[k] + 1;
            }
            nrun = nc;
        }
        __syncthreads();
        // ---- materialise the new hypotheses: yseq = parent's + token (+ eos at the last position), CTC state
        const bool lastpos = i == maxlen - 1;
        for (int s = 0; s < nrun; ++s) {
            const int k = nsrc[s] / P;
            for (int e = tid; e < nlen[s] - 1; e += NT) ynew[s * S + e] = ycur[k * S + e];
            if (tid == 0) {
                ynew[s * S + nlen[s] - 1] = ntokn[s];
                if (lastpos) ynew[s * S + nlen[s]] = a.eos;
            }
            const float* src = Rnew + (long long)nsrc[s] * a.T * 2;
            float* dst = Rcur + (long long)s * a.T * 2;
            for (int e = tid; e < 2 * Tb; e += NT) dst[e] = src[e];
        }
        __syncthreads();
        // ---- post_process (search.py:401-451): ended hypotheses leave the beam; end detection
        if (tid == 0) {
            int keep = 0;
            for (int s = 0; s < nrun; ++s) {
                const int len = nlen[s] + (lastpos ? 1 : 0);
                const int lastt = ynew[s * S + len - 1];
                if (lastt == a.eos) {
                    const float sc = nscore[s];
                    if (!haslen[len] || sc > bylen[len]) bylen[len] = sc;
                    haslen[len] = 1;
                    best_end = fmaxf(best_end, sc);
                    // n-best list, stable for equal scores (sorted(ended_hyps, reverse=True))
                    int pos = nend < a.nbest ? nend : a.nbest;
                    while (pos > 0 && escore[pos - 1] < sc) --pos;
                    if (pos < a.nbest) {
                        const int last = (nend < a.nbest ? nend : a.nbest - 1);
                        for (int q = last; q > pos; --q) {
                            escore[q] = escore[q - 1];
                            elen[q] = elen[q - 1];
                            for (int e = 0; e < elen[q]; ++e) yend[q * S + e] = yend[(q - 1) * S + e];
                        }
                        escore[pos] = sc;
                        elen[pos] = len;
                        for (int e = 0; e < len; ++e) yend[pos * S + e] = ynew[s * S + e];
                        if (nend < a.nbest) ++nend;
                    }
                } else {   // stays on the beam: compact in order (slot keep <= s)
                    if (keep != s) {
                        for (int e = 0; e < nlen[s]; ++e) ynew[keep * S + e] = ynew[s * S + e];
                        float* dst = Rcur + (long long)keep * a.T * 2;
                        const float* src = Rcur + (long long)s * a.T * 2;
                        for (int e = 0; e < 2 * Tb; ++e) dst[e] = src[e];
                    }
                    hscore[keep] = nscore[s];
                    hprev[keep] = nprev[s];
                    hlen[keep] = nlen[s];
                    ++keep;
                }
            }
            nrun = keep;
            if (a.end_detect && nend > 0) {   // metrics/common.py:18-46
                int count = 0;
                for (int m = 0; m < 3; ++m) {
                    const int hl = i - m;
                    if (hl >= 0 && hl <= S && haslen[hl] && bylen[hl] - best_end < D_END) ++count;
                }
                if (count == 3) stop = 1;
            }
            if (nrun == 0) stop = 1;
        }
        __syncthreads();
        // ynew -> ycur for the survivors
        for (int s = 0; s < nrun; ++s)
            for (int e = tid; e < hlen[s]; e += NT) ycur[s * S + e] = ynew[s * S + e];
        __syncthreads();
    }
    // ---- n-best token ids: yseq[1:-1] without eos / sos / blank
    if (tid == 0) {
        for (int n = 0; n < a.nbest; ++n) {
            int* out = a.tokens + ((long long)b * a.nbest + n) * a.Lcap;
            if (n >= nend) {
                a.olen[b * a.nbest + n] = -1;
                a.oscore[b * a.nbest + n] = -INFINITY;
                continue;
            }
            int cnt = 0;
            for (int e = 1; e < elen[n] - 1; ++e) {
                const int tkn = yend[n * S + e];
                if (tkn == a.eos || tkn == a.sos || tkn == a.blank) continue;
                if (cnt < a.Lcap) out[cnt] = tkn;
                ++cnt;
            }
            a.olen[b * a.nbest + n] = cnt;
            a.oscore[b * a.nbest + n] = escore[n];
        }
    }
}

}  // namespace

hipError_t pfm_logsoftmax_rows(float* x, long long rows, long long ld, int V, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(logsoftmax_rows_kernel, dim3((unsigned)rows), dim3(256), 0, st, x, ld, V);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}

// scratch sizes per utterance for pfm_ctc_beam
long long pfm_ctc_beam_fscratch(int K, int P, int T, int L) {
    return (long long)K * T * 2 + (long long)K * P * T * 2 + (long long)T * P + T + (L + 3);
}
long long pfm_ctc_beam_iscratch(int K, int nbest, int L) { return (long long)(2 * K + nbest) * (L + 2) + (L + 3); }

hipError_t pfm_ctc_beam(const float* am, int L, const float* x, int T, const int* lens, const int* ntok, int B, int V,
                        int K, int P, int nbest, float wctc, float pen, int use_pen, int end_detect, int sos, int eos,
                        int blank, float* fs, int* is, int* tokens, int Lcap, int* olen, float* oscore,
                        hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (K < 1 || K > MAXK || P < 1 || P > MAXP || nbest < 1 || nbest > MAXN || nbest > K || Lcap < 0)
        return hipErrorInvalidValue;
    BeamArgs a;
    a.am = am; a.L = L; a.x = x; a.T = T; a.lens = lens; a.ntok = ntok; a.V = V; a.K = K; a.P = P; a.nbest = nbest;
    a.wctc = wctc; a.pen = pen; a.use_pen = use_pen; a.end_detect = end_detect; a.sos = sos; a.eos = eos;
    a.blank = blank; a.fs = fs; a.is = is; a.fstride = pfm_ctc_beam_fscratch(K, P, T, L);
    a.istride = pfm_ctc_beam_iscratch(K, nbest, L); a.tokens = tokens; a.Lcap = Lcap; a.olen = olen;
    a.oscore = oscore;
    hipLaunchKernelGGL(ctc_beam_kernel, dim3(B), dim3(NT), 0, st, a);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
