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

// log1p(u) for u in [0, 1) (u = exp(-|a - b|) of logaddexp): 2 atanh(s), s = u / (2 + u) in [0, 1/3), as a series
// in f64 (terms to s^17: truncation < 2^-34 relative; 1 / (2 + u) by v_rcp_f64 + two Newton steps) rounded once to
// f32 — the correctly rounded value in all but rare halfway cases (the C library's log1pf is within 1 ulp of it),
// at about a tenth of the f32 library routine's instructions
__device__ __forceinline__ float log1p_unit(float u) {
    const double x = (double)u, d = 2.0 + x;
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    const double sd = x * r, z = sd * sd;
    double p = 1.0 / 17.0;
    p = fma(p, z, 1.0 / 15.0);
    p = fma(p, z, 1.0 / 13.0);
    p = fma(p, z, 1.0 / 11.0);
    p = fma(p, z, 1.0 / 9.0);
    p = fma(p, z, 1.0 / 7.0);
    p = fma(p, z, 1.0 / 5.0);
    p = fma(p, z, 1.0 / 3.0);
    p = fma(p, z, 1.0);
    return (float)(2.0 * sd * p);
}

// numpy's npy_logaddexpf (float32): equal operands -> x + ln 2, else max + log1p(exp(-|d|)); branch-free (both
// signs of d in one wave), the same values (a NaN operand still gives NaN through the arithmetic)
__device__ __forceinline__ float lae(float a, float b) {
#pragma clang fp contract(off)
    const float m = a > b ? a : b;
    const float r = m + log1p_unit(expf(-fabsf(a - b)));
    return a == b ? a + 0.693147180559945309417232121458176568f : r;
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
    int wlds;            // the position's ws0 row staged in dynamic LDS (V floats)
};

// (value, index) order of the pre-beam: larger value first, equal values lower index first
__device__ __forceinline__ bool beats(float w, int v, float bw, int bv) { return w > bw || (w == bw && v < bv); }

__global__ __launch_bounds__(NT) void ctc_beam_kernel(BeamArgs a) {
#pragma clang fp contract(off)   // every product rounded before its sum, as the reference's numpy / torch ops
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int V = a.V, K = a.K, P = a.P, Tb = min(a.lens[b], a.T), maxlen = min(a.ntok[b], a.L);
    const int S = a.L + 2;   // yseq capacity: sos + L tokens + eos
    const int kk = min(K, P), KP = K * P;
    const float* am = a.am + (long long)b * a.L * V;
    const float* x = a.x + (long long)b * a.T * V;
    // scratch (floats): Rb [2][T][K*P] float2 | xs [T][P] | xb [T] | Rs [K][T] | bylen [S + 1]
    // The CTC states (r^n, r^b) of position i's candidates are column k*P + j of buffer i & 1 (frame-major: one
    // recurrence step's stores are contiguous across lanes); a running hypothesis is the column it was created in,
    // read from the other buffer at the next position, so nothing is copied between positions.
    float2* Rb = (float2*)(a.fs + b * a.fstride);
    float* xs = (float*)(Rb + 2LL * a.T * KP);
    float* xb = xs + (long long)a.T * P;
    float* Rs = xb + a.T;
    float* bylen = Rs + (long long)K * a.T;
    // (ints): bpar [L][K] parent slot, btok [L][K] token of the hypothesis in beam slot k after position i |
    // has_len [S + 1] (ended lengths reach S) | raw [S] (n-best output staging)
    int* bpar = a.is + b * a.istride;
    int* btok = bpar + (long long)a.L * K;
    int* haslen = btok + (long long)a.L * K;
    int* raw = haslen + S + 1;

    __shared__ int cs[MAXP];
    __shared__ float ws0c[MAXP];
    __shared__ float psi[MAXK][MAXP], wsc[MAXK][MAXP];
    __shared__ float hscore[MAXK], hprev[MAXK];
    __shared__ int hlen[MAXK], hlast[MAXK], hcol[MAXK];   // running beam: length, last token, state column
    __shared__ float nscore[MAXK], nprev[MAXK];
    __shared__ int nsrc[MAXK], ntokn[MAXK], nlen[MAXK];
    __shared__ float csc[MAXK * MAXK];
    __shared__ int csrc[MAXK * MAXK];
    __shared__ float escore[MAXN];
    __shared__ int elen[MAXN], epos[MAXN], epar[MAXN], etok[MAXN], eeos[MAXN];   // n-best list, best first
    __shared__ int nrun, nend, stop;
    __shared__ float best_end;
    __shared__ float redv[2][NT / 64];
    __shared__ int redi[2][NT / 64];
    extern __shared__ float ws0s[];   // [V] when a.wlds
    const bool wlds = a.wlds != 0;

    for (int q = tid; q <= S; q += NT) haslen[q] = 0;
    if (tid == 0) {
        nrun = 1; nend = 0; stop = maxlen < 1; best_end = -INFINITY;
        hscore[0] = 0.f; hprev[0] = 0.f; hlen[0] = 1; hlast[0] = a.sos; hcol[0] = 0;
        // CTCPrefixScore.initial_state (r^n = logzero, r^b = cumulative blank log-probs) as column 0 of buffer 1,
        // the "previous" buffer of position 0
        float rb = 0.f;
        float2* r0 = Rb + (long long)a.T * KP;
        for (int t = 0; t < Tb; ++t) {
            rb = t == 0 ? x[a.blank] : rb + x[(long long)t * V + a.blank];
            r0[(long long)t * KP] = make_float2(LOGZERO, rb);
        }
    }
    for (int t = tid; t < Tb; t += NT) xb[t] = x[(long long)t * V + a.blank];
    __syncthreads();

    for (int i = 0; i < maxlen && !stop; ++i) {
        const float* ami = am + (long long)i * V;
        const int nr = nrun;
        const float2* Rprev = Rb + (long long)((i + 1) & 1) * a.T * KP;
        float2* Rcur = Rb + (long long)(i & 1) * a.T * KP;
        // ---- pre-beam: the top P of ws0 in (value desc, id asc) order. Each thread caches the best of its
        // strided ids; per round the block-wide best is taken and only its owner rescans (for the best element
        // after the taken one in that order)
        if (P == V) {   // no pre-beam: the candidates are the whole vocabulary in id order
            for (int v = tid; v < V; v += NT) { cs[v] = v; ws0c[v] = a.use_pen ? ami[v] + a.pen : ami[v]; }
        } else {
            // ws0 of this position: staged in LDS when the vocabulary fits (the owner rescans read it from there)
            const float* wsrc = ami;
            if (wlds) {
                for (int v = tid; v < V; v += NT) ws0s[v] = a.use_pen ? ami[v] + a.pen : ami[v];
                wsrc = ws0s;
            }
            const bool pen_in = !wlds && a.use_pen;
            float bv = -INFINITY;
            int bi = 0x7fffffff;
            for (int v = tid; v < V; v += NT) {
                const float w = pen_in ? wsrc[v] + a.pen : wsrc[v];
                if (bi == 0x7fffffff || beats(w, v, bv, bi)) { bv = w; bi = v; }
            }
            for (int r = 0; r < P; ++r) {
                float gv = bv;
                int gi = bi;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const float ov = __shfl_xor(gv, o, 64);
                    const int oi = __shfl_xor(gi, o, 64);
                    if (oi != 0x7fffffff && (gi == 0x7fffffff || beats(ov, oi, gv, gi))) { gv = ov; gi = oi; }
                }
                if (lane == 0) { redv[r & 1][wv] = gv; redi[r & 1][wv] = gi; }
                __syncthreads();
                gv = redv[r & 1][0];
                gi = redi[r & 1][0];
#pragma unroll
                for (int q = 1; q < NT / 64; ++q) {
                    const float ov = redv[r & 1][q];
                    const int oi = redi[r & 1][q];
                    if (oi != 0x7fffffff && (gi == 0x7fffffff || beats(ov, oi, gv, gi))) { gv = ov; gi = oi; }
                }
                if (tid == 0) { cs[r] = gi; ws0c[r] = gv; }
                if (gi % NT == tid) {   // owner of the taken id: next best strictly after (gv, gi)
                    bv = -INFINITY;
                    bi = 0x7fffffff;
                    for (int v = tid; v < V; v += NT) {
                        const float w = pen_in ? wsrc[v] + a.pen : wsrc[v];
                        if (!beats(w, v, gv, gi) && !(w == gv && v == gi) && (bi == 0x7fffffff || beats(w, v, bv, bi))) {
                            bv = w;
                            bi = v;
                        }
                    }
                }
            }
        }
        __syncthreads();
        // ---- the candidates' CTC log-probs over the frames, gathered once per position; r_sum of every running
        // hypothesis (logaddexp(r^n, r^b), the log_phi of a non-repeated label)
        {   // 8 gathers in flight per thread
            int e = tid;
            for (; e + 7 * NT < Tb * P; e += 8 * NT) {
                float g8[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int q = e + u * NT, t = q / P, j = q - t * P;
                    g8[u] = x[(long long)t * V + cs[j]];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) xs[e + u * NT] = g8[u];
            }
            for (; e < Tb * P; e += NT) {
                const int t = e / P, j = e - t * P;
                xs[e] = x[(long long)t * V + cs[j]];
            }
        }
        for (int e = tid; e < nr * Tb; e += NT) {
            const int k = e / Tb, t = e - k * Tb;
            const float2 rp = Rprev[(long long)t * KP + hcol[k]];
            Rs[(long long)k * a.T + t] = lae(rp.x, rp.y);
        }
        __syncthreads();
        // ---- CTC prefix scores and weighted scores: one thread per (hypothesis, candidate)
        for (int w = tid; w < nr * P; w += NT) {
            const int k = w / P, j = w - k * P;
            const int c = cs[j];
            const int ol = hlen[k] - 1;                 // output_length (sos ignored)
            const bool phi_b = ol > 0 && c == hlast[k]; // log_phi = r^b(g) for a repeated label
            const float2* rp = Rprev + hcol[k];         // frame t at rp[t * KP]
            const float* rsum = Rs + (long long)k * a.T;
            float2* rn = Rcur + w;
            float r0, r1, lpsi;
            const int start = max(ol, 1);
            if (ol == 0) {
                r0 = xs[j];
                r1 = LOGZERO;
                if (Tb > 0) rn[0] = make_float2(r0, r1);
            } else {
                r0 = LOGZERO;
                r1 = LOGZERO;
                if (ol - 1 < Tb) rn[(long long)(ol - 1) * KP] = make_float2(r0, r1);
            }
            lpsi = r0;   // r[start - 1, 0]
            int t = start;
            // 8 frames per trip: the trip's inputs are loaded together (one memory latency per 8 recurrence steps)
            for (; t + 8 <= Tb; t += 8) {
                float ph[8], xv[8], bq[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    ph[u] = phi_b ? rp[(long long)(t + u - 1) * KP].y : rsum[t + u - 1];
                    xv[u] = xs[(t + u) * P + j];
                    bq[u] = xb[t + u];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float n0 = lae(r0, ph[u]) + xv[u];
                    const float n1 = lae(r0, r1) + bq[u];
                    lpsi = lae(lpsi, ph[u] + xv[u]);
                    r0 = n0;
                    r1 = n1;
                    rn[(long long)(t + u) * KP] = make_float2(r0, r1);
                }
            }
            for (; t < Tb; ++t) {
                const float phi = phi_b ? rp[(long long)(t - 1) * KP].y : rsum[t - 1];
                const float xt = xs[t * P + j];
                const float n0 = lae(r0, phi) + xt;
                const float n1 = lae(r0, r1) + xb[t];
                lpsi = lae(lpsi, phi + xt);
                r0 = n0;
                r1 = n1;
                rn[(long long)t * KP] = make_float2(r0, r1);
            }
            if (c == a.eos) lpsi = Tb > 0 ? rsum[Tb - 1] : LOGZERO;   // r_sum[-1]
            if (c == a.blank) lpsi = LOGZERO;
            psi[k][j] = lpsi;
            const float ts = lpsi - hprev[k];
            wsc[k][j] = (ws0c[j] + a.wctc * ts) + hscore[k];
        }
        __syncthreads();
        // ---- per-hypothesis top kk (descending, equal scores: lower pre-beam rank), appended in hypothesis order
        for (int w = tid; w < nr * P; w += NT) {
            const int k = w / P, j = w - k * P;
            const float v = wsc[k][j];
            int r = 0;
            for (int q = 0; q < P; ++q) r += (wsc[k][q] > v || (wsc[k][q] == v && q < j)) ? 1 : 0;
            if (r < kk) { csc[k * kk + r] = v; csrc[k * kk + r] = w; }
        }
        __syncthreads();
        // ---- sort-and-prune after each hypothesis (search.py:330-332) keeps the top K of all appended candidates in
        // (score desc, append order) order: rank every candidate by counting those before it
        const int nall = nr * kk, nc = min(K, nall);
        for (int q = tid; q < nall; q += NT) {
            const float v = csc[q];
            int g = 0;
            for (int o = 0; o < nall; ++o) g += (csc[o] > v || (csc[o] == v && o < q)) ? 1 : 0;
            if (g < K) {
                const int src = csrc[q], k = src / P, j = src - k * P;
                nscore[g] = v;
                nprev[g] = psi[k][j];
                nsrc[g] = src;
                ntokn[g] = cs[j];
                nlen[g] = hlen[k] + 1;
            }
        }
        __syncthreads();
        // ---- post_process (search.py:401-451): hypotheses ending in <eos> (all of them at the last position, where
        // <eos> is appended) go to the n-best list, the others keep their order on the beam (back-pointers only)
        if (tid == 0) {
            const bool lastpos = i == maxlen - 1;
            int keep = 0;
            for (int q = 0; q < nc; ++q) {
                const int len = nlen[q] + (lastpos ? 1 : 0);
                const int par = nsrc[q] / P;
                if (lastpos || ntokn[q] == a.eos) {
                    const float sc = nscore[q];
                    if (!haslen[len] || sc > bylen[len]) bylen[len] = sc;
                    haslen[len] = 1;
                    best_end = fmaxf(best_end, sc);
                    // n-best list, stable for equal scores (sorted(ended_hyps, reverse=True))
                    int pos = nend < a.nbest ? nend : a.nbest;
                    while (pos > 0 && escore[pos - 1] < sc) --pos;
                    if (pos < a.nbest) {
                        const int last = nend < a.nbest ? nend : a.nbest - 1;
                        for (int e = last; e > pos; --e) {
                            escore[e] = escore[e - 1]; elen[e] = elen[e - 1]; epos[e] = epos[e - 1];
                            epar[e] = epar[e - 1]; etok[e] = etok[e - 1]; eeos[e] = eeos[e - 1];
                        }
                        escore[pos] = sc; elen[pos] = len; epos[pos] = i; epar[pos] = par; etok[pos] = ntokn[q];
                        eeos[pos] = lastpos ? 1 : 0;
                        if (nend < a.nbest) ++nend;
                    }
                } else {
                    hscore[keep] = nscore[q];
                    hprev[keep] = nprev[q];
                    hlen[keep] = nlen[q];
                    hlast[keep] = ntokn[q];
                    hcol[keep] = nsrc[q];
                    bpar[(long long)i * K + keep] = par;
                    btok[(long long)i * K + keep] = ntokn[q];
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
            if (keep == 0) stop = 1;
        }
        __syncthreads();
    }
    // ---- n-best token ids: yseq[1:-1] without eos / sos / blank; the tokens of an ended hypothesis are its own
    // (position epos) and its parent chain's, found by walking the back-pointers
    if (tid == 0) {
        for (int n = 0; n < a.nbest; ++n) {
            int* out = a.tokens + ((long long)b * a.nbest + n) * a.Lcap;
            if (n >= nend) {
                a.olen[b * a.nbest + n] = -1;
                a.oscore[b * a.nbest + n] = -INFINITY;
                continue;
            }
            // raw = y_0 .. y_epos (+ eos): tokens after sos; yseq[1:-1] drops its last element
            const int p = epos[n];
            raw[p] = etok[n];
            int slot = epar[n];
            for (int q = p - 1; q >= 0; --q) {
                raw[q] = btok[(long long)q * K + slot];
                slot = bpar[(long long)q * K + slot];
            }
            const int nraw = p + 1 + eeos[n] - 1;   // elen[n] - 2 elements between sos and the last one
            if (eeos[n]) raw[p + 1] = a.eos;
            int cnt = 0;
            for (int e = 0; e < nraw; ++e) {
                const int tkn = raw[e];
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
    return (2LL * T * K * P * 2 + (long long)T * P + T + (long long)K * T + (L + 3) + 1) & ~1LL;   // even: float2 rows
}
long long pfm_ctc_beam_iscratch(int K, int nbest, int L) { return 2LL * L * K + (L + 3) + (L + 2); }

hipError_t pfm_ctc_beam(const float* am, int L, const float* x, int T, const int* lens, const int* ntok, int B, int V,
                        int K, int P, int nbest, float wctc, float pen, int use_pen, int end_detect, int sos, int eos,
                        int blank, float* fs, int* is, int* tokens, int Lcap, int* olen, float* oscore,
                        hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (K < 1 || K > MAXK || P < 1 || P > MAXP || nbest < 1 || nbest > MAXN || Lcap < 0)
        return hipErrorInvalidValue;
    BeamArgs a;
    a.am = am; a.L = L; a.x = x; a.T = T; a.lens = lens; a.ntok = ntok; a.V = V; a.K = K; a.P = P; a.nbest = nbest;
    a.wctc = wctc; a.pen = pen; a.use_pen = use_pen; a.end_detect = end_detect; a.sos = sos; a.eos = eos;
    a.blank = blank; a.fs = fs; a.is = is; a.fstride = pfm_ctc_beam_fscratch(K, P, T, L);
    a.istride = pfm_ctc_beam_iscratch(K, nbest, L); a.tokens = tokens; a.Lcap = Lcap; a.olen = olen;
    a.oscore = oscore;
    const size_t lds = (size_t)V * sizeof(float);
    a.wlds = lds <= 128 * 1024 ? 1 : 0;
    if (a.wlds) {
        static bool attr = false;
        if (!attr) {
            attr = true;
            (void)hipFuncSetAttribute((const void*)ctc_beam_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
        }
    }
    hipLaunchKernelGGL(ctc_beam_kernel, dim3(B), dim3(NT), a.wlds ? lds : 0, st, a);
    PFM_LAUNCH_CHECK();
    return hipSuccess;
}
