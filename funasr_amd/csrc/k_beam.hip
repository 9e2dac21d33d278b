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
#include <cstdlib>

#include "pfm_common.h"

#include <hip/hip_runtime.h>

namespace {

constexpr float LOGZERO = -10000000000.0f;   // CTCPrefixScore.logzero
constexpr float D_END = -10.0f;              // end_detect D_end = log(1 * exp(-10))
constexpr int NT = 256;
constexpr int MAXK = 16;                     // beam
constexpr int MAXP = 64;                     // pre-beam candidates (int(1.5 beam), or the vocabulary without pre-beam)
constexpr int MAXN = 16;                     // n-best

// Phase timing of the search (tools/beam_bench.hip builds with -DBEAM_PROF; the library never does): thread 0 of every
// workgroup adds the wall-clock ticks of each phase of every position and writes them to beam_prof[b][8] at the end.
#ifdef BEAM_PROF
__device__ unsigned long long beam_prof[1024][8];
#define BPROF_MARK(k) do { if (tid == 0) { const unsigned long long n_ = wall_clock64(); pt[k] += n_ - pt_last; pt_last = n_; } } while (0)
#else
#define BPROF_MARK(k) do { } while (0)
#endif

// log1p(u) for u in [0, 1) (u = exp(-|a - b|) of logaddexp): 2 atanh(s), s = u / (2 + u) in [0, 1/3), as a series
// in f64 (terms to s^17: truncation < 2^-34 relative; 1 / (2 + u) by v_rcp_f64 (2^-23) + one Newton step (2^-46))
// rounded once to f32 — the correctly rounded value in all but rare near-halfway cases (the C library's log1pf is
// within 1 ulp of it), at about a tenth of the f32 library routine's instructions. The series in z = s^2 is evaluated
// in Estrin form (four dependent FMA levels instead of Horner's eight: logaddexp is the step of every sequential
// recurrence of the search, so its dependency depth is the search's clock)
// a * b + c as one VOP3 v_fma_f64 (the compiler's two-address v_fmac_f64 form copies the loop-invariant addend into
// the destination first: one v_mov_b64 per Horner step)
__device__ __forceinline__ double fma64(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

__device__ __forceinline__ float log1p_unit(float u) {
    const double x = (double)u, d = 2.0 + x;
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    const double sd = x * r, z = sd * sd, z2 = z * z, z4 = z2 * z2, z8 = z4 * z4;
    const double q0 = fma64(z, 1.0 / 3.0, 1.0), q1 = fma64(z, 1.0 / 7.0, 1.0 / 5.0);
    const double q2 = fma64(z, 1.0 / 11.0, 1.0 / 9.0), q3 = fma64(z, 1.0 / 15.0, 1.0 / 13.0);
    const double h0 = fma64(q1, z2, q0), h1 = fma64(q3, z2, q2);
    const double p = fma64(1.0 / 17.0, z8, fma64(h1, z4, h0));
    return (float)(2.0 * sd * p);
}

// log1p(u) for u in (0, 1] by a 65-entry table in LDS (tools/beam_bench.hip -DBEAM_LOG1P_TABLE, diagnostic): i =
// floor(64 u), r = (u - i/64) / (1 + i/64) in [0, 1/64) (the difference exact), log1p(u) = log(1 + i/64) + log1p(r)
// with a degree-6 polynomial in f64, rounded once to f32
__device__ __forceinline__ float log1p_table(float u, const double2* __restrict__ tab) {
    const int i = (int)(u * 64.f);
    const double2 e = tab[i];   // {1 / (1 + i/64), log(1 + i/64)}
    const double r = ((double)u - (double)i * 0.015625) * e.x;
    double q = fma(r, -1.0 / 6.0, 1.0 / 5.0);
    q = fma(q, r, -0.25);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    q = fma(q, r, 1.0);
    return (float)fma(q, r, e.y);
}

// numpy's npy_logaddexpf (float32): equal operands -> x + ln 2, else max + log1p(exp(-|d|)); branch-free (both
// signs of d in one wave), the same values (a NaN operand still gives NaN through the arithmetic)
__device__ __forceinline__ float lae(float a, float b, const double2* tab = nullptr) {
#pragma clang fp contract(off)
    const float m = a > b ? a : b;
#ifdef BEAM_LOG1P_TABLE
    const float r = m + log1p_table(expf(-fabsf(a - b)), tab);
#else
    (void)tab;
    const float r = m + log1p_unit(expf(-fabsf(a - b)));
#endif
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
    int L;               // decoder positions per utterance in the decoder log-probs
    int T;               // frames per utterance in the CTC log-probs (the transposed copy at the head of fs)
    const int* lens;     // [B] frames of each utterance (encoder_out_lens)
    const int* ntok;     // [B] decoder positions (pre_token_length)
    int V, K, P, nbest;
    float wctc, pen;
    int use_pen, end_detect;
    int sos, eos, blank;
    float* fs;           // per-utterance float scratch (fstride floats): the CTC log-probs transposed, [V][T], first
    int* is;             // per-utterance int scratch (istride ints)
    long long fstride, istride;
    int* tokens;         // [B][nbest][Lcap]
    int Lcap;
    int* olen;           // [B][nbest] token count of each n-best hypothesis, -1 = none
    float* oscore;       // [B][nbest]
    int B, G, Gr;        // utterances; workgroups per utterance (Gr pair workgroups, then the log-psi ones)
    unsigned spin_cap;   // arrival-barrier wait bound (s_sleep rounds); past it the search fails (fail word set)
};

// Workgroups of one search (BeamSearchPara of one utterance). The prefix recurrences of position i are three
// independent f32 chains per (hypothesis k, candidate j) = column c = kP + j over the frames: r^n (its own previous
// value), r^b (the previous r^n and r^b) and log psi (an accumulation of phi + x). Each is one logaddexp per frame;
// the recurrence is instruction-issue bound, so the columns' chains are spread over the SIMDs of several CUs:
//   pair workgroup g < Gr: columns [128 g, 128 g + 128): waves 0-1 run r^n, waves 2-3 run r^b one block of BL frames
//     behind (r^n of the block before comes through LDS, one barrier per block);
//   log-psi workgroup g >= Gr: columns [256 (g - Gr), +256): log psi, then psi and the weighted score of the column.
// Every workgroup of an utterance keeps the whole search state (the pre-beam, the beam, the n-best list) and runs the
// selection steps redundantly on identical data; the columns' scores and the states cross workgroups through global
// memory and one arrival barrier per position. All workgroups of an utterance sit on one XCD (same L2).
#ifndef BEAM_BL
#define BEAM_BL 16
#endif
// frames per r^n -> r^b hand-off block (a multiple of 8): the r^b chains start one block late, so a position costs
// nblk + 1 rounds of BL frames; 16 measured best (21.4 ms per B = 64 batch vs 22.0 at 32 and 22.1 at 8: more rounds,
// more barriers)
constexpr int BL = BEAM_BL;
static_assert(BL % 8 == 0 && BL <= 32, "hand-off block");

__host__ __device__ __forceinline__ long long pfm_align2(long long n) { return (n + 1) & ~1LL; }   // float2 rows

// (value, index) order of the pre-beam: larger value first, equal values lower index first
__device__ __forceinline__ bool beats(float w, int v, float bw, int bv) { return w > bw || (w == bw && v < bv); }

__global__ __launch_bounds__(NT) void ctc_beam_kernel(BeamArgs a) {
#pragma clang fp contract(off)   // every product rounded before its sum, as the reference's numpy / torch ops
    // block -> (utterance b, role grp): the G workgroups of b share blockIdx mod 8 (one XCD)
    const int tid = threadIdx.x;
    const int per = 8 * a.G, chunk = blockIdx.x / per, within = blockIdx.x - chunk * per;
    const int grp = within >> 3, b = chunk * 8 + (within & 7);
    if (b >= a.B) return;
    const bool pairw = grp < a.Gr;
    const int V = a.V, K = a.K, P = a.P, Tb = min(a.lens[b], a.T), maxlen = min(a.ntok[b], a.L);
    const int S = a.L + 2;   // yseq capacity: sos + L tokens + eos
    const int kk = min(K, P), KP = K * P;
    // scratch (floats): xt [V][T] (the utterance's CTC log-probs, frame-contiguous per id: a candidate's column over the
    // frames is one contiguous row) | Rb [2][T][K*P] float2 | xch [2][2][K*P] (the columns' weighted scores and psi,
    // per position parity) | Rsum [2][T][K*P] (r_sum = logaddexp(r^n, r^b) of every column, written by the r^b chains
    // as they go: a running hypothesis's r_sum at the next position is its column there) | per workgroup: bylen [S + 1]
    // The CTC states (r^n, r^b) of position i's candidates are column k*P + j of buffer i & 1 (frame-major: one
    // recurrence step's stores are contiguous across lanes); a running hypothesis is the column it was created in,
    // read from the other buffer at the next position, so nothing is copied between positions.
    const float* xt = a.fs + b * a.fstride;
    const float* xb = xt + (long long)a.blank * a.T;   // the blank's row
    float2* Rb = (float2*)(a.fs + b * a.fstride + pfm_align2((long long)V * a.T));
    float* xch = (float*)(Rb + 2LL * a.T * KP);
    float* Rsum = xch + 4LL * KP;
    float* bylen = Rsum + 2LL * a.T * KP + (long long)grp * (S + 1);
    // (ints): bpar [L][K] parent slot, btok [L][K] token of the hypothesis in beam slot k after position i (written
    // by workgroup 0) | raw [S] (n-best output staging) | per workgroup: has_len [S + 1] (ended lengths reach S)
    unsigned* sync = (unsigned*)(a.is + b * a.istride);   // [0]: arrivals of the per-position barrier, [1]: timeout
    int* bpar = a.is + b * a.istride + 2;
    int* btok = bpar + (long long)a.L * K;
    int* raw = btok + (long long)a.L * K;
    int* haslen = raw + S + (long long)grp * (S + 1);

    __shared__ int cs[MAXP];
    __shared__ float ws0c[MAXP];
    __shared__ float psi[MAXK][MAXP];
    __shared__ __attribute__((aligned(16))) float wsc[MAXK][MAXP];
    __shared__ float hscore[MAXK], hprev[MAXK];
    __shared__ int hlen[MAXK], hlast[MAXK], hcol[MAXK];   // running beam: length, last token, state column
    __shared__ float nscore[MAXK], nprev[MAXK];
    __shared__ int nsrc[MAXK], ntokn[MAXK], nlen[MAXK];
    __shared__ __attribute__((aligned(16))) float csc[MAXK * MAXK];
    __shared__ int csrc[MAXK * MAXK];
    __shared__ float escore[MAXN];
    __shared__ int elen[MAXN], epos[MAXN], epar[MAXN], etok[MAXN], eeos[MAXN];   // n-best list, best first
    __shared__ int nrun, nend, stop;
    __shared__ float best_end;
    __shared__ float lag[2][BL][128];   // pair workgroups: r^n of the last two blocks of frames per column
    __shared__ double2 l1p[65];
    if (tid < 65) l1p[tid] = make_double2(1.0 / (1.0 + tid / 64.0), log(1.0 + tid / 64.0));

#ifdef BEAM_PROF
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt_last = wall_clock64();
#endif
    for (int q = tid; q <= S; q += NT) haslen[q] = 0;
    if (tid == 0) {
        nrun = 1; nend = 0; stop = maxlen < 1; best_end = -INFINITY;
        hscore[0] = 0.f; hprev[0] = 0.f; hlen[0] = 1; hlast[0] = a.sos; hcol[0] = 0;
        // CTCPrefixScore.initial_state (r^n = logzero, r^b = cumulative blank log-probs) as column 0 of buffer 1,
        // the "previous" buffer of position 0
        float rb = 0.f;
        float2* r0 = Rb + (long long)a.T * KP;
        for (int t = 0; t < Tb; ++t) {
            rb = t == 0 ? xb[0] : rb + xb[t];
            r0[(long long)t * KP] = make_float2(LOGZERO, rb);
        }
    }
    __syncthreads();
    {   // ... and its r_sum (column 0 of Rsum buffer 1)
        const float2* r0 = Rb + (long long)a.T * KP;
        float* s0 = Rsum + (long long)a.T * KP;
        for (int t = tid; t < Tb; t += NT) s0[(long long)t * KP] = lae(LOGZERO, r0[(long long)t * KP].y, l1p);
    }

    for (int i = 0; i < maxlen && !stop; ++i) {
        const int nr = nrun;
        const float2* Rprev = Rb + (long long)((i + 1) & 1) * a.T * KP;
        float2* Rcur = Rb + (long long)(i & 1) * a.T * KP;
        const float* RsPrev = Rsum + (long long)((i + 1) & 1) * a.T * KP;
        float* RsCur = Rsum + (long long)(i & 1) * a.T * KP;
        // ---- pre-beam: the top P of ws0 (value desc, id asc) of this position, selected beforehand for every position
        // by prebeam_kernel (it depends on the decoder log-probs only)
        if (tid < P) {
            // (at the tails of the utterance's int / float scratch, [L][P] each)
            cs[tid] = a.is[(b + 1) * a.istride - (long long)a.L * P + (long long)i * P + tid];
            ws0c[tid] = a.fs[(b + 1) * a.fstride - (long long)a.L * P + (long long)i * P + tid];
        }
        __syncthreads();
        BPROF_MARK(0);
        // (the r_sum of every running hypothesis — logaddexp(r^n, r^b), the log_phi of a non-repeated label — is its
        // column of RsPrev: the r^b chains wrote it at the previous position)
        BPROF_MARK(1);
        // ---- CTC prefix scores (CTCPrefixScore.__call__): this workgroup's chains of the columns c = kP + j < nr P
        const int ncol = nr * P;
        if (pairw) {
            const int half = tid >> 7, col = 128 * grp + (tid & 127);   // half 0: r^n, 1: r^b (same column)
            const bool act = col < ncol;
            const int k = act ? col / P : 0, j = act ? col - k * P : 0;
            const int c = cs[j];
            const float* xc = xt + (long long)c * a.T;
            // output_length (sos ignored): every running hypothesis has length i + 1 (BeamSearchPara appends one token per
            // position and moves the ended ones out), so the block count below is uniform over the workgroup
            const int ol = hlen[0] - 1;
            const bool phi_b = ol > 0 && c == hlast[k]; // log_phi = r^b(g) for a repeated label
            const float2* rp = Rprev + hcol[k];         // frame t at rp[t * KP]
            const float* rsum = RsPrev + hcol[k];       // frame t at rsum[t KP]
            float* rn = (float*)(Rcur + col) + half;    // this chain's component of frame t at rn[2 t KP]
            float* rsc = RsCur + col;                   // r_sum of this column (r^b lanes)
            const int start = max(ol, 1);
            // r[start - 1] = (xs[0], logzero) at ol == 0, else (logzero, logzero)
            const float init0 = (ol == 0 && Tb > 0) ? xc[0] : LOGZERO;
            if (act && start - 1 < Tb) {
                rn[2LL * (start - 1) * KP] = half == 0 ? init0 : LOGZERO;
                if (half) rsc[(long long)(start - 1) * KP] = lae(init0, LOGZERO, l1p);
            }
            const int nblk = Tb > start ? (Tb - start + BL - 1) / BL : 0;
            float r = half == 0 ? init0 : LOGZERO;
            float prev0 = init0;                         // r^b lanes: r^n of the frame before the block
            // inputs of a block (r^n: phi and x of the candidate, r^b: x of blank) for BL frames, loaded one block ahead
            // of their use (the loads of block m + 1 are in flight while block m computes)
            float ca[BL], cb[BL];
            auto load_blk = [&](int mb, float (&pa)[BL], float (&pb)[BL]) __attribute__((always_inline)) {
                const int t0 = start + mb * BL;
#pragma unroll
                for (int u = 0; u < BL; ++u) {
                    const int t = min(t0 + u, Tb - 1);
                    if (half == 0) {
                        pa[u] = phi_b ? rp[(long long)(t - 1) * KP].y : rsum[(long long)(t - 1) * KP];
                        pb[u] = xc[t];
                    } else {
                        pb[u] = xb[t];
                    }
                }
            };
            if (act && nblk > 0) load_blk(0, ca, cb);
            for (int m = 0; m <= nblk; ++m) {
                const int mb = half == 0 ? m : m - 1;    // the block this lane computes in this round
                if (act && mb >= 0 && mb < nblk) {
                    float na[BL], nb[BL];
                    if (mb + 1 < nblk) load_blk(mb + 1, na, nb);
                    const int t0 = start + mb * BL;
                    float* pr = rn + 2LL * t0 * KP;
                    const long long stp = 2LL * KP;
                    const bool full = t0 + BL <= Tb;     // uniform: no per-frame guard inside full blocks
                    if (half == 0) {                     // r^n over block m
                        if (full) {
#pragma unroll
                            for (int u = 0; u < BL; ++u) {
                                r = lae(r, ca[u], l1p) + cb[u];
                                pr[u * stp] = r;
                                lag[mb & 1][u][tid & 127] = r;
                            }
                        } else {
#pragma unroll
                            for (int u = 0; u < BL; ++u) {
                                if (t0 + u < Tb) {
                                    r = lae(r, ca[u], l1p) + cb[u];
                                    pr[u * stp] = r;
                                }
                                lag[mb & 1][u][tid & 127] = r;
                            }
                        }
                    } else {                             // r^b over block m - 1 (r^n of its frames from the lag buffer)
#pragma unroll
                        for (int u0 = 0; u0 < BL; u0 += 8) {
                            float rq[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) rq[u] = lag[mb & 1][u0 + u][tid & 127];
                            if (full) {
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    r = lae(prev0, r, l1p) + cb[u0 + u];
                                    pr[(u0 + u) * stp] = r;
                                    prev0 = rq[u];
                                    // off the chain: r_sum of frame t = logaddexp(r^n_t, r^b_t)
                                    rsc[(long long)(t0 + u0 + u) * KP] = lae(prev0, r, l1p);
                                }
                            } else {
#pragma unroll
                                for (int u = 0; u < 8; ++u) {
                                    if (t0 + u0 + u < Tb) {
                                        r = lae(prev0, r, l1p) + cb[u0 + u];
                                        pr[(u0 + u) * stp] = r;
                                        rsc[(long long)(t0 + u0 + u) * KP] = lae(rq[u], r, l1p);
                                    }
                                    prev0 = rq[u];
                                }
                            }
                        }
                    }
                    if (mb + 1 < nblk) {
#pragma unroll
                        for (int u = 0; u < BL; ++u) { ca[u] = na[u]; cb[u] = nb[u]; }
                    }
                }
                __syncthreads();
            }
        } else {
            const int col = 256 * (grp - a.Gr) + tid;
            if (col < ncol) {
                const int k = col / P, j = col - k * P;
                const int c = cs[j];
                const float* xc = xt + (long long)c * a.T;
                const int ol = hlen[0] - 1;
                const bool phi_b = ol > 0 && c == hlast[k];
                const float2* rp = Rprev + hcol[k];
                const float* rsum = RsPrev + hcol[k];
                const int start = max(ol, 1);
                float lpsi = (ol == 0 && Tb > 0) ? xc[0] : LOGZERO;   // r[start - 1, 0]
                // phi + x of 16 frames per batch, the next batch's loads in flight while one computes
                constexpr int PB = 16;
                float cs16[PB];
                auto load_b = [&](int t0, float (&d)[PB]) __attribute__((always_inline)) {
#pragma unroll
                    for (int u = 0; u < PB; ++u) {
                        const int t = min(t0 + u, Tb - 1);
                        d[u] = (phi_b ? rp[(long long)(t - 1) * KP].y : rsum[(long long)(t - 1) * KP]) + xc[t];
                    }
                };
                if (start < Tb) load_b(start, cs16);
                for (int t0 = start; t0 < Tb; t0 += PB) {
                    float nx[PB];
                    if (t0 + PB < Tb) load_b(t0 + PB, nx);
#pragma unroll
                    for (int u = 0; u < PB; ++u)
                        if (t0 + u < Tb) lpsi = lae(lpsi, cs16[u], l1p);
                    if (t0 + PB < Tb) {
#pragma unroll
                        for (int u = 0; u < PB; ++u) cs16[u] = nx[u];
                    }
                }
                // r_sum[-1]; frames below the previous position's start were never computed (the reference's
                // fresh logzero state there: logaddexp(logzero, logzero) = logzero in f32)
                if (c == a.eos)
                    lpsi = Tb > 0 ? (Tb - 1 >= max(ol - 2, 0) ? rsum[(long long)(Tb - 1) * KP] : lae(LOGZERO, LOGZERO, l1p))
                                  : LOGZERO;
                if (c == a.blank) lpsi = LOGZERO;
                const float ts = lpsi - hprev[k];
                float* xo = xch + (long long)(i & 1) * 2 * KP;
                xo[col] = (ws0c[j] + a.wctc * ts) + hscore[k];
                xo[KP + col] = lpsi;
            }
        }
        // ---- every workgroup of the utterance has written its chains: arrival barrier (release / acquire at agent
        // scope: the states and scores written by the others become visible), bounded wait
        __syncthreads();
        if (tid == 0) {
            __threadfence();
            atomicAdd(sync, 1u);
            const unsigned want = (unsigned)a.G * (unsigned)(i + 1);
            unsigned spins = 0;
            while (__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > a.spin_cap) { atomicExch(sync + 1, 1u); stop = 1; break; }   // never expected
            }
            __threadfence();
        }
        __syncthreads();
        {
            const float* xi = xch + (long long)(i & 1) * 2 * KP;
            for (int w = tid; w < ncol; w += NT) {
                const int k = w / P, j = w - k * P;
                wsc[k][j] = __hip_atomic_load(xi + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                psi[k][j] = __hip_atomic_load(xi + KP + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        BPROF_MARK(2);
        // ---- per-hypothesis top kk (descending, equal scores: lower pre-beam rank), appended in hypothesis order
        for (int w = tid; w < nr * P; w += NT) {
            const int k = w / P, j = w - k * P;
            const float v = wsc[k][j];
            int r = 0;
            for (int q0 = 0; q0 < P; q0 += 4) {   // 16-B LDS reads (broadcast): four comparisons per round trip
                const float4 c4 = *(const float4*)&wsc[k][q0];
                const float c[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = q0 + u;
                    r += (q < P && (c[u] > v || (c[u] == v && q < j))) ? 1 : 0;
                }
            }
            if (r < kk) { csc[k * kk + r] = v; csrc[k * kk + r] = w; }
        }
        __syncthreads();
        BPROF_MARK(3);
        // ---- sort-and-prune after each hypothesis (search.py:330-332) keeps the top K of all appended candidates in
        // (score desc, append order) order: rank every candidate by counting those before it
        const int nall = nr * kk, nc = min(K, nall);
        for (int q = tid; q < nall; q += NT) {
            const float v = csc[q];
            int g = 0;
            for (int o0 = 0; o0 < nall; o0 += 4) {
                const float4 c4 = *(const float4*)&csc[o0];
                const float c[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int o = o0 + u;
                    g += (o < nall && (c[u] > v || (c[u] == v && o < q))) ? 1 : 0;
                }
            }
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
        BPROF_MARK(4);
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
                    if (grp == 0) {
                        bpar[(long long)i * K + keep] = par;
                        btok[(long long)i * K + keep] = ntokn[q];
                    }
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
        BPROF_MARK(5);
    }
#ifdef BEAM_PROF
    if (tid == 0 && grp == 0 && b < 1024)
        for (int q = 0; q < 8; ++q) beam_prof[b][q] = pt[q];
#endif
    // ---- n-best token ids: yseq[1:-1] without eos / sos / blank; the tokens of an ended hypothesis are its own
    // (position epos) and its parent chain's, found by walking the back-pointers
    if (tid == 0 && grp == 0) {
        const bool failed = __hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        for (int n = 0; n < a.nbest; ++n) {
            int* out = a.tokens + ((long long)b * a.nbest + n) * a.Lcap;
            if (n >= nend || failed) {
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

// Pre-beam of every decoder position (BeamSearchPara with pre_beam_score_key "full": the top P = int(1.5 beam) of the
// position's full weighted scores ws0 = am (+ the length bonus), search.py:281-299), one workgroup per (position,
// utterance) row, before the search: it depends on the decoder log-probs only. Output in (value desc, id asc) order,
// the order the serial top-k produces. Threshold selection: the P-th best tau of the NT per-thread bests (over strided
// ids) is not better than the P-th best id overall (the P threads above it hold P distinct ids not worse than tau), so
// the top P are among the ids not worse than tau: at most P threads contribute, ceil(V / NT) ids each; those survivors
// (dynamic LDS) are ranked by counting.
__global__ __launch_bounds__(NT) void prebeam_kernel(const float* __restrict__ am, int L, int V, int P, float pen,
                                                     int use_pen, const int* __restrict__ ntok, int* __restrict__ is,
                                                     long long istride, float* __restrict__ fs, long long fstride) {
#pragma clang fp contract(off)
    const int i = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    if (i >= min(ntok[b], L)) return;
    const float* ami = am + ((long long)b * L + i) * V;
    int* oid = is + (b + 1) * istride - (long long)L * P + (long long)i * P;       // the scratch tails, [L][P]
    float* oval = fs + (b + 1) * fstride - (long long)L * P + (long long)i * P;
    __shared__ __attribute__((aligned(16))) float lbv[NT];
    __shared__ __attribute__((aligned(16))) int lbi[NT];
    __shared__ float tau_v;
    __shared__ int tau_i, ncand;
    extern __shared__ int cand[];   // [2][cap]: value bits | ids
    const int cap = P * ((V + NT - 1) / NT) + 1;
    int* cv = cand;
    int* ci = cand + cap;
    if (P == V) {   // no pre-beam: the whole vocabulary in id order
        for (int v = tid; v < V; v += NT) { oid[v] = v; oval[v] = use_pen ? ami[v] + pen : ami[v]; }
        return;
    }
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int v0 = tid; v0 < V; v0 += 16 * NT) {   // 16 loads in flight per thread
        float r16[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) r16[u] = ami[min(v0 + u * NT, V - 1)];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int v = v0 + u * NT;
            const float w = use_pen ? r16[u] + pen : r16[u];
            if (v < V && (bi == 0x7fffffff || beats(w, v, bv, bi))) { bv = w; bi = v; }
        }
    }
    lbv[tid] = bv;
    lbi[tid] = bi;
    if (tid == 0) ncand = 0;
    __syncthreads();
    if (bi != 0x7fffffff) {   // rank among the per-thread bests (16 per trip, vector LDS reads)
        int r = 0;
        for (int q0 = 0; q0 < NT && r < P; q0 += 16) {
            float4 vv[4];
            int4 ii[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                vv[u] = *(const float4*)&lbv[q0 + 4 * u];
                ii[u] = *(const int4*)&lbi[q0 + 4 * u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                r += (ii[u].x != 0x7fffffff && beats(vv[u].x, ii[u].x, bv, bi)) ? 1 : 0;
                r += (ii[u].y != 0x7fffffff && beats(vv[u].y, ii[u].y, bv, bi)) ? 1 : 0;
                r += (ii[u].z != 0x7fffffff && beats(vv[u].z, ii[u].z, bv, bi)) ? 1 : 0;
                r += (ii[u].w != 0x7fffffff && beats(vv[u].w, ii[u].w, bv, bi)) ? 1 : 0;
            }
        }
        if (r == P - 1) { tau_v = bv; tau_i = bi; }
    }
    __syncthreads();
    const float tv = tau_v;
    const int ti = tau_i;
    if (!beats(tv, ti, bv, bi))   // (tau strictly better than this thread's best: none of its ids survives)
        for (int v = tid; v < V; v += NT) {
            const float w = use_pen ? ami[v] + pen : ami[v];
            if (beats(w, v, tv, ti)) {
                const int q = atomicAdd(&ncand, 1);
                cv[q] = __float_as_int(w);
                ci[q] = v;
            }
        }
    if (tid == 0) {   // tau itself
        const int q = atomicAdd(&ncand, 1);
        cv[q] = __float_as_int(tv);
        ci[q] = ti;
    }
    __syncthreads();
    const int M = ncand;
    for (int q = tid; q < M; q += NT) {
        const float w = __int_as_float(cv[q]);
        const int v = ci[q];
        int r = 0;
        for (int o = 0; o < M && r < P; ++o) r += beats(__int_as_float(cv[o]), ci[o], w, v) ? 1 : 0;
        if (r < P) { oid[r] = v; oval[r] = w; }
    }
}

// [B][T][V] -> [B] x [V][T] at dst + b * dstride (64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void transpose_tv_kernel(const float* __restrict__ src, int T, int V,
                                                           float* __restrict__ dst, long long dstride) {
    __shared__ float tile[64][65];
    const int v0 = blockIdx.x * 64, t0 = blockIdx.y * 64, b = blockIdx.z;
    const float* s = src + (long long)b * T * V;
    float* d = dst + (long long)b * dstride;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    for (int r = r0; r < 64; r += 4) {
        const int t = t0 + r, v = v0 + c;
        tile[r][c] = (t < T && v < V) ? s[(long long)t * V + v] : 0.f;
    }
    __syncthreads();
    for (int r = r0; r < 64; r += 4) {
        const int v = v0 + r, t = t0 + c;
        if (v < V && t < T) d[(long long)v * T + t] = tile[c][r];
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
static int pair_wgs(int K, int P) { return (K * P + 127) / 128; }
static int groups(int K, int P) { return pair_wgs(K, P) + (K * P + 255) / 256; }
long long pfm_ctc_beam_fscratch(int K, int P, int T, int L, int V) {
    const long long KP = (long long)K * P, S = L + 2;
    return pfm_align2((long long)V * T) +
           pfm_align2(4LL * T * KP + 4 * KP + 2LL * T * KP + groups(K, P) * (S + 1) + (long long)L * P);
}
long long pfm_ctc_beam_iscratch(int K, int nbest, int L, int P, int V) {
    const long long S = L + 2;
    (void)nbest;
    (void)V;
    return 2 + 2LL * L * K + S + groups(K, P) * (S + 1) + (long long)L * P;
}

// OR of the utterances' fail words (a search whose arrival barrier timed out) into one device word
__global__ __launch_bounds__(256) void beam_fail_kernel(const int* __restrict__ is, long long istride, int B,
                                                        unsigned* __restrict__ fail) {
    __shared__ int any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    int f = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) f |= is[(long long)b * istride + 1];
    if (f) atomicOr(&any, 1);
    __syncthreads();
    if (threadIdx.x == 0) fail[0] = any ? 1u : 0u;
}

hipError_t pfm_ctc_beam(const float* am, int L, const float* x, int T, const int* lens, const int* ntok, int B, int V,
                        int K, int P, int nbest, float wctc, float pen, int use_pen, int end_detect, int sos, int eos,
                        int blank, float* fs, int* is, int* tokens, int Lcap, int* olen, float* oscore,
                        unsigned* fail, hipStream_t st) {
    if (fail) {
        const hipError_t e0 = hipMemsetAsync(fail, 0, sizeof(unsigned), st);
        if (e0 != hipSuccess) return e0;
    }
    if (B <= 0) return hipSuccess;
    if (K < 1 || K > MAXK || P < 1 || P > MAXP || P > V || nbest < 1 || nbest > MAXN || Lcap < 0)
        return hipErrorInvalidValue;
    BeamArgs a;
    a.L = L; a.T = T; a.V = V; a.K = K; a.P = P; a.nbest = nbest;
    a.wctc = wctc; a.pen = pen; a.use_pen = use_pen; a.end_detect = end_detect; a.sos = sos; a.eos = eos;
    a.blank = blank; a.fstride = pfm_ctc_beam_fscratch(K, P, T, L, V);
    a.istride = pfm_ctc_beam_iscratch(K, nbest, L, P, V); a.Lcap = Lcap;
    a.Gr = pair_wgs(K, P);
    a.G = groups(K, P);
    {   // PFM_BEAM_SPIN_CAP: a small bound forces the timeout path (tests/test_gpu_beam.py); default 2^24 rounds
        const char* sc = getenv("PFM_BEAM_SPIN_CAP");
        a.spin_cap = (sc && sc[0]) ? (unsigned)strtoul(sc, nullptr, 10) : (1u << 24);
    }
    hipError_t e;
    if (T > 0) {   // the CTC log-probs, frame-contiguous per id, at the head of each utterance's float scratch
        hipLaunchKernelGGL(transpose_tv_kernel, dim3((V + 63) / 64, (T + 63) / 64, B), dim3(256), 0, st, x, T, V, fs,
                           a.fstride);
        PFM_LAUNCH_CHECK();
    }
    // the pre-beam of every position: [L][P] ids / values at the tail of each utterance's int / float scratch
    if (L > 0) {
        const size_t cand = (size_t)2 * (P * ((V + NT - 1) / NT) + 1) * sizeof(int);
        if (cand > 64 * 1024) return hipErrorInvalidValue;
        static bool attr = false;
        if (!attr) {
            attr = true;
            (void)hipFuncSetAttribute((const void*)prebeam_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
        }
        hipLaunchKernelGGL(prebeam_kernel, dim3((unsigned)L, (unsigned)B), dim3(NT), cand, st, am, L, V, P, pen, use_pen,
                           ntok, is, a.istride, fs, a.fstride);
        PFM_LAUNCH_CHECK();
    }
    // the [sync, fail] words at the head of every utterance's int scratch start at zero
    e = hipMemset2DAsync(is, (size_t)a.istride * sizeof(int), 0, 2 * sizeof(int), (size_t)B, st);
    if (e != hipSuccess) return e;
    // The workgroups of an utterance wait for each other once per position, so all of a launch must be resident at
    // once: a cooperative launch guarantees it (or fails); utterances go in chunks that fit the device.
    int dev = 0, ncu = 0, per_cu = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)ctc_beam_kernel, NT, 0)) != hipSuccess)
        return e;
    const int cap_wg = ncu * per_cu;
    const int Bc = (cap_wg / a.G) / 8 * 8;   // utterances per launch (whole XCD rounds: 8 consecutive utterances)
    if (Bc < 8) return hipErrorInvalidConfiguration;
    for (int b0 = 0; b0 < B; b0 += Bc) {
        const int nb = B - b0 < Bc ? B - b0 : Bc;
        BeamArgs c = a;
        c.B = nb;
        c.lens = lens + b0;
        c.ntok = ntok + b0;
        c.fs = fs + (long long)b0 * a.fstride;
        c.is = is + (long long)b0 * a.istride;
        c.tokens = tokens + (long long)b0 * nbest * Lcap;
        c.olen = olen + (long long)b0 * nbest;
        c.oscore = oscore + (long long)b0 * nbest;
        void* args[] = {&c};
        const dim3 grid((unsigned)(((nb + 7) / 8) * 8 * a.G));
        e = hipLaunchCooperativeKernel((const void*)ctc_beam_kernel, grid, dim3(NT), args, 0u, st);
        if (e != hipSuccess) return e;
    }
    if (fail) {
        hipLaunchKernelGGL(beam_fail_kernel, dim3(1), dim3(256), 0, st, is, a.istride, B, fail);
        PFM_LAUNCH_CHECK();
    }
    return hipSuccess;
}
