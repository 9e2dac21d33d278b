// Shared device/host helpers for the MI355X (gfx950) Paraformer path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16;

#define PFM_WAVE 64

// dtype codes shared with include/pfm.h
enum { DT_F32 = 0, DT_BF16 = 1,
       // internal: three bf16 planes x0 | x1 | x2 (x = x0 + x1 + x2 exactly) per row, plane stride = the
       // row's logical width; the A operand layout of the EXACT-mode split-bf16 x6 GEMM
       DT_X3 = 2 };

__device__ __forceinline__ void split3_bf16(float x, bf16& a, bf16& b, bf16& c) {
    a = (bf16)x;
    const float r = x - (float)a;
    b = (bf16)r;
    c = (bf16)(r - (float)b);
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }   // RNE, v_cvt_pk_bf16_f32 on gfx950

template <typename T> __device__ __forceinline__ float to_f(T x);
template <> __device__ __forceinline__ float to_f<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f<bf16>(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Row addressing shared by GEMM operands and element kernels: logical row m lives at
//   base + (m / rows_per_seg) * seg_stride + (m % rows_per_seg) * ld
// (rows_per_seg == 0 means a plain [M, ld] matrix). Lets the predictor/cross-attention
// read the encoder output from its zero-padded [B][T+2][D] layout without copies.
struct RowMap {
    int rows_per_seg;
    long long seg_stride;
    long long ld;
    __host__ __device__ __forceinline__ long long off(long long m) const {
        if (rows_per_seg <= 0) return m * ld;
        return (m / rows_per_seg) * seg_stride + (m % rows_per_seg) * ld;
    }
};
static inline RowMap rowmap_plain(long long ld) { RowMap r; r.rows_per_seg = 0; r.seg_stride = 0; r.ld = ld; return r; }
static inline RowMap rowmap_seg(int rows, long long seg_stride, long long ld) {
    RowMap r; r.rows_per_seg = rows; r.seg_stride = seg_stride; r.ld = ld; return r;
}

// ---- host-side launch helpers (all return hipError_t) --------------------------------
#define PFM_LAUNCH_CHECK() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return _e; } while (0)

// Epilogue descriptor for C = act(A . W^T + bias) (+ res0) (+ res1), stored as f32 or bf16.
struct GemmEpi {
    const float* bias;      // [N] or null
    const float* res0;      // residual #1 [M, ld_res0] f32 or null (added after activation)
    const float* res1;      // residual #2 (same layout as res0, ld_res1) or null
    long long ld_res0, ld_res1;
    int relu;               // 1: relu before residual adds
    int res0_bf16;          // res0 points at bf16 data (fast mode FSMN memory)
    float alpha;            // scale applied to A.W^T before bias
    void* out;              // C
    RowMap out_map;         // row addressing of C (and of residuals via their own ld)
    int out_dtype;          // DT_F32 / DT_BF16
    // optional second output (bf16 copy of the f32 result, same RowMap) for fast mode
    void* out2;
    RowMap out2_map;
    // optional fused row-argmax (output layer): per (row, n-tile) best value + index
    float* amax_val;        // [M, n_tiles] or null
    int* amax_idx;
    int n_tiles;
    // set by the launcher: N, residual strides and output row offsets are multiples of 4
    // (float4 / bf16x4 vector epilogue legal)
    int vec_ok;
    // set by the bf16 launcher: bf16-only output with 16-B aligned rows -> 8 columns per lane,
    // one 16-B store each (halves the store-issue tail of the big bf16 outputs)
    int st16_ok;
    int res_batch;          // epilogue: residual loads of 4 row groups issued before their stores
    // three-way split bf16 emulation of an f32 GEMM (EXACT mode, bf16 256-tile kernel): A = [A0 | A1 | A2]
    // ([M, 3 x6_k], x = x0 + x1 + x2 exactly), W = three bf16 planes x6_ws elements apart; the kernel runs
    // K' = 6 x6_k over the segments (A2,W0) (A1,W1) (A0,W2) (A1,W0) (A0,W1) (A0,W0). 0 = plain GEMM.
    // x6_terms 3 (bf16x3): only the last three segments (A1,W0) (A0,W1) (A0,W0), K' = 3 x6_k (relative
    // error ~2^-16 instead of ~2^-24); 0 / 6 = all six. x6_terms 2 (fast mode, precise weights): A is ONE bf16
    // operand [M, x6_k], W = w0 + w1 two planes x6_ws apart, K' = 2 x6_k over (A, W1) (A, W0).
    int x6_k;
    long long x6_ws;
    int x6_terms;
};

static inline bool rowmap_vec4(const RowMap& m) {
    return m.ld % 4 == 0 && (m.rows_per_seg <= 0 || m.seg_stride % 4 == 0);
}
static inline int epi_vec_ok(const GemmEpi& e, int N) {
    if (N % 4) return 0;
    if (e.res0 && e.ld_res0 % 4) return 0;
    if (e.res1 && e.ld_res1 % 4) return 0;
    if (e.out && !rowmap_vec4(e.out_map)) return 0;
    if (e.out2 && !rowmap_vec4(e.out2_map)) return 0;
    return 1;
}

// ---- A/B knobs (PFM_* environment variables) ------------------------------------------
// Read once per top-level C-ABI call on the calling thread (pfm_knobs_refresh at pfm_create, pfm_run,
// pfm_run_ctc, pfm_run_punc, pfm_stream_step, ...), never per launch. Launchers read the calling
// thread's snapshot through pfm_knobs(). `sig` hashes every field: captured streaming graphs are keyed
// by it, so a changed knob never replays a graph recorded under other settings.
struct PfmKnobs {
    int attn_fsmn;          // PFM_ATTN_FSMN (default 1): encoder FSMN fused into the attention epilogue
    int attn_waves;         // PFM_ATTN_WAVES (default 8)
    int kv_overlap;         // PFM_KV_OVERLAP (default 1): memory K|V projection on the side stream
    int subbatch;           // PFM_SUBBATCH (default 2): concurrent encoder utterance groups
    int stream_graph;       // PFM_STREAM_GRAPH (default 1): streaming steps through HIP graphs
    int punc_graph;         // PFM_PUNC_GRAPH (default 1): fast-mode pfm_run_punc_host pads the sentence to a multiple
                            // of 16 words and replays its launches from one HIP graph per padded length
    int gemm_gm;            // PFM_GEMM_GM: grouped tile order override (-1 = default)
    int gemm_cfg;           // PFM_GEMM_CFG: forced tile configuration (0 = policy)
    int gemm_st16;          // PFM_GEMM_ST16 (default 1): 16-B bf16 epilogue stores
    int gemm_resbatch;      // PFM_GEMM_RESBATCH (default 1): residual loads batched ahead of the stores
    int gemm_skinny;        // PFM_GEMM_SKINNY (default 1): weight-streaming kernel for <= 64-row GEMMs
    int ffn_fused;          // PFM_FFN_FUSED (default 1): fused LN2 + FFN + LN1_next encoder kernel (k_ffn.hip)
    int exact_x6;           // PFM_EXACT_X6 (default 1): EXACT-mode GEMMs as split bf16 x6 MFMA (f32 MFMA if 0)
    int dec_subbatch;       // PFM_DEC_SUBBATCH (default 2): decoder utterance groups on concurrent streams
    int ffn_op;             // PFM_FFN_OP (default 1): encoder out-projection folded into the fused FFN kernel
    int dec_ffn_fused;      // PFM_DEC_FFN_FUSED (default 1): decoder LN1-FFN(LN_F folded)-LN kernel (fast mode)
    int ffn_kernel;         // PFM_FFN_KERNEL (default 2): encoder fused FFN as 128-row workgroups (k_ffn2.hip, with
                            // the next layer's QKV projection folded in); 1 = 64-row workgroups (k_ffn.hip)
    int ffn_qkv;            // PFM_FFN_QKV (default 1): with the 128-row fused FFN, the next layer's QKV projection as
                            // its phase 3 (k_ffn2.hip MODE 4; the separate LN1 + QKV GEMM otherwise)
    int fast_xw;            // PFM_FAST_XW (bitmask, default 7): fast mode keeps these weights as two bf16 planes
                            // w = w0 + w1 (~2^-17 relative; activations stay bf16): 1 = the CIF predictor conv,
                            // 2 = encoder layer 0 (QKV, out-projection, FFN; runs unfused), 4 = the v rows of every
                            // QKV projection (ffn2_kernel MODE 5), 8 = every encoder out-projection (MODE 6 / 3;
                            // implies 4). tools/fast_emul.py: the weights' bf16 rounding, not the activations', is
                            // what moves the fast path's decisions off the reference's (7: B=64 flips 25 -> 10 %,
                            // +3-5 % step; 15: 5 %, +9 %)
    unsigned long long sig;
};
#define PFM_KNOB_FIELDS 19
const PfmKnobs& pfm_knobs();   // the calling thread's snapshot (refreshed lazily if no entry point did yet)
void pfm_knobs_refresh();
