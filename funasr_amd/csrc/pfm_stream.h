// Streaming Paraformer: per-stream chunk parameters and the k_stream.hip launchers.
#pragma once
#include "pfm_common.h"

// One entry per stream of a pfm_stream_step batch (uploaded once per step).
struct SPrm {
    int slot;    // state slot
    int nfeat;   // new LFR rows of this chunk (0: tail chunk, the cached overlap only)
    int start;   // StreamSinusoidalPositionEncoder start_idx before this chunk
    int tw;      // encoder window rows (overlap cache + nfeat)
    int fin;     // is_final
    int cle;     // encoder K/V cache rows before this chunk
    int cld;     // decoder K/V cache rows before this chunk
    int pad;
};

hipError_t pfm_stream_window(const float* feats, int Tn, const SPrm* prm, int n, const float* fcache, const float* pe,
                             int I, int C0, int Tw, float scale, float* x, hipStream_t st);
hipError_t pfm_stream_fcache(const float* x, const SPrm* prm, int n, int I, int C0, int Tw, float* fcache,
                             hipStream_t st);
hipError_t pfm_kv_gather(int dtype, const void* cache, int C, const SPrm* prm, int n, int dec, const void* src,
                         long long src_ld, int Tw, void* buf, int Tk, int W, hipStream_t st);
hipError_t pfm_kv_retain(int dtype, const void* buf, int Tk, const SPrm* prm, int n, int dec, int drop, const int* ntok,
                         void* cache, int C, int W, hipStream_t st);
hipError_t pfm_stream_mask_rows(float* encp, bf16* encpb, const SPrm* prm, int n, int Tw, int D, hipStream_t st);
hipError_t pfm_cif_chunk(const float* hc, const float* wout, const float* bout, const float* encp, const SPrm* prm,
                         int n, int Tw, int D, int cs0, int keep, float smooth, float noise, float tail, float thr,
                         float* chid, float* calpha, float* emb, int Lcap, int* ntok, float* alphas_out,
                         hipStream_t st);
hipError_t pfm_dec_fsmn_stream(int dtype, const void* v, const float* wT, int K, float* state, const SPrm* prm,
                               const int* ntok, int n, int L, int D, float* x, hipStream_t st);
hipError_t pfm_pad_rows_zero(float* encp, bf16* encpb, int n, int Tw, int D, hipStream_t st);
hipError_t pfm_rows_copy(float* dst, long long dld, const float* src, long long sld, int w, int rows, hipStream_t st);
