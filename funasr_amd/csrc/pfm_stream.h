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

// Attention keys of one layer = [K/V cache (cl rows) ; the window's K|V rows (tw rows)] (sanm/attention.py:327-334
// encoder, 733-737 decoder): key row r of stream i into buf [n][Tk][W] (W = 2d: K | V), 16-B copies by threads
// tid, tid + nth, ...; rows past cl + tw are zeros
template <typename T>
__device__ __forceinline__ void kv_gather_row(const T* __restrict__ cache, int C, const SPrm& p, int dec,
                                              const T* __restrict__ src, long long src_ld, int Tw, T* __restrict__ buf,
                                              int Tk, int W, int i, int r, int tid, int nth) {
    const int cl = dec ? p.cld : p.cle;
    constexpr int V = 16 / sizeof(T);
    uint4* dst = (uint4*)(buf + ((long long)i * Tk + r) * W);
    const uint4* s = nullptr;
    if (r < cl) s = (const uint4*)(cache + ((long long)p.slot * C + r) * W);
    else if (r < cl + p.tw) s = (const uint4*)(src + ((long long)i * Tw + (r - cl)) * src_ld);
    for (int c = tid; c < W / V; c += nth) dst[c] = s ? s[c] : make_uint4(0, 0, 0, 0);
}

hipError_t pfm_stream_window(const float* feats, int Tn, const SPrm* prm, int n, const float* fcache, const float* pe,
                             int I, int C0, int Tw, float scale, float* x, hipStream_t st);
hipError_t pfm_stream_fcache(const float* x, const SPrm* prm, int n, int I, int C0, int Tw, float* fcache,
                             hipStream_t st);
hipError_t pfm_kv_gather(int dtype, const void* cache, int C, const SPrm* prm, int n, int dec, const void* src,
                         long long src_ld, int Tw, void* buf, int Tk, int W, hipStream_t st);
// ... for `layers` layers in one launch (grid.z): layer l reads cache + l cache_ls and src + l src_ls, writes buf + l buf_ls
// (strides in elements; the streaming decoder gathers all its layers' keys up front, before any layer's retain)
hipError_t pfm_kv_gather_layers(int dtype, const void* cache, long long cache_ls, int C, const SPrm* prm, int n, int dec,
                                const void* src, long long src_ls, long long src_ld, int Tw, void* buf, long long buf_ls,
                                int Tk, int W, int layers, hipStream_t st);
// streaming encoder layer, one launch: the key buffer gather above and the window's FSMN memory block
// (fsmn_win_kernel<11, bf16, 5> of k_elem.hip on the window's V rows, lens = tw) side by side
hipError_t pfm_kv_gather_fsmn(const bf16* cache, int C, const SPrm* prm, int n, const bf16* src, long long src_ld, int Tw,
                              bf16* buf, int Tk, int W, const bf16* v, RowMap vmap, const int* len, int D, const float* wT,
                              bf16* out_bf, hipStream_t st);
hipError_t pfm_kv_retain(int dtype, const void* buf, int Tk, const SPrm* prm, int n, int dec, int drop, const int* ntok,
                         void* cache, int C, int W, hipStream_t st);
hipError_t pfm_stream_mask_rows(float* encp, bf16* encpb, const SPrm* prm, int n, int Tw, int D, hipStream_t st);
hipError_t pfm_cif_chunk(const float* hc, const float* wout, const float* bout, const float* encp, const SPrm* prm,
                         int n, int Tw, int D, int cs0, int keep, float smooth, float noise, float tail, float thr,
                         float* chid, float* calpha, float* emb, int Lcap, int* ntok, float* alphas_out,
                         hipStream_t st);
hipError_t pfm_dec_fsmn_stream(int dtype, const void* v, const float* wT, int K, float* state, const SPrm* prm,
                               const int* ntok, int n, int L, int D, float* x, hipStream_t st);
// fast mode: the decoder layer's norm2 (LayerNorm of the FFN output rows, f32) fused in front of the FSMN above;
// hipErrorNotSupported (nothing launched) for shapes it does not take
hipError_t pfm_dec_fsmn_ln_stream(const float* tin, const float* g, const float* b, float eps, const float* wT, int K,
                                  float* state, const SPrm* prm, const int* ntok, int n, int L, int D, float* x,
                                  hipStream_t st);
hipError_t pfm_pad_rows_zero(float* encp, bf16* encpb, int n, int Tw, int D, hipStream_t st);
hipError_t pfm_rows_copy(float* dst, long long dld, const float* src, long long sld, int w, int rows, hipStream_t st);
