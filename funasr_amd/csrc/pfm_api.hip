// C-ABI implementation (include/pfm.h): weight registry, workspace and the Paraformer
// forward pipeline on one HIP stream. Host code only; kernels live in k_*.hip.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include <atomic>
#include <map>
#include <array>

#include "../../include/pfm.h"
#include "pfm_common.h"
#include "pfm_stream.h"

// ---- kernel launchers (k_*.hip)
hipError_t pfm_gemm(int dtype, const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                    const GemmEpi& epi, hipStream_t st);
int pfm_gemm_amax_tiles(int N);
bool pfm_gemm_bf16_256_ok(RowMap amap, long long ldw, int K);
int pfm_gemm_bf16_256_amax_tiles(int N);
hipError_t pfm_gemm_bf16_256(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                             const GemmEpi& epi, hipStream_t st);
hipError_t pfm_attention(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                         RowMap vmap, float* o, long long ldo, void* o2, const int* klen, int B, int Tq, int Tk,
                         int heads, int dk, float scale, hipStream_t st);
hipError_t pfm_attention_fsmn(int dtype, const void* q, RowMap qmap, const void* k, RowMap kmap, const void* v,
                              RowMap vmap, float* o, long long ldo, void* o2, const int* klen, int B, int Tq,
                              int Tk, int heads, int dk, float scale, const float* fsmn_wT, bf16* fsmn_out,
                              long long fsmn_ld, hipStream_t st);
int pfm_attention_lds_bytes(int dtype);
hipError_t pfm_layernorm(const float* x, RowMap xmap, int M, int D, const float* g, const float* b, float eps,
                         const float* pe, int pe_T, float in_scale, void* out, RowMap omap, int odt, void* out2,
                         RowMap o2map, int o2dt, hipStream_t st);
hipError_t pfm_layernorm_bf16in(const bf16* x, RowMap xmap, int M, int D, const float* g, const float* b, float eps,
                                void* out, RowMap omap, int odt, hipStream_t st);
hipError_t pfm_fsmn(const float* v, RowMap vmap, const int* len, int B, int T, int D, const float* w, int K,
                    int left, const float* res, float* out, bf16* out_bf, hipStream_t st);
hipError_t pfm_fsmn_ln_bf16in(const bf16* v, RowMap vmap, const int* len, int B, int T, int D, const float* wT,
                              int K, int left, const float* res, float* out, const float* g, const float* b, float eps,
                              bf16* ln_out, hipStream_t st);
hipError_t pfm_fsmn_bf16in(const bf16* v, RowMap vmap, const int* len, int B, int T, int D, const float* wT, int K,
                           int left, const float* res, float* out, bf16* out_bf, hipStream_t st);
hipError_t pfm_cif_alpha(const float* hc, int D, const float* wout, const float* bout, const int* len, int B,
                         int T, float smooth, float noise, float tail, float* alphas, hipStream_t st);
hipError_t pfm_cif_fire(const float* alphas, const float* h, RowMap hmap, int B, int T, int D, int Lcap,
                        float* emb, float* peaks, int* n_fire, int* ntok, hipStream_t st);
hipError_t pfm_argmax_reduce(const float* val, const int* idx, int ntiles, int ncount, int B, int L, const int* ntok,
                             int Lcap, int* tokens, float* score, hipStream_t st);
hipError_t pfm_fill_i32(int* p, long long n, int v, hipStream_t st);
hipError_t pfm_sv_input(const float* feats, const int* lens, const float* embed, const int* qid, int nq, int B, int T,
                        int I, float* x, int* olen, hipStream_t st);
hipError_t pfm_ctc_collapse(const int* ids, long long ld, const int* olen, int B, int blank, int Lcap, int* tokens,
                            int* ntok, hipStream_t st);
hipError_t pfm_f32_to_bf16(const float* x, bf16* y, long long n, hipStream_t st);
hipError_t pfm_swap_last2(const float* x, float* y, long long A, long long Bd, long long C, hipStream_t st);
hipError_t pfm_logsoftmax_rows(float* x, long long rows, long long ld, int V, hipStream_t st);
long long pfm_ctc_beam_fscratch(int K, int P, int T, int L, int V);
hipError_t pfm_attention_retain(const void* q, RowMap qmap, const void* kv, int B, int Tq, int Tk, void* o2, long long ldo,
                                const int* klen, int heads, int dk, float scale, const SPrm* prm, void* cache, int C,
                                int drop, int dec, const int* ntok, hipStream_t st);
long long pfm_ctc_beam_iscratch(int K, int nbest, int L, int P, int V);
hipError_t pfm_ctc_beam(const float* am, int L, const float* x, int T, const int* lens, const int* ntok, int B, int V,
                        int K, int P, int nbest, float wctc, float pen, int use_pen, int end_detect, int sos, int eos,
                        int blank, float* fs, int* is, int* tokens, int Lcap, int* olen, float* oscore,
                        unsigned* fail, hipStream_t st);
size_t pfm_ffn_packed_elems();
hipError_t pfm_emis_stats(const float* logits, long long rows, int V, float* mx, float* inv, int* amax, hipStream_t st);
hipError_t pfm_ctc_align_run(const float* logits, const float* mx, const float* inv, const int* amax, int B, int Tf,
                             int V, int blank, const int* olen, const int* tg, const int* tlen, int Lmax,
                             unsigned char* bp, int* align, hipStream_t st);
hipError_t pfm_split3_rows(const float* x, RowMap xm, int M, int K, int Kp, bf16* out, hipStream_t st);
hipError_t pfm_split3_planes(const float* x, bf16* p, long long plane, long long n, hipStream_t st);
hipError_t pfm_attention_x3(const float* q, RowMap qmap, const float* k, RowMap kmap, const float* v, RowMap vmap,
                            bf16* out3, const int* klen, int B, int Tq, int Tk, int heads, int dk, float scale,
                            const float* fsmn_wT, float* fsmn_out, long long fsmn_ld, hipStream_t st);
hipError_t pfm_ffn_pack(const bf16* W1, const bf16* W2, bf16* Wp, hipStream_t st);
size_t pfm_ffn_packed_o_elems();
hipError_t pfm_ffn_pack_dec(const bf16* W1, const float* W2, const float* gF, const float* bF, bf16* Wp, float* c1,
                            float* c2, hipStream_t st);
hipError_t pfm_ffn_fused_dec(const float* x, int M, const float* g1, const float* be1, float eps, const bf16* Wp,
                             const float* b1, const float* c1, const float* c2, float* xo, const float* gn,
                             const float* bn, bf16* xn, const bf16* o, const float* bo, hipStream_t st);
hipError_t pfm_ffn_pack_o(const bf16* Wo, bf16* Wp, hipStream_t st);
hipError_t pfm_ffn_dec_consts(const float* W2, const float* gF, const float* bF, float* c1, float* c2, hipStream_t st);
// k_ffn2.hip: the decoder FFN with its hidden split over two workgroups per 128-row tile (MODE 7 / 8)
size_t pfm_ffn2_dec_packed_elems();
hipError_t pfm_ffn2_pack_dec(const bf16* W1, const float* W2, const float* gF, const bf16* Wo, bf16* Wp, hipStream_t st,
                             bool split);
size_t pfm_ffn2_dec_scratch_floats(int M);
size_t pfm_ffn2_dec_counters(int M);
hipError_t pfm_ffn2_fused_dec(const float* x, int M, const float* g1, const float* be1, float eps, const bf16* Wp,
                              const float* b1, const float* c1, const float* c2, float* xo, const float* gn,
                              const float* bn, bf16* xn, const bf16* o, const float* bo, float* part, unsigned* cnt,
                              hipStream_t st);
// k_ffn2.hip: the encoder's fused sub-layers at 128 rows per workgroup (same packed sizes, its own fragment order)
hipError_t pfm_ffn2_pack(const bf16* W1, const bf16* W2, bf16* Wp, hipStream_t st);
hipError_t pfm_ffn2_pack_o(const bf16* Wo, bf16* Wp, hipStream_t st);
hipError_t pfm_ffn2_fused(const float* x, int M, const float* g2, const float* be2, float eps, const bf16* Wp,
                          const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn,
                          hipStream_t st);
hipError_t pfm_ffn2_fused_op(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                             const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                             const float* gn, const float* bn, bf16* xn, hipStream_t st);
hipError_t pfm_ffn_fused_op(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                            const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                            const float* gn, const float* bn, bf16* xn, hipStream_t st);
hipError_t pfm_ffn2_pack_qkv_v(const bf16* Wqkv_lo, bf16* Wp, hipStream_t st);
hipError_t pfm_ffn2_fused_op_qkv_xv(const bf16* o, const bf16* f, const float* bo, const float* x, int M,
                                    const float* g2, const float* be2, float eps, const bf16* Wop, const float* b1,
                                    const float* b2, float* xo, const float* gn, const float* bn, const float* bq,
                                    bf16* qkv, bool xo_planes, hipStream_t st);
hipError_t pfm_ffn2_fused_op_xo(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                                const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2,
                                float* xo, const float* gn, const float* bn, bf16* xn, hipStream_t st);
hipError_t pfm_ffn2_fused_op_qkv(const bf16* o, const bf16* f, const float* bo, const float* x, int M, const float* g2,
                                 const float* be2, float eps, const bf16* Wop, const float* b1, const float* b2, float* xo,
                                 const float* gn, const float* bn, const float* bq, bf16* qkv, hipStream_t st);
hipError_t pfm_ffn2_pack_qkv(const bf16* Wqkv, bf16* Wp, hipStream_t st);
hipError_t pfm_ffn_fused(const float* x, int M, const float* g2, const float* be2, float eps, const bf16* Wp,
                         const float* b1, const float* b2, float* xo, const float* gn, const float* bn, bf16* xn,
                         hipStream_t st);
hipError_t pfm_fbank_launch(const float* wav, const int* nsamp, int B, int S_max, const float* cmvn,
                            const unsigned char* tables, float* fb_ws, int N_cap, float* feats, int T_cap, int* T_out,
                            hipStream_t st);
bool pfm_gemm_skinny_ok(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                        const GemmEpi& e);
bool pfm_gemm_skinny_ln2048_ok(const bf16* X, RowMap xmap, const void* W, long long ldw, int M, int N, int K,
                               const GemmEpi& e);
hipError_t pfm_gemm_skinny_ln2048(const bf16* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                                  long long ldw, int M, int N, const GemmEpi& e, hipStream_t st);
bool pfm_gemm_skinny_ln_ok(const float* X, RowMap xmap, const void* W, long long ldw, int M, int N, int K,
                           const GemmEpi& e);
hipError_t pfm_gemm_skinny_ln(const float* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                              long long ldw, int M, int N, const GemmEpi& e, hipStream_t st);
hipError_t pfm_gemm_skinny(const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                           const GemmEpi& e, hipStream_t st);
hipError_t pfm_gemm_skinny_ln_qkv(const float* X, RowMap xmap, const float* g, const float* b, float eps, const void* W,
                                  long long ldw, int M, int N, const GemmEpi& e, const SPrm* prm, int n, int Tw,
                                  const bf16* cache, int C, bf16* buf, int Tk, const float* wT, bf16* fout, int D,
                                  hipStream_t st);
hipError_t pfm_punc_embed(const int* ids, const int* lens, int B, int T, const float* embed, int n_embed,
                          const float* pe, int D, float scale, float* X, hipStream_t st);
hipError_t pfm_punc_head(const float* x, int B, int T, const int* lens, const float* W, const float* bias, int NP,
                         int D, int* punc, float* logits, hipStream_t st);
hipError_t pfm_vad_dense(const float* X, int ldx, int M, int K, const float* W, const float* b, int N, int relu,
                         float* Y, int ldy, hipStream_t st);
hipError_t pfm_vad_fsmn(const float* x, int T, int D, float* cache, float* cache_tmp, const float* w, int L, float* y,
                        hipStream_t st);
hipError_t pfm_vad_softmax(const float* logits, int M, int N, float* p_sil, float* probs, hipStream_t st);
hipError_t pfm_vad_frame_energy(const float* wav, int nframes, int fl, int fs, float* e, hipStream_t st);
hipError_t pfm_fbank_raw_launch(const float* wav, const int* nsamp, int B, int S_max, const unsigned char* tables,
                                float* fb, int N_cap, hipStream_t st);
hipError_t pfm_lfr_gather_launch(const float* frames, const int* idx, int rows, int m, const float* cmvn, float* out,
                                 hipStream_t st);
int pfm_fbank_frames(int nsamp);
int pfm_fbank_nframes(int nsamp);
void pfm_fbank_tables(float* melw, int* lo, int* hi, float* window, double* tw);
size_t pfm_fbank_table_bytes();
size_t pfm_fbank_twoff();

// ---- error plumbing
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// after a synchronised pfm_ctc_beam: the device fail word -> PFM_E_DEVICE (a search whose workgroups lost each other
// at the per-position arrival barrier returns no hypotheses, which must not pass for "search found none")
static int beam_failed(const unsigned* fail_dev, const char* who) {
    unsigned f = 0;
    if (hipMemcpy(&f, fail_dev, sizeof(f), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(PFM_E_HIP, std::string(who) + ": reading the search's fail word");
    return f ? fail(PFM_E_DEVICE, std::string(who) + ": the beam search's cross-workgroup barrier timed out")
             : PFM_OK;
}
// the host-only translation units (vad_detector.hip) report errors through the same thread-local string
int pfm_fail(int code, const char* msg) { return fail(code, msg); }
#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(PFM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));           \
    } while (0)

// Device operands of the C ABI must be device memory of the call's GPU: a host (pageable or pinned) or unregistered
// address handed to a kernel faults the device instead of failing the call, so every entry point asks the runtime
// what each operand is before it launches anything and refuses with PFM_E_ARG, naming the operand. Interior pointers
// of an allocation (tensor slices) resolve to the allocation. `dev` < 0: the calling thread's current device.
struct DevOp { const char* name; const void* p; };
static int check_dev(const char* fn, int dev, std::initializer_list<DevOp> ops) {
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return fail(PFM_E_HIP, std::string(fn) + ": no current HIP device");
    }
    for (const DevOp& o : ops) {
        if (!o.p) continue;   // optional operand not given (required ones are null-checked before this)
        hipPointerAttribute_t a{};
        const hipError_t e = hipPointerGetAttributes(&a, o.p);
        if (e != hipSuccess) (void)hipGetLastError();   // an unknown address sets the sticky error: clear it
        const bool device = e == hipSuccess && (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged);
        if (!device)
            return fail(PFM_E_ARG, std::string(fn) + ": operand '" + o.name +
                                       "' is not device memory (host or unregistered address); device operands must be "
                                       "allocated on the GPU");
        if (a.type == hipMemoryTypeDevice && a.device != dev)
            return fail(PFM_E_ARG, std::string(fn) + ": operand '" + o.name + "' is on device " +
                                       std::to_string(a.device) + ", the call runs on device " + std::to_string(dev));
    }
    return PFM_OK;
}
#define CHECK_DEV(fn, dev, ...)                                 \
    do {                                                        \
        const int _rc = check_dev(fn, dev, {__VA_ARGS__});      \
        if (_rc) return _rc;                                    \
    } while (0)

// Every field is an int; the FNV hash below walks them all. A thread that reads the knobs before any
// C-ABI entry point refreshed them gets the documented defaults (lazy first refresh), never zero-fill.
static_assert(sizeof(PfmKnobs) == (PFM_KNOB_FIELDS * sizeof(int) + 7) / 8 * 8 + sizeof(unsigned long long),
              "PfmKnobs: PFM_KNOB_FIELDS int fields + sig");
static thread_local PfmKnobs t_knobs;
static thread_local bool t_knobs_set = false;

const PfmKnobs& pfm_knobs() {
    if (!t_knobs_set) pfm_knobs_refresh();
    return t_knobs;
}

void pfm_knobs_refresh() {
    auto iv = [](const char* name, int dflt) {
        const char* e = getenv(name);
        return (e && e[0]) ? atoi(e) : dflt;
    };
    PfmKnobs k;
    k.attn_fsmn = iv("PFM_ATTN_FSMN", 1) != 0;
    k.attn_waves = iv("PFM_ATTN_WAVES", 8);
    k.kv_overlap = iv("PFM_KV_OVERLAP", 1) != 0;
    k.subbatch = std::max(1, std::min(iv("PFM_SUBBATCH", 2), 4));
    k.stream_graph = iv("PFM_STREAM_GRAPH", 1) != 0;
    k.punc_graph = iv("PFM_PUNC_GRAPH", 1) != 0;
    k.gemm_gm = iv("PFM_GEMM_GM", -1);
    k.gemm_cfg = iv("PFM_GEMM_CFG", 0);
    k.gemm_st16 = iv("PFM_GEMM_ST16", 1) != 0;
    k.gemm_resbatch = iv("PFM_GEMM_RESBATCH", 1) != 0;
    k.gemm_skinny = iv("PFM_GEMM_SKINNY", 1) != 0;
    k.ffn_fused = iv("PFM_FFN_FUSED", 1) != 0;
    k.exact_x6 = iv("PFM_EXACT_X6", 1) != 0;
    k.dec_subbatch = std::max(1, iv("PFM_DEC_SUBBATCH", 2));
    k.ffn_op = iv("PFM_FFN_OP", 1) != 0;
    // 0 unfused; 1 the 64-row k_ffn.hip DEC kernel; 2 the 128-row k_ffn2.hip kernel, hidden split over two workgroups;
    // 3 the 128-row k_ffn2.hip kernel, whole hidden per workgroup
    k.dec_ffn_fused = std::max(0, std::min(iv("PFM_DEC_FFN_FUSED", 1), 3));
    k.ffn_kernel = iv("PFM_FFN_KERNEL", 2) == 1 ? 1 : 2;
    k.ffn_qkv = iv("PFM_FFN_QKV", 1) != 0;
    k.fast_xw = iv("PFM_FAST_XW", 7) & 15;
    if (k.fast_xw & 8) k.fast_xw |= 4;   // the out-projection's planes ride on MODE 6 (v rows split too)
    const int* f = &k.attn_fsmn;
    unsigned long long s = 1469598103934665603ull;   // FNV-1a over the fields
    for (int i = 0; i < PFM_KNOB_FIELDS; ++i) s = (s ^ (unsigned long long)(unsigned)f[i]) * 1099511628211ull;
    k.sig = s;
    t_knobs = k;
    t_knobs_set = true;
}

namespace {

// Workspace generation of one owner (a pfm_handle or a pfm_streams): bumped whenever one of the owner's
// DevBufs is (re)allocated. Captured HIP graphs hold raw buffer addresses, so a graph recorded against
// (handle gen, streams gen) is valid only while both are unchanged. The DevBuf members of an owner bind
// to its counter at construction (GenBind as the owner's first member, GenUnbind as its last).
thread_local std::atomic<unsigned long long>* t_bind_gen = nullptr;
struct GenBind { explicit GenBind(std::atomic<unsigned long long>* g) { t_bind_gen = g; } };
struct GenUnbind { GenUnbind() { t_bind_gen = nullptr; } };

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    std::atomic<unsigned long long>* gen = t_bind_gen;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (gen) gen->fetch_add(1);
        if (p) { hipError_t e = hipFree(p); if (e != hipSuccess) return e; p = nullptr; bytes = 0; }
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    template <typename T> T* as() const { return (T*)p; }
};

// Captured HIP graphs of one owner's launch sequences, keyed by (shape..., knob signature). At most MAX execs
// are kept; the least recently replayed one is evicted (a server's active-stream and token counts vary without
// bound). A graph is valid while its owner's workspace generation is the one it was captured at.
struct GraphCache {
    struct Graph {
        hipGraphExec_t exec = nullptr;
        unsigned long long gen = 0, last_use = 0;
        int seen = 0;
        bool bad = false;
    };
    static constexpr size_t MAX = 64;
    std::map<std::array<unsigned long long, 5>, Graph> graphs;
    unsigned long long use_clock = 0;
    GraphCache() = default;
    GraphCache(const GraphCache&) = delete;
    GraphCache& operator=(const GraphCache&) = delete;
    ~GraphCache() {
        for (auto& kv : graphs)
            if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    }
};

// One registry entry per reference state_dict tensor we consume.
struct WEntry {
    std::vector<int64_t> shape;
    size_t off = 0;        // element offset in the f32 arena
    size_t numel = 0;
    bool set = false;
    int kind = 0;          // 0 plain, 1 cif conv [O][I][k] -> [O][k*I], 2 ignored, 3 fsmn [D,1,K] -> [K][D]
};

struct EncLayer {
    size_t ln1g, ln1b, wqkv, bqkv, wo, bo, fsmn, ln2g, ln2b, w1, b1, w2, b2;
    int din;
    size_t ffp = 0;   // fast mode: element offset of the packed W1 | W2 ring tiles in ffn_pack (k_ffn.hip)
    size_t opp = 0;   // ... and of the layer's first packed tile (Wo, or Wo's two planes under PFM_FAST_XW bit 8)
    bool qkv_next = false;   // k_ffn2.hip: ... followed by the next layer's packed Wqkv (ffn2_kernel MODE 4)
};
struct DecLayer { size_t fsmn, wq, bq, wo, bo, w1, b1, w2, ng, nb, n1g, n1b, n2g, n2b, n3g, n3b; };

}  // namespace

struct pfm_handle {
    std::atomic<unsigned long long> buf_gen{0};   // workspace generation (captured streaming graphs)
    GenBind gen_bind_{&buf_gen};                  // binds every DevBuf member below to buf_gen
    pfm_config cfg;
    int device = 0;
    std::unordered_map<std::string, WEntry> reg;
    size_t arena_elems = 0;
    DevBuf arena;                  // all f32 weights
    DevBuf arena_bf;               // bf16 copies of GEMM weights (same element offsets)
    DevBuf qkv0_pad;               // fast mode: layer 0's bf16 QKV weights with K padded to a multiple of 64
    DevBuf ffn_pack;               // fused-FFN weight tiles of every encoder layer (bf16, LDS-image order)
    bool ffn_ready = false;
    // fast mode, PFM_FAST_XW: weights as two bf16 planes [hi | lo] (split3 planes 0, 1; plane 2 unused): the
    // predictor conv ([D][3D]), encoder layer 0's QKV (K padded to 64) / Wo / W1 / W2, and layer 1's QKV with
    // only its v rows' lo plane nonzero (bit 4: layer 1's QKV follows the unfused layer 0 as a GEMM)
    DevBuf xw_pred, xw_qkv0, xw_wo0, xw_w10, xw_w20, xw_qkv1, xw_tmp;
    int xw_kind = 0;               // the PFM_FAST_XW bits the planes / the ffn_pack layout were built for
    bool xw_ready = false;
    DevBuf logits, ctcx, beam_fs, beam_is;   // pfm_run_beam: decoder / CTC log-probs and the search's scratch
    DevBuf beam_fail;                        // one device word: a search's cross-workgroup barrier timed out
    DevBuf beam_nf;                          // pfm_stream_step_beam: CIF fire counts when the caller passes none
    bool want_logits = false;      // set by pfm_run_beam around its pfm_run: the output layer writes logits
    int last_L = 0;                // decoder positions of the last pfm_run (max token count)
    int ffn_kind = 0;              // which fused-FFN kernel the packed encoder weights (ffn_pack) are ordered for
    DevBuf dffn_pack, dffn_c;      // decoder FFNs (16 blocks + decoders3): W1 | W2 diag(gamma_F) tiles; c1 | c2
    bool dffn_ready = false;
    int dffn_kind = 0;             // PFM_DEC_FFN_FUSED the decoder pack is ordered for (1 k_ffn.hip, 2 k_ffn2.hip split)
    DevBuf dffn2_part, dffn2_cnt;  // split decoder FFN: per-group partial y / LN_F statistics, tile counters (zeroed)
    size_t dffn2_cnt_n = 0;
    DevBuf arena_x6;               // EXACT mode: three bf16 planes of every GEMM weight (x = x0 + x1 + x2)
    bool x6_ready = false;
    std::map<hipStream_t, std::unique_ptr<DevBuf>> x6_scratch;   // split A operands, one buffer per stream
    std::map<size_t, std::unique_ptr<DevBuf>> x6_pad;   // weights with K % 64 != 0: planes [N][round64(K)] by offset
    std::vector<std::pair<size_t, size_t>> gemm_ranges;   // (off, numel) converted to bf16
    bool bf_ready = false;
    int missing = 0;
    std::vector<EncLayer> enc;
    std::vector<DecLayer> dec;
    size_t an_g, an_b, cif_w, cif_b, cif_ow, cif_ob, dan_g, dan_b, out_w, out_b, d3w1, d3b1, d3w2, d3ng, d3nb,
        d3n1g, d3n1b, wkv_all, bkv_all;
    // SenseVoice (PFM_ARCH_SENSEVOICE): tp_norm, CTC head, query embedding table
    size_t tp_g = 0, tp_b = 0, ctc_w = 0, ctc_b = 0, embed = 0;
    DevBuf Xin, X2, olen, fids, ban_bias;   // query-prefixed input, tp-stack residual, lens + 4, frame argmax
    int ban_tok = -1;                        // token whose bias in ban_bias is -inf
    // workspace
    int capB = 0, capT = 0;
    DevBuf pe, X, Xn, QKV, QKVb, F, O, Ob, H, encp, encpb, Hc, alphas, peaks, nfire, ntok, emb, KV, Xd, Xdn, Hd,
        Hdn, Td, Tdn, Qd, Od, Odb, amv, ami, tok_tmp;
    int pe_T = 0;
    DevBuf fb_ws, fb_tab;
    bool fb_tab_ready = false;
    int32_t* host_ntok = nullptr;
    int host_ntok_cap = 0;
    DevBuf punc_io;                // pfm_run_punc_host: device ids | lens | punc of one call
    int32_t* punc_pin = nullptr;   // ... and their pinned host staging
    int punc_cap = 0;
    hipStream_t punc_st = nullptr;   // ... its work stream (graph capture needs a non-null stream) and entry event
    hipEvent_t punc_ev = nullptr;
    GraphCache punc_graphs;          // ... and one HIP graph of the model's launches per (mode, word count)
    // encoder sub-batch streams: the batch is split into NSUB utterance groups whose layer sequences run
    // concurrently, so one group's HBM-bound phases (LayerNorm, GEMM epilogues, attention) overlap the
    // other's MFMA main loops
    static constexpr int MAXSUB = 4;
    hipStream_t sub_st[MAXSUB] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[MAXSUB] = {nullptr, nullptr, nullptr, nullptr};
    DevBuf Xf;                               // SenseVoice: tp_norm output (CTC GEMM input), [M, D]
    DevBuf lnst1, lnst2;                     // folded LayerNorm row statistics: [M, D/64] (mean, M2) partials
    // side stream: the decoder's memory K|V projection overlaps the predictor / CIF / token-count sync
    hipStream_t st2 = nullptr;
    hipEvent_t ev_enc = nullptr, ev_kv = nullptr;
    // fast mode: the projection in KVG layer groups, one event each (the decoder's layer l waits for its group only)
    static constexpr int KVG = 4;
    hipEvent_t ev_kvg[KVG] = {};
    // live profiling: event pairs per launch, per kernel class
    struct ProfRec { hipEvent_t a, b; int kc, kc2; double flops, bytes; };
    bool prof_on = false;
    std::vector<ProfRec> prof;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    double prof_ms[4] = {0, 0, 0, 0}, prof_fl[4] = {0, 0, 0, 0}, prof_by[4] = {0, 0, 0, 0};
    long long prof_n[4] = {0, 0, 0, 0};

    GenUnbind gen_unbind_;                   // last member: DevBufs created later are unbound

    float* w(size_t off) const { return arena.as<float>() + off; }
    bf16* wb(size_t off) const { return arena_bf.as<bf16>() + off; }
};

namespace {

size_t add_entry(pfm_handle* h, const std::string& name, std::vector<int64_t> shape, int kind = 0,
                 bool gemm = false) {
    WEntry e;
    e.shape = shape;
    e.numel = 1;
    for (auto s : shape) e.numel *= (size_t)s;
    e.kind = kind;
    if (kind != 2) {
        e.off = h->arena_elems;
        h->arena_elems += (e.numel + 63) & ~size_t(63);   // 256-B aligned tensors
        if (gemm) h->gemm_ranges.push_back({e.off, e.numel});
        h->missing++;
    }
    h->reg[name] = e;
    return e.off;
}

void build_registry(pfm_handle* h) {
    const pfm_config& c = h->cfg;
    const int D = c.d_model, F = c.ffn, K = c.kernel_size, I = c.input_size, V = c.vocab_size;
    const bool sv = c.arch == PFM_ARCH_SENSEVOICE;
    const bool punc = c.arch == PFM_ARCH_PUNC;
    const int n_enc = c.enc_blocks + (sv ? c.tp_blocks : 0);
    for (int l = 0; l < n_enc; ++l) {
        const std::string p = l == 0 ? "encoder.encoders0.0"
                              : l < c.enc_blocks ? "encoder.encoders." + std::to_string(l - 1)
                                                 : "encoder.tp_encoders." + std::to_string(l - c.enc_blocks);
        const int din = l == 0 ? I : D;
        EncLayer L;
        L.din = din;
        L.wo = add_entry(h, p + ".self_attn.linear_out.weight", {D, D}, 0, true);
        L.bo = add_entry(h, p + ".self_attn.linear_out.bias", {D});
        L.wqkv = add_entry(h, p + ".self_attn.linear_q_k_v.weight", {3 * D, din}, 0, true);
        L.bqkv = add_entry(h, p + ".self_attn.linear_q_k_v.bias", {3 * D});
        L.fsmn = add_entry(h, p + ".self_attn.fsmn_block.weight", {D, 1, K}, 3);
        L.w1 = add_entry(h, p + ".feed_forward.w_1.weight", {F, D}, 0, true);
        L.b1 = add_entry(h, p + ".feed_forward.w_1.bias", {F});
        L.w2 = add_entry(h, p + ".feed_forward.w_2.weight", {D, F}, 0, true);
        L.b2 = add_entry(h, p + ".feed_forward.w_2.bias", {D});
        L.ln1g = add_entry(h, p + ".norm1.weight", {din});
        L.ln1b = add_entry(h, p + ".norm1.bias", {din});
        L.ln2g = add_entry(h, p + ".norm2.weight", {D});
        L.ln2b = add_entry(h, p + ".norm2.bias", {D});
        h->enc.push_back(L);
    }
    h->an_g = add_entry(h, "encoder.after_norm.weight", {D});
    h->an_b = add_entry(h, "encoder.after_norm.bias", {D});
    if (punc) {   // ct_transformer/model.py:63-68: word embedding + punctuation head
        h->embed = add_entry(h, "embed.weight", {c.n_embed, I});
        h->ctc_w = add_entry(h, "decoder.weight", {V, D});
        h->ctc_b = add_entry(h, "decoder.bias", {V});
        return;
    }
    if (sv) {   // sense_voice/model.py:542-548, ctc/ctc.py:33, model.py:646-648
        h->tp_g = add_entry(h, "encoder.tp_norm.weight", {D});
        h->tp_b = add_entry(h, "encoder.tp_norm.bias", {D});
        h->ctc_w = add_entry(h, "ctc.ctc_lo.weight", {V, D}, 0, true);
        h->ctc_b = add_entry(h, "ctc.ctc_lo.bias", {V});
        h->embed = add_entry(h, "embed.weight", {c.n_embed, I});
        return;
    }
    add_entry(h, "decoder.embed.0.weight", {V, D}, 2);
    h->dan_g = add_entry(h, "decoder.after_norm.weight", {D});
    h->dan_b = add_entry(h, "decoder.after_norm.bias", {D});
    h->out_w = add_entry(h, "decoder.output_layer.weight", {V, D}, 0, true);
    h->out_b = add_entry(h, "decoder.output_layer.bias", {V});
    if (c.ctc_head) {   // Paraformer trained with ctc_weight > 0 (paraformer/model.py:95-100, ctc/ctc.py:33)
        h->ctc_w = add_entry(h, "ctc.ctc_lo.weight", {V, D}, 0, true);
        h->ctc_b = add_entry(h, "ctc.ctc_lo.bias", {V});
    }
    // cross-attention K/V projections of all decoder layers live in one [nL*2D, D] matrix so the
    // encoder memory is projected by ONE GEMM (N = nL*2D) instead of nL small ones.
    const size_t kv_rows = (size_t)c.dec_blocks * 2 * D;
    h->wkv_all = h->arena_elems;
    h->arena_elems += (kv_rows * D + 63) & ~size_t(63);
    h->gemm_ranges.push_back({h->wkv_all, kv_rows * D});
    h->bkv_all = h->arena_elems;
    h->arena_elems += (kv_rows + 63) & ~size_t(63);
    for (int l = 0; l < c.dec_blocks; ++l) {
        const std::string p = "decoder.decoders." + std::to_string(l);
        DecLayer L;
        L.fsmn = add_entry(h, p + ".self_attn.fsmn_block.weight", {D, 1, K}, 3);
        L.wq = add_entry(h, p + ".src_attn.linear_q.weight", {D, D}, 0, true);
        L.bq = add_entry(h, p + ".src_attn.linear_q.bias", {D});
        {   // k_v slices point into wkv_all / bkv_all
            WEntry e; e.shape = {2 * D, D}; e.numel = (size_t)2 * D * D; e.off = h->wkv_all + (size_t)l * 2 * D * D;
            h->reg[p + ".src_attn.linear_k_v.weight"] = e; h->missing++;
            WEntry f; f.shape = {2 * D}; f.numel = 2 * D; f.off = h->bkv_all + (size_t)l * 2 * D;
            h->reg[p + ".src_attn.linear_k_v.bias"] = f; h->missing++;
        }
        L.wo = add_entry(h, p + ".src_attn.linear_out.weight", {D, D}, 0, true);
        L.bo = add_entry(h, p + ".src_attn.linear_out.bias", {D});
        L.w1 = add_entry(h, p + ".feed_forward.w_1.weight", {F, D}, 0, true);
        L.b1 = add_entry(h, p + ".feed_forward.w_1.bias", {F});
        L.w2 = add_entry(h, p + ".feed_forward.w_2.weight", {D, F}, 0, true);
        L.ng = add_entry(h, p + ".feed_forward.norm.weight", {F});
        L.nb = add_entry(h, p + ".feed_forward.norm.bias", {F});
        L.n1g = add_entry(h, p + ".norm1.weight", {D});
        L.n1b = add_entry(h, p + ".norm1.bias", {D});
        L.n2g = add_entry(h, p + ".norm2.weight", {D});
        L.n2b = add_entry(h, p + ".norm2.bias", {D});
        L.n3g = add_entry(h, p + ".norm3.weight", {D});
        L.n3b = add_entry(h, p + ".norm3.bias", {D});
        h->dec.push_back(L);
    }
    const std::string p3 = "decoder.decoders3.0";
    h->d3w1 = add_entry(h, p3 + ".feed_forward.w_1.weight", {F, D}, 0, true);
    h->d3b1 = add_entry(h, p3 + ".feed_forward.w_1.bias", {F});
    h->d3w2 = add_entry(h, p3 + ".feed_forward.w_2.weight", {D, F}, 0, true);
    h->d3ng = add_entry(h, p3 + ".feed_forward.norm.weight", {F});
    h->d3nb = add_entry(h, p3 + ".feed_forward.norm.bias", {F});
    h->d3n1g = add_entry(h, p3 + ".norm1.weight", {D});
    h->d3n1b = add_entry(h, p3 + ".norm1.bias", {D});
    const int kp = c.cif_l_order + c.cif_r_order + 1;
    h->cif_w = add_entry(h, "predictor.cif_conv1d.weight", {D, D, kp}, 1, true);
    h->cif_b = add_entry(h, "predictor.cif_conv1d.bias", {D});
    h->cif_ow = add_entry(h, "predictor.cif_output.weight", {1, D});
    h->cif_ob = add_entry(h, "predictor.cif_output.bias", {1});
}

// Sinusoidal PE table [T][depth] in f32 exactly as funasr/models/transformer/embedding.py:389-413
// evaluates it: inc = f32(log(f32 1e4)) / (depth/2 - 1); inv_i = f32 exp(-i * inc);
// arg = f32(pos * inv_i) with pos = 1..T; sin/cos of the f32 argument, rounded to f32.
void make_pe(std::vector<float>& pe, int T, int depth) {
    const int half = depth / 2;
    pe.assign((size_t)T * depth, 0.f);
    const float lg = logf(10000.0f);
    const float inc = (float)(lg / (double)((float)depth / 2.f - 1.f));
    std::vector<float> inv(half);
    for (int i = 0; i < half; ++i) inv[i] = (float)exp((double)((float)i * -inc));
    for (int t = 0; t < T; ++t) {
        const float pos = (float)(t + 1);
        for (int i = 0; i < half; ++i) {
            const float st = pos * inv[i];
            pe[(size_t)t * depth + i] = (float)sin((double)st);
            pe[(size_t)t * depth + half + i] = (float)cos((double)st);
        }
    }
}

// the fused FFN kernel is written for the Paraformer / SenseVoice encoder width (512 -> 2048 -> 512)
bool ffn_shape_ok(const pfm_config& c) { return c.d_model == 512 && c.ffn == 2048; }

// PFM_FAST_XW bits that apply to this model: the 512 / 2048 encoder (the fused kernels' shapes), Paraformer's
// predictor conv (bit 1) only where the handle has one
int fast_xw_bits(const pfm_handle* h) {
    const pfm_config& c = h->cfg;
    if (c.d_model != 512 || c.ffn != 2048 || h->enc.empty()) return 0;
    int b = pfm_knobs().fast_xw;
    if (c.arch == PFM_ARCH_PUNC) return 0;
    if (c.arch == PFM_ARCH_SENSEVOICE) b &= ~1;
    return b;
}

int ensure_bf16(pfm_handle* h, hipStream_t st) {
    if (!h->bf_ready) {
        HIP_TRY(h->arena_bf.ensure(h->arena_elems * sizeof(bf16)));
        for (auto& r : h->gemm_ranges)
            HIP_TRY(pfm_f32_to_bf16(h->w(r.first), h->wb(r.first), (long long)r.second, st));
        // layer 0's QKV weights (K = input_size, e.g. 560) zero-padded to a multiple of 64, so the first
        // projection runs on the 256x256 LDS-DMA kernel (K % 64 == 0) instead of the odd-K fallback
        if (!h->enc.empty() && h->enc[0].din % 64) {
            const int din = h->enc[0].din, Kp = (din + 63) / 64 * 64, N = 3 * h->cfg.d_model;
            HIP_TRY(h->qkv0_pad.ensure((size_t)N * Kp * sizeof(bf16)));
            HIP_TRY(hipMemsetAsync(h->qkv0_pad.p, 0, (size_t)N * Kp * sizeof(bf16), st));
            HIP_TRY(hipMemcpy2DAsync(h->qkv0_pad.p, (size_t)Kp * 2, h->wb(h->enc[0].wqkv), (size_t)din * 2,
                                     (size_t)din * 2, N, hipMemcpyDeviceToDevice, st));
        }
        h->bf_ready = true;
    }
    // k_ffn.hip (1) and k_ffn2.hip (2) order their fragments differently (the decoder always runs k_ffn.hip)
    const int fk = pfm_knobs().ffn_kernel;
    if (h->ffn_kind != fk) { h->ffn_ready = false; h->ffn_kind = fk; }
    const int xw = fast_xw_bits(h);
    if (h->xw_kind != xw) { h->xw_ready = false; h->ffn_ready = false; h->xw_kind = xw; }
    if (!h->xw_ready && xw) {
        const int D = h->cfg.d_model, Fd = h->cfg.ffn;
        // planes of an f32 [N][K] weight into dst [3][N][Kp] (K zero-padded to Kp)
        auto planes = [&](DevBuf& dst, const float* w, int N, int K, int Kp) -> hipError_t {
            const size_t n = (size_t)N * Kp;
            hipError_t e = dst.ensure(3 * n * sizeof(bf16));
            if (e != hipSuccess) return e;
            const float* src = w;
            if (Kp != K) {
                if ((e = h->xw_tmp.ensure(n * sizeof(float))) != hipSuccess) return e;
                if ((e = hipMemsetAsync(h->xw_tmp.p, 0, n * sizeof(float), st)) != hipSuccess) return e;
                if ((e = hipMemcpy2DAsync(h->xw_tmp.p, (size_t)Kp * 4, w, (size_t)K * 4, (size_t)K * 4, N,
                                          hipMemcpyDeviceToDevice, st)) != hipSuccess)
                    return e;
                src = h->xw_tmp.as<float>();
            }
            return pfm_split3_planes(src, dst.as<bf16>(), (long long)n, (long long)n, st);
        };
        if (xw & 1) HIP_TRY(planes(h->xw_pred, h->w(h->cif_w), D, 3 * D, 3 * D));
        if ((xw & 2) && !h->enc.empty()) {
            const EncLayer& L0 = h->enc[0];
            const int Kp0 = (L0.din + 63) / 64 * 64;
            HIP_TRY(planes(h->xw_qkv0, h->w(L0.wqkv), 3 * D, L0.din, Kp0));
            HIP_TRY(planes(h->xw_wo0, h->w(L0.wo), D, D, D));
            HIP_TRY(planes(h->xw_w10, h->w(L0.w1), Fd, D, D));
            HIP_TRY(planes(h->xw_w20, h->w(L0.w2), D, Fd, Fd));
            if (h->enc.size() > 1) {   // layer 1's QKV as a split-weight GEMM: lo plane only where bit 4 asks
                const size_t n = (size_t)3 * D * h->enc[1].din;
                HIP_TRY(planes(h->xw_qkv1, h->w(h->enc[1].wqkv), 3 * D, h->enc[1].din, h->enc[1].din));
                HIP_TRY(hipMemsetAsync(h->xw_qkv1.as<bf16>() + n, 0, (size_t)((xw & 4) ? 2 : 3) * D * h->enc[1].din * 2,
                                       st));
            }
        }
        h->xw_ready = true;
    }
    auto pack = [&](const bf16* w1, const bf16* w2, bf16* wp) { return fk == 2 ? pfm_ffn2_pack(w1, w2, wp, st) : pfm_ffn_pack(w1, w2, wp, st); };
    auto pack_o = [&](int kind, const bf16* wo, bf16* wp) { return kind == 2 ? pfm_ffn2_pack_o(wo, wp, st) : pfm_ffn_pack_o(wo, wp, st); };
    if (!h->ffn_ready && ffn_shape_ok(h->cfg) && pfm_knobs().ffn_fused && !h->enc.empty()) {
        // per layer: the out-projection's 32 tiles, then the FFN's 256 (ffp = the FFN tiles); k_ffn2.hip layouts add
        // the next layer's Wqkv as 3 x 32 more (ffn2_kernel MODE 4, the QKV projection as phase 3)
        const bool xv = fk == 2 && (xw & 4);   // MODE 5: the v rows' lo-plane fragments behind the QKV passes
        const bool xo = fk == 2 && (xw & 8);   // MODE 6 / 3: Wo's lo-plane fragments behind its hi ones
        const size_t po = pfm_ffn_packed_o_elems(), pfe = pfm_ffn_packed_elems(),
                     per = (xo ? 2 : 1) * po + pfe + (fk == 2 ? (xv ? 4 : 3) * po : 0);
        const int D = h->cfg.d_model;
        HIP_TRY(h->ffn_pack.ensure(h->enc.size() * per * sizeof(bf16)));
        for (size_t l = 0; l < h->enc.size(); ++l) {
            // [Wo (hi) | Wo lo (bit 8) | FFN | next Wqkv (3 passes) | its v rows' lo plane (bit 4)]
            bf16* base = h->ffn_pack.as<bf16>() + l * per;
            const size_t pw = (xo ? 2 : 1) * po;
            h->enc[l].opp = l * per;
            h->enc[l].ffp = l * per + pw;
            HIP_TRY(pack_o(fk, h->wb(h->enc[l].wo), base));
            if (xo) {
                const size_t n = (size_t)D * D;
                HIP_TRY(h->xw_tmp.ensure(3 * n * sizeof(bf16)));
                HIP_TRY(pfm_split3_planes(h->w(h->enc[l].wo), h->xw_tmp.as<bf16>(), (long long)n, (long long)n, st));
                HIP_TRY(pack_o(fk, h->xw_tmp.as<bf16>() + n, base + po));
            }
            HIP_TRY(pack(h->wb(h->enc[l].w1), h->wb(h->enc[l].w2), base + pw));
            h->enc[l].qkv_next = fk == 2 && l + 1 < h->enc.size() && h->enc[l + 1].din == D;
            if (h->enc[l].qkv_next) HIP_TRY(pfm_ffn2_pack_qkv(h->wb(h->enc[l + 1].wqkv), base + pw + pfe, st));
            if (h->enc[l].qkv_next && xv) {   // lo plane of the next layer's Wqkv; only its v rows are packed
                const size_t n = (size_t)3 * D * D;
                HIP_TRY(h->xw_tmp.ensure(3 * n * sizeof(bf16)));
                HIP_TRY(pfm_split3_planes(h->w(h->enc[l + 1].wqkv), h->xw_tmp.as<bf16>(), (long long)n, (long long)n, st));
                HIP_TRY(pfm_ffn2_pack_qkv_v(h->xw_tmp.as<bf16>() + n, base + pw + pfe + 3 * po, st));
            }
        }
        h->ffn_ready = true;
    }
    const int ndf = h->cfg.dec_blocks > 0 ? h->cfg.dec_blocks + 1 : 0;
    const int dk = pfm_knobs().dec_ffn_fused;
    if (h->dffn_kind != dk) { h->dffn_ready = false; h->dffn_kind = dk; }
    if (!h->dffn_ready && ffn_shape_ok(h->cfg) && dk && ndf > 0 && !h->dec.empty()) {
        // k_ffn.hip (1): per FFN j the 32 out-projection tiles of decoder block j - 1 (folded in front; none for j = 0),
        // then the FFN's 256 tiles; k_ffn2.hip (2): [Wo | half-0 stream][Wo | half-1 stream] (pfm_ffn2_pack_dec)
        const size_t po = pfm_ffn_packed_o_elems(), per = dk >= 2 ? pfm_ffn2_dec_packed_elems() : po + pfm_ffn_packed_elems();
        const int D = h->cfg.d_model;
        HIP_TRY(h->dffn_pack.ensure((size_t)ndf * per * sizeof(bf16)));
        HIP_TRY(h->dffn_c.ensure((size_t)ndf * 2 * D * sizeof(float)));
        for (int j = 0; j < ndf; ++j) {
            const bool d3 = j == ndf - 1;
            const size_t w1 = d3 ? h->d3w1 : h->dec[j].w1, w2 = d3 ? h->d3w2 : h->dec[j].w2;
            const size_t gF = d3 ? h->d3ng : h->dec[j].ng, bF = d3 ? h->d3nb : h->dec[j].nb;
            float* cc = h->dffn_c.as<float>() + (size_t)j * 2 * D;
            bf16* blk = h->dffn_pack.as<bf16>() + (size_t)j * per;
            if (dk >= 2) {
                HIP_TRY(pfm_ffn2_pack_dec(h->wb(w1), h->w(w2), h->w(gF), j > 0 ? h->wb(h->dec[j - 1].wo) : nullptr, blk,
                                          st, dk == 2));
                HIP_TRY(pfm_ffn_dec_consts(h->w(w2), h->w(gF), h->w(bF), cc, cc + D, st));
                continue;
            }
            if (j > 0) HIP_TRY(pfm_ffn_pack_o(h->wb(h->dec[j - 1].wo), blk, st));
            HIP_TRY(pfm_ffn_pack_dec(h->wb(w1), h->w(w2), h->w(gF), h->w(bF), blk + po, cc, cc + D, st));
        }
        h->dffn_ready = true;
    }
    return PFM_OK;
}

// EXACT mode: the split-bf16 planes of every GEMM weight (emulated f32 GEMMs, k_gemm_bf16.hip x6 path)
int ensure_x6(pfm_handle* h, hipStream_t st) {
    if (h->x6_ready || !pfm_knobs().exact_x6) return PFM_OK;
    const size_t n = h->arena_elems;
    HIP_TRY(h->arena_x6.ensure(3 * n * sizeof(bf16)));
    for (auto& r : h->gemm_ranges)
        HIP_TRY(pfm_split3_planes(h->w(r.first), h->arena_x6.as<bf16>() + r.first, (long long)n, (long long)r.second, st));
    // weights whose K is not a multiple of the kernel's 64-deep step (the input_size-wide layer-0 QKV): zero-padded
    // planes [N][3 Kp], built here on the caller's stream BEFORE any utterance-group stream forks from it (the
    // fork event orders every group after them). The buffers are kept across weight reloads and re-split in
    // place, so their addresses (held by captured streaming graphs) stay valid.
    for (auto& L : h->enc) {
        const int K = L.din, N = 3 * h->cfg.d_model;
        if (K % 64 == 0) continue;
        const int Kp = (K + 63) / 64 * 64;
        auto& pb = h->x6_pad[L.wqkv];
        if (!pb) {
            pb.reset(new DevBuf());
            pb->gen = &h->buf_gen;
        }
        HIP_TRY(pb->ensure((size_t)N * Kp * 3 * sizeof(bf16)));
        // rows of W [N][K] -> [N][3 Kp] (x0 | x1 | x2), read by gemm_x6 as three [N][Kp] planes
        HIP_TRY(pfm_split3_rows(h->w(L.wqkv), rowmap_plain(K), N, K, Kp, pb->as<bf16>(), st));
    }
    h->x6_ready = true;
    return PFM_OK;
}

// bytes per row of the encoder LN output buffer: f32 [input_size | d_model] or DT_X3 [3 d_model] bf16
size_t xn_row_bytes(const pfm_config& c) {
    return std::max((size_t)std::max(c.input_size, c.d_model) * 4, (size_t)c.d_model * 6);
}

int reserve(pfm_handle* h, int B, int T) {
    if (B <= h->capB && T <= h->capT) return PFM_OK;
    B = std::max(B, h->capB);
    T = std::max(T, h->capT);
    const pfm_config& c = h->cfg;
    const bool sv = c.arch == PFM_ARCH_SENSEVOICE || c.arch == PFM_ARCH_PUNC;   // encoder-only families
    const size_t D = c.d_model, F = c.ffn, I = c.input_size;
    const size_t M = (size_t)B * T, Lc = (size_t)T + 1, Ml = (size_t)B * Lc;
    const size_t nkv = (size_t)c.dec_blocks * 2 * D;
    const int nt = std::max(pfm_gemm_amax_tiles(c.vocab_size), pfm_gemm_bf16_256_amax_tiles(c.vocab_size));
    HIP_TRY(hipDeviceSynchronize());
    // encoder (both families)
    HIP_TRY(h->X.ensure(M * D * 4));
    HIP_TRY(h->Xn.ensure(M * xn_row_bytes(c)));
    HIP_TRY(h->QKV.ensure(M * 3 * D * 4));
    HIP_TRY(h->QKVb.ensure(M * 3 * D * 2));
    HIP_TRY(h->F.ensure(M * D * 4));
    HIP_TRY(h->O.ensure(M * D * 6));   // f32 rows, or DT_X3 rows (EXACT split operand)
    HIP_TRY(h->Ob.ensure(M * D * 2));
    HIP_TRY(h->H.ensure(M * F * 6));
    HIP_TRY(h->lnst1.ensure(M * (D / 64) * 8));
    HIP_TRY(h->lnst2.ensure(M * (D / 64) * 8));
    if (sv) {   // query-prefixed input, tp residual, CTC argmax partials (rows = frames)
        HIP_TRY(h->Xin.ensure(M * I * 4));
        HIP_TRY(h->X2.ensure(M * D * 4));
        HIP_TRY(h->Xf.ensure(M * D * 4));
        HIP_TRY(h->olen.ensure((size_t)B * 4));
        HIP_TRY(h->fids.ensure(M * 4));
        HIP_TRY(h->amv.ensure(M * nt * 4));
        HIP_TRY(h->ami.ensure(M * nt * 4));
    } else {
        HIP_TRY(h->encp.ensure((size_t)B * (T + 2) * D * 4));
        HIP_TRY(h->encpb.ensure((size_t)B * (T + 2) * D * 2));
        HIP_TRY(h->Hc.ensure(M * D * 4));
        HIP_TRY(h->alphas.ensure((size_t)B * (T + 1) * 4));
        HIP_TRY(h->peaks.ensure((size_t)B * (T + 1) * 4));
        HIP_TRY(h->nfire.ensure((size_t)B * 4));
        HIP_TRY(h->ntok.ensure((size_t)B * 4));
        HIP_TRY(h->emb.ensure(Ml * D * 4));
        HIP_TRY(h->KV.ensure(M * nkv * 4));
        HIP_TRY(h->Xd.ensure(Ml * D * 4));
        HIP_TRY(h->Xdn.ensure(Ml * D * 6));   // EXACT mode: split operands (three bf16 planes)
        HIP_TRY(h->Hd.ensure(Ml * F * 4));
        HIP_TRY(h->Hdn.ensure(Ml * F * 6));
        HIP_TRY(h->Td.ensure(Ml * D * 4));
        HIP_TRY(h->Tdn.ensure(Ml * D * 4));
        HIP_TRY(h->Qd.ensure(Ml * D * 4));
        HIP_TRY(h->Od.ensure(Ml * D * 6));
        HIP_TRY(h->Odb.ensure(Ml * D * 2));
        HIP_TRY(h->amv.ensure(Ml * nt * 4));
        HIP_TRY(h->ami.ensure(Ml * nt * 4));
        HIP_TRY(h->tok_tmp.ensure(Ml * 4));
        // zero the padded encoder layouts once: rows 0 and T+1 of each utterance are never written
        HIP_TRY(hipMemset(h->encp.p, 0, h->encp.bytes));
        HIP_TRY(hipMemset(h->encpb.p, 0, h->encpb.bytes));
    }
    // positional encoding table for the encoder input (depth = input_size)
    std::vector<float> pe;
    make_pe(pe, T, (int)I);
    HIP_TRY(h->pe.ensure(pe.size() * 4));
    HIP_TRY(hipMemcpy(h->pe.p, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
    h->pe_T = T;
    if (h->host_ntok_cap < B) {
        if (h->host_ntok) (void)hipHostFree(h->host_ntok);
        HIP_TRY(hipHostMalloc((void**)&h->host_ntok, (size_t)B * 4, 0));
        h->host_ntok_cap = B;
    }
    h->capB = B;
    h->capT = T;
    return PFM_OK;
}

hipEvent_t next_event(pfm_handle* h) {
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        h->ev_pool.push_back(e);
    }
    return h->ev_pool[h->ev_used++];
}

// Bracket one launch with events when profiling is on.
// kc2 >= 0: the launch is also counted in a second class (PFM_K_FFN2: the dominant kernel inside PFM_K_GEMM).
struct ProfScope {
    pfm_handle* h; hipStream_t st; int kc, kc2; double fl, by; hipEvent_t a = nullptr;
    ProfScope(pfm_handle* h_, hipStream_t st_, int kc_, double fl_, double by_, int kc2_ = -1)
        : h(h_), st(st_), kc(kc_), kc2(kc2_), fl(fl_), by(by_) {
        if (h->prof_on) { a = next_event(h); if (a) (void)hipEventRecord(a, st); }
    }
    ~ProfScope() {
        if (!a) return;
        hipEvent_t b = next_event(h);
        if (!b) return;
        (void)hipEventRecord(b, st);
        h->prof.push_back({a, b, kc, kc2, fl, by});
    }
};

void prof_collect(pfm_handle* h) {
    for (auto& r : h->prof) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            for (const int k : {r.kc, r.kc2}) {
                if (k < 0) continue;
                h->prof_ms[k] += ms;
                h->prof_fl[k] += r.flops;
                h->prof_by[k] += r.bytes;
                h->prof_n[k] += 1;
            }
        }
    }
    h->prof.clear();
    h->ev_used = 0;
}

// Kernel choice: bf16 operands go to the 256x256 LDS-DMA kernel whenever its alignment
// contract holds (K % 64 == 0, 16-B aligned rows); f32 (exact mode) and odd shapes use the
// 128x128 register-staged kernel.
bool use_big_bf16(int dtype, RowMap amap, long long ldw, int K) {
    return dtype == DT_BF16 && pfm_gemm_bf16_256_ok(amap, ldw, K);
}

hipError_t gemm_dispatch(int dtype, const void* A, RowMap amap, const void* W, long long ldw, int M, int N, int K,
                         const GemmEpi& e, hipStream_t st) {
    // <= 64 rows (streaming chunks): weight-streaming kernel over N instead of 2-8 big tiles
    if (dtype == DT_BF16 && pfm_gemm_skinny_ok(A, amap, W, ldw, M, N, K, e))
        return pfm_gemm_skinny(A, amap, W, ldw, M, N, K, e, st);
    if (use_big_bf16(dtype, amap, ldw, K)) return pfm_gemm_bf16_256(A, amap, W, ldw, M, N, K, e, st);
    return pfm_gemm(dtype, A, amap, W, ldw, M, N, K, e, st);
}

bool attn_fsmn_enabled() {   // PFM_ATTN_FSMN=0: separate FSMN kernel (A/B; parity test compares both)
    const PfmKnobs& k = pfm_knobs();
    return k.attn_fsmn && k.attn_waves == 8;
}

bool kv_overlap_enabled() { return pfm_knobs().kv_overlap; }   // 0: memory K|V in-line on the caller's stream

// EXACT-mode GEMM on the split-bf16 path: f32 weights with ld == K inside the arena, K a multiple of 64
bool x6_route(const pfm_handle* h, int dtype, const void* W, long long ldw, int K) {
    if (dtype != DT_F32 || !h || !h->x6_ready || !pfm_knobs().exact_x6 || K % 4 || ldw != K) return false;
    const float* w = (const float*)W;
    return w >= h->arena.as<float>() && w < h->arena.as<float>() + h->arena_elems;
}

int amax_tiles(int dtype, RowMap amap, long long ldw, int N, int K, const pfm_handle* h = nullptr,
               const void* W = nullptr) {
    if (x6_route(h, dtype, W, ldw, K)) return pfm_gemm_bf16_256_amax_tiles(N);
    return use_big_bf16(dtype, amap, ldw, K) ? pfm_gemm_bf16_256_amax_tiles(N) : pfm_gemm_amax_tiles(N);
}

GemmEpi epi_default() {
    GemmEpi e;
    memset(&e, 0, sizeof(e));
    e.alpha = 1.f;
    e.out_map = rowmap_plain(0);
    e.out2_map = rowmap_plain(0);
    return e;
}



// f32 GEMM as split bf16 x6 MFMA: A rows -> [A0 | A1 | A2] in the stream's scratch, then the bf16 256-tile
// kernel over K' = 6K with the weight planes (the same epilogue as every other GEMM)
hipError_t gemm_x6(pfm_handle* h, const float* A, RowMap am, const float* W, int M, int N, int K, const GemmEpi& e,
                   hipStream_t s, const bf16* A3 = nullptr) {
    if (M <= 0 || N <= 0) return hipSuccess;
    constexpr int terms = 6;   // the six products of three bf16 planes that reproduce the f32 GEMM
    if (A3) {   // the producer already wrote [A0 | A1 | A2] (DT_X3 rows, am.ld = 3K)
        if (K % 64) return hipErrorInvalidValue;
        GemmEpi e2 = e;
        e2.x6_k = K;
        e2.x6_ws = (long long)h->arena_elems;
        e2.x6_terms = terms;
        const size_t off = (size_t)(W - h->arena.as<float>());
        return pfm_gemm_bf16_256(A3, am, h->arena_x6.as<bf16>() + off, K, M, N, terms * K, e2, s);
    }
    auto& sc = h->x6_scratch[s];
    if (!sc) {
        sc.reset(new DevBuf());
        sc->gen = &h->buf_gen;   // captured streaming graphs hold its address
    }
    const int Kp = (K + 63) / 64 * 64;   // segments zero-padded to the kernel's K step
    const size_t off = (size_t)(W - h->arena.as<float>());
    const bf16* planes = h->arena_x6.as<bf16>() + off;
    long long ws = (long long)h->arena_elems;
    if (Kp != K) {   // padded planes of this weight (ensure_x6 built them on the caller's stream)
        auto it = h->x6_pad.find(off);
        if (it == h->x6_pad.end() || !it->second || it->second->bytes < (size_t)N * Kp * 3 * sizeof(bf16))
            return hipErrorInvalidValue;
        planes = it->second->as<bf16>();
        ws = Kp;   // plane p of row n at n * 3Kp + p * Kp: ldw = 3 Kp, plane stride Kp
    }
    const size_t need = (size_t)M * 3 * Kp * sizeof(bf16);
    if (need > sc->bytes) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        hipError_t e0 = hipStreamIsCapturing(s, &cs);
        if (e0 != hipSuccess) return e0;
        if (cs != hipStreamCaptureStatusNone) return hipErrorStreamCaptureUnsupported;
        e0 = hipStreamSynchronize(s);   // the old buffer may still be read by queued work
        if (e0 != hipSuccess) return e0;
        e0 = sc->ensure(need);
        if (e0 != hipSuccess) return e0;
    }
    hipError_t er = pfm_split3_rows(A, am, M, K, Kp, sc->as<bf16>(), s);
    if (er != hipSuccess) return er;
    GemmEpi e2 = e;
    e2.x6_k = Kp;
    e2.x6_ws = ws;
    e2.x6_terms = terms;
    return pfm_gemm_bf16_256(sc->p, rowmap_plain(3LL * Kp), planes, Kp == K ? K : 3LL * Kp, M, N, terms * Kp, e2, s);
}

// Per-call launch context shared by the Paraformer and SenseVoice pipelines: numerics mode,
// weight views and launch wrappers that attach algorithmic flops / bytes to every MFMA launch
// for the live roofline (pfm_profile).
struct Run {
    pfm_handle* h;
    hipStream_t st;
    bool fast;
    int dt;          // operand dtype of every contraction: DT_BF16 (fast) / DT_F32 (exact)
    double es;       // operand element size
    float qscale;    // d_k ** -0.5
    bool fuse_fsmn;  // fast mode: encoder FSMN in the attention epilogue
    bool fuse_fsmn_x6 = false;   // EXACT mode (x3): the f32 FSMN in the x6 attention epilogue
    bool x3 = false;     // EXACT mode on split-bf16 x6: producers write GEMM operands as three bf16 planes
    bool raw_input = false;                 // streaming: the stack input is already x sqrt(d) + PE
    const struct ChunkKV* ck = nullptr;     // streaming: self-attention keys = K/V cache ++ window

    Run(pfm_handle* h_, hipStream_t st_, bool fast_) : h(h_), st(st_), fast(fast_) {
        const pfm_config& c = h->cfg;
        dt = fast ? DT_BF16 : DT_F32;
        es = fast ? 2.0 : 4.0;
        qscale = (float)(1.0 / sqrt((double)(c.d_model / c.heads)));
        const int lenc = (c.kernel_size - 1) / 2 + (c.enc_sanm_shift > 0 ? c.enc_sanm_shift : 0);
        fuse_fsmn = fast && c.kernel_size == 11 && lenc == 5 && c.d_model / c.heads == 128 && attn_fsmn_enabled();
        x3 = !fast && h->x6_ready && pfm_knobs().exact_x6 && c.d_model % 64 == 0 && c.ffn % 64 == 0 &&
             c.d_model / c.heads == 128;
        fuse_fsmn_x6 = x3 && c.kernel_size == 11 && lenc == 5 && pfm_knobs().attn_fsmn;
    }
    const void* W(size_t off) const { return fast ? (const void*)h->wb(off) : (const void*)h->w(off); }
    const float* P(size_t off) const { return h->w(off); }

    hipError_t gemm(int dtp, const void* A, RowMap am, const void* Wt, long long ldw, int Mm, int N, int Kk,
                    const GemmEpi& e, hipStream_t s = nullptr) const {
        if (!s) s = st;
        const double fl = 2.0 * Mm * N * Kk;
        const double by = ((double)Mm * Kk + (double)N * Kk) * es +
                          (double)Mm * N * (e.out ? (e.out_dtype == DT_F32 ? 4.0 : 2.0) : 0.0) +
                          (e.res0 ? (e.res0_bf16 ? 2.0 : 4.0) * Mm * N : 0.0) + (e.res1 ? 4.0 * Mm * N : 0.0) +
                          (e.out2 ? 2.0 * Mm * N : 0.0);
        ProfScope ps(h, s, PFM_K_GEMM, fl, by);
        if (!fast && x6_route(h, dtp, Wt, ldw, Kk))
            return gemm_x6(h, (const float*)A, am, (const float*)Wt, Mm, N, Kk, e, s);
        return gemm_dispatch(dtp, A, am, Wt, ldw, Mm, N, Kk, e, s);
    }
    // fast mode, PFM_FAST_XW: bf16 A [Mm, Kk] times a weight kept as two bf16 planes (planes: [hi | lo], `plane`
    // elements apart, rows of ldw): the 256-tile kernel's split-weight mode, K' = 2 Kk (2 M N K algorithmic flops)
    hipError_t gemm_xw(const void* A, RowMap am, const bf16* planes, long long ldw, long long plane, int Mm, int N,
                       int Kk, const GemmEpi& e, hipStream_t s = nullptr) const {
        if (!s) s = st;
        const double fl = 2.0 * Mm * N * Kk;
        const double by = ((double)Mm * Kk + 2.0 * N * Kk) * 2.0 +
                          (double)Mm * N * (e.out ? (e.out_dtype == DT_F32 ? 4.0 : 2.0) : 0.0) +
                          (e.res0 ? (e.res0_bf16 ? 2.0 : 4.0) * Mm * N : 0.0) + (e.res1 ? 4.0 * Mm * N : 0.0);
        ProfScope ps(h, s, PFM_K_GEMM, fl, by);
        GemmEpi e2 = e;
        e2.x6_k = Kk;
        e2.x6_ws = plane;
        e2.x6_terms = 2;
        return pfm_gemm_bf16_256(A, am, planes, ldw, Mm, N, 2 * Kk, e2, s);
    }
    // A = LN(x) g + b, then the GEMM: chunk-sized fast-mode steps (<= 64 rows, K 512) run both in one skinny kernel
    // (the rows normalised into LDS, k_gemm_skinny.hip); otherwise the LayerNorm writes `xn` (layout xnm, the GEMM's
    // operand dtype) and the GEMM reads it
    hipError_t ln_gemm(const float* x, RowMap xm, size_t g, size_t b, void* xn, RowMap xnm, const void* Wt, long long ldw,
                       int Mm, int N, int Kk, const GemmEpi& e) const {
        const pfm_config& c = h->cfg;
        if (fast && pfm_gemm_skinny_ln_ok(x, xm, Wt, ldw, Mm, N, Kk, e)) {
            ProfScope ps(h, st, PFM_K_GEMM, 2.0 * Mm * N * Kk,
                         (double)Mm * Kk * 4.0 + (double)N * Kk * 2.0 +
                             (double)Mm * N * (e.out_dtype == DT_F32 ? 4.0 : 2.0));
            return pfm_gemm_skinny_ln(x, xm, P(g), P(b), c.ln_eps, Wt, ldw, Mm, N, e, st);
        }
        hipError_t er = pfm_layernorm(x, xm, Mm, Kk, P(g), P(b), c.ln_eps, nullptr, 0, 1.f, xn, xnm, dt, nullptr,
                                      rowmap_plain(0), 0, st);
        if (er != hipSuccess) return er;
        return gemm(dt, xn, xnm, Wt, ldw, Mm, N, Kk, e);
    }
    // EXACT-mode GEMM whose A operand a producer wrote as DT_X3 rows (am.ld = 3K); weights f32 in the arena
    hipError_t gemm3(const void* A3, RowMap am, const void* Wt, long long ldw, int Mm, int N, int Kk, const GemmEpi& e,
                     hipStream_t s = nullptr) const {
        if (!s) s = st;
        if (!x6_route(h, DT_F32, Wt, ldw, Kk) || Kk % 64) return hipErrorInvalidValue;
        const double fl = 2.0 * Mm * N * Kk;
        const double by = ((double)Mm * Kk + (double)N * Kk) * 4.0 +
                          (double)Mm * N * (e.out ? (e.out_dtype == DT_F32 ? 4.0 : e.out_dtype == DT_X3 ? 6.0 : 2.0) : 0.0) +
                          (e.res0 ? (e.res0_bf16 ? 2.0 : 4.0) * Mm * N : 0.0) + (e.res1 ? 4.0 * Mm * N : 0.0);
        ProfScope ps(h, s, PFM_K_GEMM, fl, by);
        return gemm_x6(h, nullptr, am, (const float*)Wt, Mm, N, Kk, e, s, (const bf16*)A3);
    }
    // EXACT-mode attention writing the out-projection's split operand (out3 rows of 3 x d_model bf16)
    // (fsmn_wT / fsmn_out: the encoder FSMN block fused into the epilogue, f32 rows of d_model)
    hipError_t attn3(const float* q, RowMap qm, const float* k, RowMap km, const float* v, RowMap vm, bf16* out3,
                     const int* kl, int Bb, int Tq, int Tk, const float* fsmn_wT = nullptr,
                     float* fsmn_out = nullptr) const {
        const pfm_config& c = h->cfg;
        const double dk = c.d_model / c.heads;
        const double fl = 4.0 * Bb * Tq * (double)Tk * dk * c.heads;
        const double by = ((double)Bb * Tq + 2.0 * Bb * Tk) * c.d_model * 4.0 + (double)Bb * Tq * c.d_model * 6.0;
        ProfScope ps(h, st, PFM_K_ATTN, fl, by);
        return pfm_attention_x3(q, qm, k, km, v, vm, out3, kl, Bb, Tq, Tk, c.heads, (int)dk, qscale, fsmn_wT,
                                fsmn_out, c.d_model, st);
    }
    // fast-mode streaming attention over the gathered [cache ; window] keys with the cache retain fused
    // (pfm_attention_retain); hipErrorNotSupported: nothing ran, the caller takes the separate launches
    hipError_t attn_rt(const bf16* q, RowMap qm, void* kv, bf16* o2, const int* kl, int Bb, int Tq, int Tk,
                       const SPrm* prm, void* cache, int C, int drop, int dec, const int* ntok) const {
        const pfm_config& c = h->cfg;
        const double dk = c.d_model / c.heads;
        const double fl = 4.0 * Bb * Tq * (double)Tk * dk * c.heads;
        const double by = ((double)Bb * Tq + 2.0 * Bb * Tk) * c.d_model * 2.0 + (double)Bb * Tq * c.d_model * 2.0;
        ProfScope ps(h, st, PFM_K_ATTN, fl, by);
        return pfm_attention_retain(q, qm, kv, Bb, Tq, Tk, o2, c.d_model, kl, c.heads, (int)dk,
                                    qscale, prm, cache, C, drop, dec, ntok, st);
    }
    hipError_t attn(int dtp, const void* q, RowMap qm, const void* k, RowMap km, const void* v, RowMap vm, float* o,
                    long long ldo, void* o2, const int* kl, int Bb, int Tq, int Tk) const {
        const pfm_config& c = h->cfg;
        const double dk = c.d_model / c.heads;
        const double fl = 4.0 * Bb * Tq * (double)Tk * dk * c.heads;
        const double by = ((double)Bb * Tq + 2.0 * Bb * Tk) * c.d_model * es + (double)Bb * Tq * c.d_model * (o ? 4 : 2);
        ProfScope ps(h, st, PFM_K_ATTN, fl, by);
        return pfm_attention(dtp, q, qm, k, km, v, vm, o, ldo, o2, kl, Bb, Tq, Tk, c.heads, (int)dk, qscale, st);
    }
};

// Streaming encoder self-attention with encoder_chunk_look_back (sanm/attention.py:313-339): per layer the
// keys are [that layer's K/V cache ; the window's K|V rows], gathered into buf [n][Tk][2d]; afterwards
// the cache keeps the last C rows of [cache ; window minus its `drop` look-ahead rows].
struct ChunkKV {
    void* cache;              // [layers][slots][C][2d] in the operand dtype
    long long layer_stride;   // elements per layer
    int C, drop, Tk;
    void* buf;                // [n][Tk][2d]
    const SPrm* prm;          // device, n entries
    const int* klen;          // device [n]: cle + tw
};

// LayerNorm that closes an encoder stack (after_norm / tp_norm): out (+ optional second copy).
struct FinalLN {
    size_t g, b;
    void* out; RowMap omap; int odt;
    void* out2; RowMap o2map; int o2dt;
};

// Encoder workspace of one utterance group: the handle's buffers from row r0 on (each buffer is
// sized for its widest row, so a group's region never overlaps another group's).
struct EncWs { void* Xn; float* QKV; bf16* QKVb; float* F; float* O; bf16* Ob; void* H; float2* st1; float2* st2; };
EncWs enc_ws(pfm_handle* h, long long r0) {
    const pfm_config& c = h->cfg;
    const long long D = c.d_model, I = c.input_size, Fd = c.ffn;
    EncWs w;
    w.Xn = (char*)h->Xn.p + r0 * (long long)xn_row_bytes(c);
    w.QKV = h->QKV.as<float>() + r0 * 3 * D;
    w.QKVb = h->QKVb.as<bf16>() + r0 * 3 * D;
    w.F = h->F.as<float>() + r0 * D;
    w.O = (float*)((char*)h->O.p + r0 * D * 6);
    w.Ob = h->Ob.as<bf16>() + r0 * D;
    w.H = (char*)h->H.p + r0 * Fd * 6;
    w.st1 = (float2*)h->lnst1.p + r0 * (D / 64);
    w.st2 = (float2*)h->lnst2.p + r0 * (D / 64);
    return w;
}

// Encoder layers [l0, l1) of h->enc (EncoderLayerSANM, sanm/encoder.py:72-148 ==
// sense_voice/model.py:329-405) on the f32 residual X [B*T, D], then the closing LayerNorm `fin`.
// l0 == 0: the stack input is x_in [B*T, input_size] (before x sqrt(d) + PE, encoder.py:378-379),
// and layer 0 has no residual (in_size != size, encoder.py:129-137). lens: valid frames per utterance.
int encoder_stack(const Run& r, const float* x_in, const int* lens, int B, int T, int l0, int l1, float* X,
                  const FinalLN& fin, const EncWs& ws) {
    pfm_handle* h = r.h;
    const pfm_config& c = h->cfg;
    const hipStream_t st = r.st;
    const bool fast = r.fast;
    const int dt = r.dt;
    const int D = c.d_model, Fd = c.ffn, I = c.input_size, K = c.kernel_size;
    const long long M = (long long)B * T;
    const int lenc = (K - 1) / 2 + (c.enc_sanm_shift > 0 ? c.enc_sanm_shift : 0);
    void* Xn = ws.Xn;   // LN output, f32 (exact) or bf16 (fast)
    float* QKV = ws.QKV;
    bf16* QKVb = ws.QKVb;
    float* Fm = ws.F;
    bf16* Fb = (bf16*)ws.F;   // fast mode: FSMN memory in bf16 (same buffer)
    float* O = ws.O;
    bf16* Ob = ws.Ob;
    void* Hh = ws.H;
    const RowMap plain = rowmap_plain(0);
    // fast mode, full-size batches: LN2 -> FFN -> residual -> next layer's LN1 as ONE kernel per layer
    // (k_ffn.hip); chunk-sized streaming steps keep the weight-streaming GEMMs
    const bool ffn_fused = fast && h->ffn_ready && pfm_knobs().ffn_fused && M >= 4096;
    // EXACT mode: LayerNorm, attention and FFN w1 write their consumer GEMM's operand in split form
    // (three bf16 planes, DT_X3) instead of f32 + a separate split pass
    const bool x3 = r.x3 && !r.ck;
    const RowMap xmap3 = rowmap_plain(x3 ? 3 * D : D);
    // fast mode, offline: layer 0's K = input_size padded to a multiple of 64 (zero columns, qkv0_pad)
    const int Kp0 = (I + 63) / 64 * 64;
    const bool pad0 = fast && !r.raw_input && !r.ck && I % 64 && h->qkv0_pad.p && l0 == 0;
    const int lndt = x3 ? DT_X3 : dt;
    bool qkv_ready = false;   // the previous layer's fused FFN kernel already wrote this layer's q|k|v (QKVb)
    // PFM_FAST_XW bit 2: layer 0 with split-plane weights, unfused (offline full batches on the fused path only)
    const int xw = fast && !r.ck && !r.raw_input && ffn_fused && h->xw_ready ? h->xw_kind : 0;
    const bool xw0 = (xw & 2) && l0 == 0 && pad0;
    for (int l = l0; l < l1; ++l) {
        const EncLayer& L = h->enc[l];
        const int din = L.din;
        // the previous layer's fused kernel wrote this layer's LN1 (and, MODE 4/5, its q|k|v)
        const bool prev_fused = ffn_fused && l > l0 && !(xw0 && l == 1);
        if (l == 0 && r.raw_input)   // streaming: the window already holds x sqrt(d) + PE
            HIP_TRY(pfm_layernorm(x_in, rowmap_plain(I), (int)M, I, r.P(L.ln1g), r.P(L.ln1b), c.ln_eps, nullptr, 0,
                                  1.f, Xn, rowmap_plain(I), dt, nullptr, plain, 0, st));
        else if (l == 0 && pad0) {   // ... into rows of Kp0 columns whose tail stays zero (padded K)
            HIP_TRY(hipMemset2DAsync((char*)Xn + (size_t)I * 2, (size_t)Kp0 * 2, 0, (size_t)(Kp0 - I) * 2, M, st));
            HIP_TRY(pfm_layernorm(x_in, rowmap_plain(I), (int)M, I, r.P(L.ln1g), r.P(L.ln1b), c.ln_eps,
                                  h->pe.as<float>(), T, sqrtf((float)D), Xn, rowmap_plain(Kp0), dt, nullptr, plain, 0,
                                  st));
        } else if (l == 0)   // x = x_in * sqrt(d_model) + PE ; LN1
            HIP_TRY(pfm_layernorm(x_in, rowmap_plain(I), (int)M, I, r.P(L.ln1g), r.P(L.ln1b), c.ln_eps,
                                  h->pe.as<float>(), T, sqrtf((float)D), Xn, rowmap_plain(I), dt, nullptr, plain, 0,
                                  st));
        else if (!prev_fused && (x3 || !fast))   // fused FFN: the previous layer's kernel wrote LN1(x)
            HIP_TRY(pfm_layernorm(X, rowmap_plain(D), (int)M, D, r.P(L.ln1g), r.P(L.ln1b), c.ln_eps, nullptr, 0, 1.f,
                                  Xn, xmap3, lndt, nullptr, plain, 0, st));
        // layer 1 behind the split-weight layer 0, v rows with split weights too: LN1 -> Xn, then the 2-plane GEMM
        if (xw0 && l == 1 && (xw & 4) && !qkv_ready) {
            HIP_TRY(pfm_layernorm(X, rowmap_plain(D), (int)M, D, r.P(L.ln1g), r.P(L.ln1b), c.ln_eps, nullptr, 0, 1.f,
                                  Xn, rowmap_plain(D), DT_BF16, nullptr, plain, 0, st));
            GemmEpi e = epi_default();
            e.bias = r.P(L.bqkv);
            e.out = QKVb; e.out_map = rowmap_plain(3 * D); e.out_dtype = DT_BF16;
            HIP_TRY(r.gemm_xw(Xn, rowmap_plain(din), h->xw_qkv1.as<bf16>(), din, 3LL * D * din, (int)M, 3 * D, din, e));
            qkv_ready = true;
        }
        // fast mode, l > 0 without the fused FFN in front: LN1 and the QKV projection through Run::ln_gemm
        const bool ln1_fold = l > 0 && fast && !x3 && !prev_fused;
        bool kv_built = false;   // streaming: the QKV launch also wrote the key buffer and the FSMN block
        if (!qkv_ready && ln1_fold) {
            GemmEpi e = epi_default();
            e.bias = r.P(L.bqkv);
            e.out = QKVb; e.out_map = rowmap_plain(3 * D); e.out_dtype = DT_BF16;
            if (r.ck && K == 11 && lenc == 5 && din == D) {
                const ChunkKV& ck = *r.ck;
                ProfScope ps(h, st, PFM_K_GEMM, 2.0 * M * 3 * D * din,
                             (double)M * din * 4.0 + 3.0 * D * din * 2.0 + (double)M * 3 * D * 2.0);
                const hipError_t eq = pfm_gemm_skinny_ln_qkv(
                    X, rowmap_plain(D), r.P(L.ln1g), r.P(L.ln1b), c.ln_eps, r.W(L.wqkv), din, (int)M, 3 * D, e, ck.prm,
                    B, T, (const bf16*)ck.cache + (size_t)l * ck.layer_stride, ck.C, (bf16*)ck.buf, ck.Tk, r.P(L.fsmn),
                    Fb, D, st);
                if (eq != hipErrorNotSupported) {
                    HIP_TRY(eq);
                    kv_built = true;
                }
            }
            if (!kv_built)
                HIP_TRY(r.ln_gemm(X, rowmap_plain(D), L.ln1g, L.ln1b, Xn, rowmap_plain(D), r.W(L.wqkv), din, (int)M,
                                  3 * D, din, e));
        } else if (!qkv_ready) {   // q|k|v = LN1(x) Wqkv^T + b   (fast mode: bf16 only — attention and FSMN read bf16)
            GemmEpi e = epi_default();
            e.bias = r.P(L.bqkv);
            if (fast) { e.out = QKVb; e.out_map = rowmap_plain(3 * D); e.out_dtype = DT_BF16; }
            else { e.out = QKV; e.out_map = rowmap_plain(3 * D); e.out_dtype = DT_F32; }
            if (x3 && l > 0) {
                HIP_TRY(r.gemm3(Xn, xmap3, r.W(L.wqkv), din, (int)M, 3 * D, din, e));
            } else if (l == 0 && xw0) {
                HIP_TRY(r.gemm_xw(Xn, rowmap_plain(Kp0), h->xw_qkv0.as<bf16>(), Kp0, 3LL * D * Kp0, (int)M, 3 * D, Kp0,
                                  e));
            } else if (l == 0 && pad0) {
                HIP_TRY(r.gemm(dt, Xn, rowmap_plain(Kp0), h->qkv0_pad.p, Kp0, (int)M, 3 * D, Kp0, e));
            } else {
                HIP_TRY(r.gemm(dt, Xn, rowmap_plain(din), r.W(L.wqkv), din, (int)M, 3 * D, din, e));
            }
        }
        qkv_ready = false;
        // FSMN memory on v (attention.py:207-223) + masked MHA. Fast mode: the FSMN runs in the attention
        // kernel's epilogue (each block owns its rows x head channels; V is L2-resident) when the shape
        // allows (K 11, left 5); bf16 in / bf16 out either way
        if (r.ck) {   // streaming with look-back: FSMN over the window, attention over cache ++ window
            const ChunkKV& ck = *r.ck;
            const size_t es = fast ? 2 : 4;
            const void* qkv = fast ? (const void*)QKVb : (const void*)QKV;
            void* cache = (char*)ck.cache + (size_t)l * ck.layer_stride * es;
            if (kv_built) {   // written by the QKV launch above
            } else if (fast && K == 11 && lenc == 5) {   // the gather and the window's FSMN as one launch
                HIP_TRY(pfm_kv_gather_fsmn((const bf16*)cache, ck.C, ck.prm, B, QKVb + D, 3 * D, T, (bf16*)ck.buf, ck.Tk,
                                           2 * D, QKVb + 2 * D, rowmap_plain(3 * D), lens, D, r.P(L.fsmn), Fb, st));
            } else {
                HIP_TRY(pfm_kv_gather(dt, cache, ck.C, ck.prm, B, 0, (const char*)qkv + (size_t)D * es, 3 * D, T, ck.buf,
                                      ck.Tk, 2 * D, st));
                if (fast)
                    HIP_TRY(pfm_fsmn_bf16in(QKVb + 2 * D, rowmap_plain(3 * D), lens, B, T, D, r.P(L.fsmn), K, lenc,
                                            nullptr, nullptr, Fb, st));
                else
                    HIP_TRY(pfm_fsmn(QKV + 2 * D, rowmap_plain(3 * D), lens, B, T, D, r.P(L.fsmn), K, lenc, nullptr, Fm,
                                     nullptr, st));
            }
            // fast mode: the cache retain runs in the attention kernel's tail
            const hipError_t ea = fast ? r.attn_rt(QKVb, rowmap_plain(3 * D), ck.buf, Ob, ck.klen, B, T, ck.Tk, ck.prm, cache, ck.C, ck.drop, 0,
                                                   nullptr)
                                       : hipErrorNotSupported;
            if (ea != hipErrorNotSupported) {
                HIP_TRY(ea);
            } else {
                const RowMap km = rowmap_seg(ck.Tk, (long long)ck.Tk * 2 * D, 2 * D);
                HIP_TRY(r.attn(dt, qkv, rowmap_plain(3 * D), ck.buf, km, (const char*)ck.buf + (size_t)D * es, km,
                               fast ? nullptr : O, D, fast ? (void*)Ob : nullptr, ck.klen, B, T, ck.Tk));
                HIP_TRY(pfm_kv_retain(dt, ck.buf, ck.Tk, ck.prm, B, 0, ck.drop, nullptr, cache, ck.C, 2 * D, st));
            }
        } else if (r.fuse_fsmn) {
            const double dk = c.d_model / c.heads;
            const double fl = 4.0 * B * (double)T * T * dk * c.heads;
            const double by = 3.0 * B * T * c.d_model * 2.0 + 2.0 * B * T * c.d_model * 2.0;
            ProfScope ps(h, st, PFM_K_ATTN, fl, by);
            HIP_TRY(pfm_attention_fsmn(DT_BF16, QKVb, rowmap_plain(3 * D), QKVb + D, rowmap_plain(3 * D),
                                       QKVb + 2 * D, rowmap_plain(3 * D), nullptr, D, Ob, lens, B, T, T, c.heads,
                                       (int)dk, r.qscale, r.P(L.fsmn), Fb, D, st));
        } else if (fast) {
            HIP_TRY(pfm_fsmn_bf16in(QKVb + 2 * D, rowmap_plain(3 * D), lens, B, T, D, r.P(L.fsmn), K, lenc, nullptr,
                                    nullptr, Fb, st));
            HIP_TRY(r.attn(DT_BF16, QKVb, rowmap_plain(3 * D), QKVb + D, rowmap_plain(3 * D), QKVb + 2 * D,
                           rowmap_plain(3 * D), nullptr, D, Ob, lens, B, T, T));
        } else if (x3 && r.fuse_fsmn_x6) {   // EXACT mode: the f32 FSMN in the x6 attention epilogue
            HIP_TRY(r.attn3(QKV, rowmap_plain(3 * D), QKV + D, rowmap_plain(3 * D), QKV + 2 * D, rowmap_plain(3 * D),
                            (bf16*)O, lens, B, T, T, r.P(L.fsmn), Fm));
        } else {
            HIP_TRY(pfm_fsmn(QKV + 2 * D, rowmap_plain(3 * D), lens, B, T, D, r.P(L.fsmn), K, lenc, nullptr, Fm,
                             nullptr, st));
            if (x3)
                HIP_TRY(r.attn3(QKV, rowmap_plain(3 * D), QKV + D, rowmap_plain(3 * D), QKV + 2 * D, rowmap_plain(3 * D),
                                (bf16*)O, lens, B, T, T));
            else
                HIP_TRY(r.attn(DT_F32, QKV, rowmap_plain(3 * D), QKV + D, rowmap_plain(3 * D), QKV + 2 * D,
                               rowmap_plain(3 * D), O, D, nullptr, lens, B, T, T));
        }
        if (xw0 && l == 0) {   // layer 0, split-plane weights, unfused: x1 = O Wo + bo + F (no residual: in 560,
                               // out 512), h = relu(LN2(x1) W1 + b1), x = x1 + h W2 + b2 (encoder.py:120-145)
            {
                GemmEpi e = epi_default();
                e.bias = r.P(L.bo);
                e.res0 = (const float*)Fb; e.ld_res0 = D; e.res0_bf16 = 1;
                if (din == D) { e.res1 = X; e.ld_res1 = D; }
                e.out = X; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
                HIP_TRY(r.gemm_xw(Ob, rowmap_plain(D), h->xw_wo0.as<bf16>(), D, (long long)D * D, (int)M, D, D, e));
            }
            HIP_TRY(pfm_layernorm(X, rowmap_plain(D), (int)M, D, r.P(L.ln2g), r.P(L.ln2b), c.ln_eps, nullptr, 0, 1.f,
                                  Xn, rowmap_plain(D), DT_BF16, nullptr, plain, 0, st));
            {
                GemmEpi e = epi_default();
                e.bias = r.P(L.b1); e.relu = 1;
                e.out = Hh; e.out_map = rowmap_plain(Fd); e.out_dtype = DT_BF16;
                HIP_TRY(r.gemm_xw(Xn, rowmap_plain(D), h->xw_w10.as<bf16>(), D, (long long)Fd * D, (int)M, Fd, D, e));
            }
            {
                GemmEpi e = epi_default();
                e.bias = r.P(L.b2);
                e.res0 = X; e.ld_res0 = D;
                e.out = X; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
                HIP_TRY(r.gemm_xw(Hh, rowmap_plain(Fd), h->xw_w20.as<bf16>(), Fd, (long long)D * Fd, (int)M, D, Fd, e));
            }
            continue;
        }
        // fast mode, full batches: the out-projection runs inside the fused FFN kernel (its phase 0)
        const bool ffn_op = ffn_fused && !r.ck && pfm_knobs().ffn_op;
        if (!ffn_op) {   // x = (x +) linear_out(att) + fsmn   (encoder.py:120-137: no residual when in != out)
            GemmEpi e = epi_default();
            e.bias = r.P(L.bo);
            e.res0 = fast ? (const float*)Fb : Fm; e.ld_res0 = D; e.res0_bf16 = fast ? 1 : 0;
            if (din == D) { e.res1 = X; e.ld_res1 = D; }
            e.out = X; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
            if (x3)
                HIP_TRY(r.gemm3(O, xmap3, r.W(L.wo), D, (int)M, D, D, e));
            else
                HIP_TRY(r.gemm(dt, fast ? (const void*)Ob : (const void*)O, rowmap_plain(D), r.W(L.wo), D, (int)M, D,
                               D, e));
            if (!ffn_fused && (x3 || !fast))   // (fast mode: LN2 runs with the w1 GEMM below, Run::ln_gemm)
                HIP_TRY(pfm_layernorm(X, rowmap_plain(D), (int)M, D, r.P(L.ln2g), r.P(L.ln2b), c.ln_eps, nullptr, 0,
                                      1.f, Xn, xmap3, lndt, nullptr, plain, 0, st));
        }
        if (ffn_fused) {   // x = x + W2 relu(W1 LN2(x) + b1) + b2 ; Xn = LN1_{l+1}(x)
            const bool nxt = l + 1 < l1;
            const double fl = 4.0 * M * (double)D * Fd;
            const double by = (double)M * D * (4.0 + 4.0 + (nxt ? 2.0 : 0.0)) + 2.0 * 2.0 * D * Fd;
            if (ffn_op) {   // x1 = (x +) O Wo^T + bo + fsmn, then the FFN on x1 (encoder.py:120-145)
                const double flo = fl + 2.0 * M * (double)D * D;
                const double byo = by + (double)M * D * 2.0 * 2.0 + 2.0 * D * D - (din == D ? 0.0 : 4.0 * M * D);
                if (nxt && L.qkv_next && h->ffn_kind == 2 && pfm_knobs().ffn_qkv) {
                    // ... and the next layer's q|k|v = LN1_{l+1}(x2) Wqkv^T + b (phase 3: LN1_{l+1} stays in registers)
                    const EncLayer& N = h->enc[l + 1];
                    ProfScope ps(h, st, PFM_K_GEMM, flo + 6.0 * M * (double)D * D,
                                 byo + (double)M * D * (6.0 - 2.0) + 6.0 * D * D, PFM_K_FFN2);
                    // PFM_FAST_XW bit 4: MODE 5 (the v rows' lo-plane fragments packed behind the QKV passes); bit 8:
                    // MODE 6 (Wo's two planes in front)
                    const bf16* wop = h->ffn_pack.as<bf16>() + L.opp;
                    if (xw & 4)
                        HIP_TRY(pfm_ffn2_fused_op_qkv_xv(Ob, Fb, r.P(L.bo), din == D ? X : nullptr, (int)M, r.P(L.ln2g),
                                                         r.P(L.ln2b), c.ln_eps, wop, r.P(L.b1), r.P(L.b2), X,
                                                         r.P(N.ln1g), r.P(N.ln1b), r.P(N.bqkv), QKVb, (xw & 8) != 0,
                                                         st));
                    else
                        HIP_TRY(pfm_ffn2_fused_op_qkv(Ob, Fb, r.P(L.bo), din == D ? X : nullptr, (int)M, r.P(L.ln2g),
                                                      r.P(L.ln2b), c.ln_eps, wop, r.P(L.b1), r.P(L.b2), X, r.P(N.ln1g),
                                                      r.P(N.ln1b), r.P(N.bqkv), QKVb, st));
                    qkv_ready = true;
                    continue;
                }
                ProfScope ps(h, st, PFM_K_GEMM, flo, byo);
                HIP_TRY(((xw & 8) && h->ffn_kind == 2 ? pfm_ffn2_fused_op_xo
                         : h->ffn_kind == 2 ? pfm_ffn2_fused_op : pfm_ffn_fused_op)(
                    Ob, Fb, r.P(L.bo), din == D ? X : nullptr, (int)M, r.P(L.ln2g), r.P(L.ln2b), c.ln_eps,
                    h->ffn_pack.as<bf16>() + L.opp, r.P(L.b1), r.P(L.b2), X, nxt ? r.P(h->enc[l + 1].ln1g) : nullptr,
                    nxt ? r.P(h->enc[l + 1].ln1b) : nullptr, nxt ? (bf16*)Xn : nullptr, st));
                continue;
            }
            ProfScope ps(h, st, PFM_K_GEMM, fl, by);
            HIP_TRY((h->ffn_kind == 2 ? pfm_ffn2_fused : pfm_ffn_fused)(X, (int)M, r.P(L.ln2g), r.P(L.ln2b), c.ln_eps, h->ffn_pack.as<bf16>() + L.ffp,
                                  r.P(L.b1), r.P(L.b2), X, nxt ? r.P(h->enc[l + 1].ln1g) : nullptr,
                                  nxt ? r.P(h->enc[l + 1].ln1b) : nullptr, nxt ? (bf16*)Xn : nullptr, st));
            continue;
        }
        {   // h = relu(LN2(x) W1^T + b1)
            GemmEpi e = epi_default();
            e.bias = r.P(L.b1); e.relu = 1;
            e.out = Hh; e.out_map = rowmap_plain(Fd); e.out_dtype = dt;
            if (x3) {   // h written as w2's split operand
                e.out_map = rowmap_plain(3 * Fd); e.out_dtype = DT_X3;
                HIP_TRY(r.gemm3(Xn, xmap3, r.W(L.w1), D, (int)M, Fd, D, e));
            } else if (fast) {
                HIP_TRY(r.ln_gemm(X, rowmap_plain(D), L.ln2g, L.ln2b, Xn, rowmap_plain(D), r.W(L.w1), D, (int)M, Fd, D, e));
            } else {
                HIP_TRY(r.gemm(dt, Xn, rowmap_plain(D), r.W(L.w1), D, (int)M, Fd, D, e));
            }
        }
        {   // x = x + h W2^T + b2
            GemmEpi e = epi_default();
            e.bias = r.P(L.b2);
            e.res0 = X; e.ld_res0 = D;
            e.out = X; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
            if (x3)
                HIP_TRY(r.gemm3(Hh, rowmap_plain(3 * Fd), r.W(L.w2), Fd, (int)M, D, Fd, e));
            else
                HIP_TRY(r.gemm(dt, Hh, rowmap_plain(Fd), r.W(L.w2), Fd, (int)M, D, Fd, e));
        }
    }
    HIP_TRY(pfm_layernorm(X, rowmap_plain(D), (int)M, D, r.P(fin.g), r.P(fin.b), c.ln_eps, nullptr, 0, 1.f, fin.out,
                          fin.omap, fin.odt, fin.out2, fin.o2map, fin.o2dt, st));
    return PFM_OK;
}


int subbatch_count(pfm_handle* h, int B) {   // PFM_SUBBATCH=n (1 disables); profiling runs unsplit
    const int v = std::min(pfm_knobs().subbatch, (int)pfm_handle::MAXSUB);
    if (h->prof_on) return 1;
    return std::max(1, std::min(v, B));
}

size_t dt_size(int dt) { return dt == DT_F32 ? 4 : 2; }

// encoder_stack over the batch split into utterance groups on concurrent streams (forked from and
// joined back into r.st). Row-addressed arguments are offset per group: x_in / X rows, lens, and the
// closing LN outputs through their RowMaps (one segment per utterance or plain rows).
int encoder_split(pfm_handle* h, const Run& r, const float* x_in, const int* lens, int B, int T, int l0, int l1,
                  float* X, const FinalLN& fin) {
    const pfm_config& c = h->cfg;
    const int ns = subbatch_count(h, B);
    if (ns == 1) return encoder_stack(r, x_in, lens, B, T, l0, l1, X, fin, enc_ws(h, 0));
    if (!h->ev_fork) HIP_TRY(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->ev_fork, r.st));
    for (int k = 0; k < ns; ++k) {
        if (!h->sub_st[k]) {
            HIP_TRY(hipStreamCreateWithFlags(&h->sub_st[k], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&h->ev_join[k], hipEventDisableTiming));
        }
        const int b0 = (int)((long long)B * k / ns), b1 = (int)((long long)B * (k + 1) / ns);
        if (b1 <= b0) continue;
        const long long r0 = (long long)b0 * T;
        HIP_TRY(hipStreamWaitEvent(h->sub_st[k], h->ev_fork, 0));
        Run rk = r;
        rk.st = h->sub_st[k];
        FinalLN fk = fin;
        fk.out = (char*)fin.out + fin.omap.off(r0) * dt_size(fin.odt);
        if (fin.out2) fk.out2 = (char*)fin.out2 + fin.o2map.off(r0) * dt_size(fin.o2dt);
        const int rc = encoder_stack(rk, x_in ? x_in + r0 * c.input_size : nullptr, lens + b0, b1 - b0, T, l0, l1,
                                     X + r0 * c.d_model, fk, enc_ws(h, r0));
        if (rc) return rc;
        HIP_TRY(hipEventRecord(h->ev_join[k], h->sub_st[k]));
        HIP_TRY(hipStreamWaitEvent(r.st, h->ev_join[k], 0));
    }
    return PFM_OK;
}

}  // namespace

// ============================================================================================
extern "C" {

void pfm_config_default(pfm_config* c) {
    c->input_size = 560; c->d_model = 512; c->heads = 4; c->ffn = 2048; c->enc_blocks = 50; c->dec_blocks = 16;
    c->kernel_size = 11; c->enc_sanm_shift = 0; c->dec_sanm_shift = 0; c->vocab_size = 8404;
    c->cif_l_order = 1; c->cif_r_order = 1; c->cif_threshold = 1.f; c->tail_threshold = 0.45f;
    c->smooth_factor = 1.f; c->noise_threshold = 0.f; c->ln_eps = 1e-12f;
    c->arch = PFM_ARCH_PARAFORMER; c->tp_blocks = 0; c->n_embed = 0; c->ctc_head = 0;
}

void pfm_config_sensevoice(pfm_config* c) {
    pfm_config_default(c);
    c->arch = PFM_ARCH_SENSEVOICE; c->dec_blocks = 0; c->tp_blocks = 20; c->n_embed = 16; c->vocab_size = 25055;
    c->ln_eps = 1e-5f;
}

void pfm_config_punc(pfm_config* c) {
    pfm_config_default(c);
    c->arch = PFM_ARCH_PUNC; c->input_size = 256; c->d_model = 256; c->heads = 8; c->ffn = 1024; c->enc_blocks = 4;
    c->dec_blocks = 0; c->tp_blocks = 0; c->vocab_size = 6; c->n_embed = 272727; c->ln_eps = 1e-12f;
}

const char* pfm_last_error(void) { return g_err.c_str(); }

int pfm_create(const pfm_config* cfg, int device, pfm_handle** out) {
    pfm_knobs_refresh();
    if (!cfg || !out) return fail(PFM_E_ARG, "pfm_create: null argument");
    *out = nullptr;
    if (cfg->heads < 1 || cfg->d_model % cfg->heads != 0 ||
        (cfg->arch == PFM_ARCH_PUNC ? (cfg->d_model / cfg->heads != 32 && cfg->d_model / cfg->heads != 64)
                                    : cfg->d_model / cfg->heads != 128))
        return fail(PFM_E_ARG, "pfm_create: head dim must be 128 (32 or 64 for the punctuation model)");
    if (cfg->input_size % 8 || cfg->d_model % 8 || cfg->ffn % 8 || cfg->input_size > 2048 || cfg->ffn > 2048)
        return fail(PFM_E_ARG, "pfm_create: dims must be multiples of 8 and <= 2048");
    if (cfg->enc_blocks < 1 || cfg->dec_blocks < 0 || cfg->kernel_size < 1 || cfg->vocab_size < 1)
        return fail(PFM_E_ARG, "pfm_create: bad block counts");
    if (cfg->arch != PFM_ARCH_PARAFORMER && cfg->arch != PFM_ARCH_SENSEVOICE && cfg->arch != PFM_ARCH_PUNC)
        return fail(PFM_E_ARG, "pfm_create: unknown arch");
    if (cfg->arch == PFM_ARCH_PUNC && (cfg->n_embed < 1 || cfg->vocab_size > 64 || cfg->dec_blocks != 0))
        return fail(PFM_E_ARG, "pfm_create: punctuation model needs n_embed >= 1, <= 64 classes, no decoder");
    if (cfg->arch == PFM_ARCH_PARAFORMER && (cfg->cif_l_order != 1 || cfg->cif_r_order != 1))
        return fail(PFM_E_ARG, "pfm_create: CIF conv must be l_order = r_order = 1");
    if (cfg->arch == PFM_ARCH_SENSEVOICE && (cfg->tp_blocks < 0 || cfg->n_embed < 1))
        return fail(PFM_E_ARG, "pfm_create: SenseVoice needs tp_blocks >= 0 and n_embed >= 1");
    if (cfg->ctc_head != 0 && (cfg->arch != PFM_ARCH_PARAFORMER || cfg->ctc_head != 1))
        return fail(PFM_E_ARG, "pfm_create: ctc_head is 0 / 1 and only for Paraformer (SenseVoice always has one)");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(PFM_E_ARG, "pfm_create: bad device index");
    HIP_TRY(hipSetDevice(device));
    std::unique_ptr<pfm_handle> h(new pfm_handle());
    h->cfg = *cfg;
    h->device = device;
    build_registry(h.get());
    hipError_t e = h->arena.ensure(h->arena_elems * 4);
    if (e != hipSuccess) return fail(PFM_E_NOMEM, "pfm_create: weight arena allocation failed");
    HIP_TRY(hipMemset(h->arena.p, 0, h->arena.bytes));
    *out = h.release();
    g_err.clear();
    return PFM_OK;
}

void pfm_destroy(pfm_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->ev_enc) (void)hipEventDestroy(h->ev_enc);
    if (h->ev_kv) (void)hipEventDestroy(h->ev_kv);
    for (auto e : h->ev_kvg)
        if (e) (void)hipEventDestroy(e);
    if (h->st2) (void)hipStreamDestroy(h->st2);
    for (int k = 0; k < pfm_handle::MAXSUB; ++k) {
        if (h->sub_st[k]) (void)hipStreamDestroy(h->sub_st[k]);
        if (h->ev_join[k]) (void)hipEventDestroy(h->ev_join[k]);
    }
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->host_ntok) (void)hipHostFree(h->host_ntok);
    if (h->punc_pin) (void)hipHostFree(h->punc_pin);
    if (h->punc_st) (void)hipStreamDestroy(h->punc_st);
    if (h->punc_ev) (void)hipEventDestroy(h->punc_ev);
    delete h;
}

// a weight changed: every derived copy (bf16 arena, LN folds, packed FFN tiles, x6 planes, banned-token bias) is stale
static void weight_written(pfm_handle* h, WEntry& e) {
    if (!e.set) { e.set = true; h->missing--; }
    h->bf_ready = false;
    h->ffn_ready = false;
    h->dffn_ready = false;
    h->x6_ready = false;   // ensure_x6 re-splits arena_x6 and the padded planes in place (stable addresses)
    h->xw_ready = false;   // PFM_FAST_XW split planes (predictor conv, layer 0, v rows) are rebuilt from the new weights
    h->ban_tok = -1;   // the banned-token bias copy follows ctc.ctc_lo.bias
}

int pfm_set_weight(pfm_handle* h, const char* name, const void* host_ptr, int dtype, const int64_t* shape,
                   int ndim) {
    pfm_knobs_refresh();
    if (!h || !name || !host_ptr || !shape) return fail(PFM_E_ARG, "pfm_set_weight: null argument");
    if (dtype != PFM_F32) return fail(PFM_E_ARG, "pfm_set_weight: only PFM_F32 host tensors are accepted");
    auto it = h->reg.find(name);
    if (it == h->reg.end()) return fail(PFM_E_NAME, std::string("pfm_set_weight: unknown key ") + name);
    WEntry& e = it->second;
    if ((int)e.shape.size() != ndim) return fail(PFM_E_ARG, std::string("pfm_set_weight: rank mismatch for ") + name);
    for (int i = 0; i < ndim; ++i)
        if (e.shape[i] != shape[i]) return fail(PFM_E_ARG, std::string("pfm_set_weight: shape mismatch for ") + name);
    if (e.kind == 2) return PFM_OK;
    HIP_TRY(hipSetDevice(h->device));
    const float* src = (const float*)host_ptr;
    std::vector<float> tmp;
    if (e.kind == 1) {   // Conv1d [O][I][k] -> GEMM W [O][k*I]: column k*I + i multiplies frame t-1+k, channel i
        const int64_t O = e.shape[0], I = e.shape[1], KK = e.shape[2];
        tmp.resize(e.numel);
        for (int64_t o = 0; o < O; ++o)
            for (int64_t i = 0; i < I; ++i)
                for (int64_t k = 0; k < KK; ++k) tmp[(o * KK + k) * I + i] = src[(o * I + i) * KK + k];
        src = tmp.data();
    }
    if (e.kind == 3) {   // depthwise taps [D][1][K] -> [K][D] (float4-coalesced tap loads)
        const int64_t Dd = e.shape[0], KK = e.shape[2];
        tmp.resize(e.numel);
        for (int64_t d = 0; d < Dd; ++d)
            for (int64_t k = 0; k < KK; ++k) tmp[k * Dd + d] = src[d * KK + k];
        src = tmp.data();
    }
    HIP_TRY(hipMemcpy(h->w(e.off), src, e.numel * 4, hipMemcpyHostToDevice));
    weight_written(h, e);
    return PFM_OK;
}

int pfm_set_weight_device(pfm_handle* h, const char* name, const void* dev_ptr, int dtype, const int64_t* shape,
                          int ndim, void* stream) {
    pfm_knobs_refresh();
    if (!h || !name || !dev_ptr || !shape) return fail(PFM_E_ARG, "pfm_set_weight_device: null argument");
    if (dtype != PFM_F32) return fail(PFM_E_ARG, "pfm_set_weight_device: only PFM_F32 tensors are accepted");
    if ((uintptr_t)dev_ptr % 4) return fail(PFM_E_ARG, "pfm_set_weight_device: source must be 4-B aligned");
    auto it = h->reg.find(name);
    if (it == h->reg.end()) return fail(PFM_E_NAME, std::string("pfm_set_weight_device: unknown key ") + name);
    WEntry& e = it->second;
    if ((int)e.shape.size() != ndim)
        return fail(PFM_E_ARG, std::string("pfm_set_weight_device: rank mismatch for ") + name);
    for (int i = 0; i < ndim; ++i)
        if (e.shape[i] != shape[i])
            return fail(PFM_E_ARG, std::string("pfm_set_weight_device: shape mismatch for ") + name);
    if (e.kind == 2) return PFM_OK;
    CHECK_DEV("pfm_set_weight_device", h->device, {"dev_ptr", dev_ptr});
    HIP_TRY(hipSetDevice(h->device));
    const hipStream_t st = (hipStream_t)stream;
    const float* src = (const float*)dev_ptr;
    if (e.kind == 1)        // Conv1d [O][I][k] -> [O][k][I] (as pfm_set_weight, on the device)
        HIP_TRY(pfm_swap_last2(src, h->w(e.off), e.shape[0], e.shape[1], e.shape[2], st));
    else if (e.kind == 3)   // depthwise taps [D][1][K] -> [K][D]
        HIP_TRY(pfm_swap_last2(src, h->w(e.off), 1, e.shape[0], e.shape[2], st));
    else
        HIP_TRY(hipMemcpyAsync(h->w(e.off), src, e.numel * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));   // the caller may free / reuse its buffer on return
    weight_written(h, e);
    return PFM_OK;
}

int pfm_missing_weights(const pfm_handle* h) { return h ? h->missing : -1; }

int pfm_reserve(pfm_handle* h, int B, int T) {
    pfm_knobs_refresh();
    if (!h || B < 1 || T < 1) return fail(PFM_E_ARG, "pfm_reserve: bad arguments");
    HIP_TRY(hipSetDevice(h->device));
    return reserve(h, B, T);
}

int pfm_lfr_frames(int nsamp) { return pfm_fbank_frames(nsamp); }

int pfm_run(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens, int B, int T,
            int32_t* tokens, int L_cap, int32_t* ntok_out, float* enc_out, float* alphas_out, float* peaks_out) {
    pfm_knobs_refresh();
    if (!h || !feats || !lens || !tokens || !ntok_out) return fail(PFM_E_ARG, "pfm_run: null argument");
    if (B < 1 || T < 1 || L_cap < 0) return fail(PFM_E_ARG, "pfm_run: bad sizes");
    if (mode != PFM_MODE_EXACT && mode != PFM_MODE_FAST) return fail(PFM_E_ARG, "pfm_run: bad mode");
    if (h->missing) return fail(PFM_E_STATE, "pfm_run: " + std::to_string(h->missing) + " weights not set");
    if (h->cfg.arch != PFM_ARCH_PARAFORMER) return fail(PFM_E_STATE, "pfm_run: handle is not a Paraformer");
    CHECK_DEV("pfm_run", h->device, {"feats", feats}, {"lens", lens}, {"tokens", tokens}, {"ntok", ntok_out},
              {"enc_out", enc_out}, {"alphas", alphas_out}, {"peaks", peaks_out});
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    int rc = reserve(h, B, T);
    if (rc) return rc;
    const bool fast = mode == PFM_MODE_FAST;
    if (fast) { rc = ensure_bf16(h, st); if (rc) return rc; }
    else { rc = ensure_x6(h, st); if (rc) return rc; }
    const pfm_config& c = h->cfg;
    const int D = c.d_model, Fd = c.ffn, K = c.kernel_size, nkv = c.dec_blocks * 2 * D;
    const long long M = (long long)B * T;
    const int dt = fast ? DT_BF16 : DT_F32;
    const int ldec = (K - 1) / 2 + (c.dec_sanm_shift > 0 ? c.dec_sanm_shift : 0);
    if (h->prof_on && h->ev_used > 4096) prof_collect(h);
    const double es = fast ? 2.0 : 4.0;
    const Run run(h, st, fast);
    auto GEMM = [&](int dtp, const void* A, RowMap am, const void* Wt, long long ldw, int Mm, int N, int Kk,
                    const GemmEpi& e) -> hipError_t { return run.gemm(dtp, A, am, Wt, ldw, Mm, N, Kk, e); };
    auto ATTN = [&](int dtp, const void* q, RowMap qm, const void* k, RowMap km, const void* v, RowMap vm, float* o,
                    long long ldo, void* o2, const int* kl, int Bb, int Tq, int Tk) -> hipError_t {
        return run.attn(dtp, q, qm, k, km, v, vm, o, ldo, o2, kl, Bb, Tq, Tk);
    };
    auto W = [&](size_t off) -> const void* { return run.W(off); };
    auto P = [&](size_t off) -> const float* { return run.P(off); };
    const RowMap plain = rowmap_plain(0);

    // after_norm -> zero-padded [B][T+2][D] (row 0 and T+1 of each utterance stay zero)
    float* encp = h->encp.as<float>();
    bf16* encpb = h->encpb.as<bf16>();
    const RowMap encmap = rowmap_seg(T, (long long)(T + 2) * D, D);
    // rows 0 and T+1 of every utterance are the conv / tail zero rows; the workspace may hold a
    // previous call's layout (other T), so clear them each call (2*B rows, negligible)
    HIP_TRY(hipMemset2DAsync(encp, (size_t)(T + 2) * D * 4, 0, (size_t)D * 4, B, st));
    HIP_TRY(hipMemset2DAsync(encp + (size_t)(T + 1) * D, (size_t)(T + 2) * D * 4, 0, (size_t)D * 4, B, st));
    if (fast) {
        HIP_TRY(hipMemset2DAsync(encpb, (size_t)(T + 2) * D * 2, 0, (size_t)D * 2, B, st));
        HIP_TRY(hipMemset2DAsync(encpb + (size_t)(T + 1) * D, (size_t)(T + 2) * D * 2, 0, (size_t)D * 2, B, st));
    }

    // ---------------- encoder (sanm/encoder.py:361-430) ----------------
    {
        const FinalLN fin = {h->an_g, h->an_b, encp + D, encmap, DT_F32, fast ? (void*)(encpb + D) : nullptr, encmap,
                             DT_BF16};
        rc = encoder_split(h, run, feats, lens, B, T, 0, c.enc_blocks, h->X.as<float>(), fin);
        if (rc) return rc;
    }
    if (enc_out)
        HIP_TRY(hipMemcpy2DAsync(enc_out, (size_t)T * D * 4, encp + D, (size_t)(T + 2) * D * 4, (size_t)T * D * 4, B,
                                 hipMemcpyDeviceToDevice, st));
    // memory K|V for all decoder layers: [B*T, nL*2D] = enc . Wkv_all^T + b. It needs only the encoder
    // output, so it runs on the side stream while the predictor, the CIF and the host's token-count
    // sync proceed; the caller's stream joins it before the first cross-attention (or any return).
    void* KV = h->KV.p;
    // layers [l0, l1) of it (columns l0 2D .. l1 2D of the [B*T, nL*2D] rows)
    auto launch_kv = [&](hipStream_t s, int l0, int l1) -> hipError_t {
        const int nc = (l1 - l0) * 2 * D;
        GemmEpi e = epi_default();
        e.bias = P(h->bkv_all + (size_t)l0 * 2 * D);
        e.out = (char*)KV + (size_t)l0 * 2 * D * (fast ? 2 : 4); e.out_map = rowmap_plain(nkv); e.out_dtype = dt;
        const void* A = fast ? (const void*)(encpb + D) : (const void*)(encp + D);
        const void* Wg = W(h->wkv_all + (size_t)l0 * 2 * D * D);
        const double fl = 2.0 * M * nc * D;
        const double by = ((double)M * D + (double)nc * D) * es + (double)M * nc * es;
        ProfScope ps(h, s, PFM_K_GEMM, fl, by);
        if (!fast && x6_route(h, dt, Wg, D, D))
            return gemm_x6(h, (const float*)A, encmap, (const float*)Wg, (int)M, nc, D, e, s);
        return gemm_dispatch(dt, A, encmap, Wg, D, (int)M, nc, D, e, s);
    };
    // fast mode: KVG launches of nL / KVG layers each, so the decoder's first layers start on their own group's K|V
    // while the later groups run beside them (the layer loop below waits per group)
    const int kv_groups = (fast && c.dec_blocks % pfm_handle::KVG == 0) ? pfm_handle::KVG : 1;
    const int kv_lpg = std::max(c.dec_blocks / kv_groups, 1);
    const bool kv_async = kv_overlap_enabled() && c.dec_blocks > 0;
    if (kv_async) {
        if (!h->st2) {
            HIP_TRY(hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&h->ev_enc, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&h->ev_kv, hipEventDisableTiming));
            for (auto& e : h->ev_kvg) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(h->ev_enc, st));
        HIP_TRY(hipStreamWaitEvent(h->st2, h->ev_enc, 0));
        for (int g = 0; g < kv_groups; ++g) {
            HIP_TRY(launch_kv(h->st2, g * kv_lpg, g == kv_groups - 1 ? c.dec_blocks : (g + 1) * kv_lpg));
            HIP_TRY(hipEventRecord(h->ev_kvg[g], h->st2));
        }
        HIP_TRY(hipEventRecord(h->ev_kv, h->st2));
    }

    // ---------------- predictor (cif_predictor.py:202-253) ----------------
    {   // relu(conv1d(k=3, pad 1)) as a GEMM over 3 adjacent rows of the padded layout (K = 3D)
        GemmEpi e = epi_default();
        e.bias = P(h->cif_b); e.relu = 1;
        e.out = h->Hc.p; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
        const void* A = fast ? (const void*)encpb : (const void*)encp;
        if (fast && h->xw_ready && (h->xw_kind & 1))   // PFM_FAST_XW bit 1: the conv weights as two bf16 planes
            HIP_TRY(run.gemm_xw(A, rowmap_seg(T, (long long)(T + 2) * D, D), h->xw_pred.as<bf16>(), 3 * D,
                                3LL * D * D, (int)M, D, 3 * D, e));
        else
            HIP_TRY(GEMM(dt, A, rowmap_seg(T, (long long)(T + 2) * D, D), W(h->cif_w), 3 * D, (int)M, D, 3 * D, e));
    }
    float* alphas = h->alphas.as<float>();
    float* peaks = h->peaks.as<float>();
    int* ntok = h->ntok.as<int>();
    const int Lc = T + 1;
    HIP_TRY(pfm_cif_alpha(h->Hc.as<float>(), D, P(h->cif_ow), P(h->cif_ob), lens, B, T, c.smooth_factor,
                          c.noise_threshold, c.tail_threshold, alphas, st));
    HIP_TRY(pfm_cif_fire(alphas, encp + D, rowmap_seg(T + 1, (long long)(T + 2) * D, D), B, T, D, Lc,
                         h->emb.as<float>(), peaks, h->nfire.as<int>(), ntok, st));
    if (alphas_out) HIP_TRY(hipMemcpyAsync(alphas_out, alphas, (size_t)B * (T + 1) * 4, hipMemcpyDeviceToDevice, st));
    if (peaks_out) HIP_TRY(hipMemcpyAsync(peaks_out, peaks, (size_t)B * (T + 1) * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(ntok_out, ntok, (size_t)B * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->host_ntok, ntok, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    int L = 0;
    for (int b = 0; b < B; ++b) L = std::max(L, (int)h->host_ntok[b]);
    L = std::min(L, Lc);   // ntok <= fires <= T+1 frames (+ rounding); decoder never exceeds the CIF rows
    if (L_cap > 0) HIP_TRY(pfm_fill_i32(tokens, (long long)B * L_cap, -1, st));
    h->last_L = L;
    if (L < 1 || c.dec_blocks < 0) {   // model.py:514-515: nothing to decode
        if (kv_async) HIP_TRY(hipStreamWaitEvent(st, h->ev_kv, 0));   // the side stream still reads encp
        return PFM_OK;
    }
    if (h->want_logits) HIP_TRY(h->logits.ensure((size_t)B * L * c.vocab_size * sizeof(float)));

    // ---------------- decoder (paraformer/decoder.py:359-411) ----------------
    const long long Ml = (long long)B * L;
    // compact CIF embeddings [B][T+1][D] -> decoder rows [B][L][D] (acoustic_embeds[:, :L])
    HIP_TRY(hipMemcpy2DAsync(h->Xd.p, (size_t)L * D * 4, h->emb.p, (size_t)Lc * D * 4, (size_t)L * D * 4, B,
                             hipMemcpyDeviceToDevice, st));
    if (!kv_async) HIP_TRY(launch_kv(st, 0, c.dec_blocks));
    // One utterance group [b0, b0 + nb) of the decoder on rg.st: every buffer is row-addressed (rows b*L + t,
    // memory K|V rows b*T + t), so a group is the same launch sequence over offset pointers.
    // split decoder FFN (PFM_DEC_FFN_FUSED=2): every concurrent group gets its own partials and tile counters
    const int ngd = std::max(1, std::min({pfm_knobs().dec_subbatch, (int)pfm_handle::MAXSUB, B, h->prof_on ? 1 : 64}));
    const int gmax = (int)(((long long)B + ngd - 1) / ngd * L);
    const size_t part_n = pfm_ffn2_dec_scratch_floats(gmax), cnt_n = pfm_ffn2_dec_counters(gmax);
    if (fast && h->dffn_ready && h->dffn_kind == 2) {
        HIP_TRY(h->dffn2_part.ensure((size_t)ngd * part_n * sizeof(float)));
        if (h->dffn2_cnt_n < (size_t)ngd * cnt_n) {   // counters start at zero; every launch leaves them zero
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(h->dffn2_cnt.ensure((size_t)ngd * cnt_n * sizeof(unsigned)));
            HIP_TRY(hipMemsetAsync(h->dffn2_cnt.p, 0, (size_t)ngd * cnt_n * sizeof(unsigned), st));
            h->dffn2_cnt_n = (size_t)ngd * cnt_n;
        }
    }
    auto dec_group = [&](const Run& rg, int b0, int nb, int gi) -> int {
        hipStream_t s = rg.st;
        const size_t esz = fast ? 2 : 4;
        // EXACT mode on split-bf16 x6: the LayerNorms feeding a GEMM (LN1, LN3, LN_F, after_norm) and the
        // cross-attention write that GEMM's A operand as three bf16 planes (DT_X3, 6 B per element)
        const bool x3d = rg.x3;
        const size_t xsz = x3d ? 6 : esz;
        const int ndt = x3d ? DT_X3 : dt;
        const RowMap xdm = rowmap_plain(x3d ? 3 * D : D), hdm = rowmap_plain(x3d ? 3 * Fd : Fd);
        const long long r0 = (long long)b0 * L;
        const int Mg = (int)((long long)nb * L);
        float* Xd = h->Xd.as<float>() + r0 * D;
        void* Xdn = h->Xdn.as<char>() + r0 * D * xsz;
        void* Hd = h->Hd.as<char>() + r0 * Fd * esz;   // fast: bf16 hidden, exact: f32
        void* Hdn = h->Hdn.as<char>() + r0 * Fd * xsz;
        float* Td = h->Td.as<float>() + r0 * D;
        void* Tdn = h->Tdn.as<char>() + r0 * D * esz;
        void* Qd = h->Qd.as<char>() + r0 * D * esz;
        float* Od = (float*)(h->Od.as<char>() + r0 * D * (x3d ? 6 : 4));
        // a GEMM whose A operand a producer wrote as rows of xdm / hdm
        auto gemmA = [&](const void* A, bool wide, const void* Wt, int N, int Kk, const GemmEpi& e) -> hipError_t {
            if (x3d) return rg.gemm3(A, wide ? hdm : xdm, Wt, Kk, Mg, N, Kk, e);
            return rg.gemm(dt, A, rowmap_plain(Kk), Wt, Kk, Mg, N, Kk, e);
        };
        bf16* Odb = h->Odb.as<bf16>() + r0 * D;
        const int* ntg = ntok + b0;
        const int* lg = lens + b0;
        const char* KVg = (const char*)KV + (size_t)b0 * T * nkv * esz;
        // fast mode: each decoder FFN (+ its LN1 before, + the LN after) as one fused kernel (k_ffn.hip DEC)
        const bool dffn = fast && h->dffn_ready && pfm_knobs().dec_ffn_fused && Mg >= 2048;
        int op_from = -1;   // fused path: the decoder block whose out-projection runs inside the next FFN launch
        auto ffn = [&](int fi, size_t lng, size_t lnb, size_t w1, size_t b1, size_t fng, size_t fnb,
                       size_t w2, float* out, size_t pg, size_t pb, void* pout, int pdt) -> int {
            // out = W2 . LN_F(relu(W1 . LN(x) + b1)); pout = LN_P(out)   (sanm/positionwise_feed_forward.py:26-33)
            if (dffn && pdt == DT_BF16 && h->dffn_kind >= 2) {   // k_ffn2.hip: 128-row tiles (2: hidden split)
                const double flo = 4.0 * Mg * (double)D * Fd + (op_from >= 0 ? 2.0 * Mg * (double)D * D : 0.0);
                const double byo = (double)Mg * D * (4.0 + 2.0) + 2.0 * 2.0 * D * Fd;
                ProfScope ps(h, s, PFM_K_GEMM, flo, byo);
                const float* cc = h->dffn_c.as<float>() + (size_t)fi * 2 * D;
                const bf16* blk = h->dffn_pack.as<bf16>() + (size_t)fi * pfm_ffn2_dec_packed_elems();
                float* part = h->dffn_kind == 2 ? h->dffn2_part.as<float>() + (size_t)gi * part_n : nullptr;
                unsigned* cnt = h->dffn_kind == 2 ? h->dffn2_cnt.as<unsigned>() + (size_t)gi * cnt_n : nullptr;
                const bool opf = op_from >= 0;   // x = x + O Wo^T + bo of block op_from, then the FFN on it
                HIP_TRY(pfm_ffn2_fused_dec(Xd, Mg, P(lng), P(lnb), c.ln_eps, blk, P(b1), cc, cc + D, opf ? Xd : nullptr,
                                           P(pg), P(pb), (bf16*)pout, opf ? Odb : nullptr,
                                           opf ? P(h->dec[op_from].bo) : nullptr, part, cnt, s));
                op_from = -1;
                return PFM_OK;
            }
            if (dffn && pdt == DT_BF16) {   // out itself is dead in the decoder: only LN_P(out) is consumed
                const double flo = 4.0 * Mg * (double)D * Fd;
                const double byo = (double)Mg * D * (4.0 + 2.0) + 2.0 * 2.0 * D * Fd;
                ProfScope ps(h, s, PFM_K_GEMM, flo, byo);
                const float* cc = h->dffn_c.as<float>() + (size_t)fi * 2 * D;
                const size_t po = pfm_ffn_packed_o_elems();
                const bf16* blk = h->dffn_pack.as<bf16>() + (size_t)fi * (po + pfm_ffn_packed_elems());
                if (op_from >= 0) {   // x = x + O Wo^T + bo of block op_from, then the FFN on it
                    HIP_TRY(pfm_ffn_fused_dec(Xd, Mg, P(lng), P(lnb), c.ln_eps, blk, P(b1), cc, cc + D, Xd, P(pg), P(pb),
                                              (bf16*)pout, Odb, P(h->dec[op_from].bo), s));
                    op_from = -1;
                } else {
                    HIP_TRY(pfm_ffn_fused_dec(Xd, Mg, P(lng), P(lnb), c.ln_eps, blk + po, P(b1), cc, cc + D, nullptr, P(pg),
                                              P(pb), (bf16*)pout, nullptr, nullptr, s));
                }
                return PFM_OK;
            }
            HIP_TRY(pfm_layernorm(Xd, rowmap_plain(D), Mg, D, P(lng), P(lnb), c.ln_eps, nullptr, 0, 1.f, Xdn, xdm, ndt,
                                  nullptr, plain, 0, s));
            GemmEpi e = epi_default();
            e.bias = P(b1); e.relu = 1;
            e.out = Hd; e.out_map = rowmap_plain(Fd); e.out_dtype = fast ? DT_BF16 : DT_F32;   // fast: bf16 hidden
            HIP_TRY(gemmA(Xdn, false, W(w1), Fd, D, e));
            if (fast)
                HIP_TRY(pfm_layernorm_bf16in((const bf16*)Hd, rowmap_plain(Fd), Mg, Fd, P(fng), P(fnb), c.ln_eps, Hdn,
                                             rowmap_plain(Fd), dt, s));
            else
                HIP_TRY(pfm_layernorm((const float*)Hd, rowmap_plain(Fd), Mg, Fd, P(fng), P(fnb), c.ln_eps, nullptr, 0,
                                      1.f, Hdn, hdm, ndt, nullptr, plain, 0, s));
            GemmEpi e2 = epi_default();
            e2.out = out; e2.out_map = rowmap_plain(D); e2.out_dtype = DT_F32;
            HIP_TRY(gemmA(Hdn, true, W(w2), D, Fd, e2));
            HIP_TRY(pfm_layernorm(out, rowmap_plain(D), Mg, D, P(pg), P(pb), c.ln_eps, nullptr, 0, 1.f, pout,
                                  rowmap_plain(pdt == DT_X3 ? 3 * D : D), pdt, nullptr, plain, 0, s));
            return PFM_OK;
        };
        for (int l = 0; l < c.dec_blocks; ++l) {
            const DecLayer& Lr = h->dec[l];
            // t = FFN(LN1(x)); x = x + FSMN(LN2(t))   (decoder.py:97-107)
            // fast mode: LN2(t) in bf16 feeding the bf16-input FSMN (x += FSMN(LN2(t)) stays f32)
            int rc2 = ffn(l, Lr.n1g, Lr.n1b, Lr.w1, Lr.b1, Lr.ng, Lr.nb, Lr.w2, Td, Lr.n2g, Lr.n2b, Tdn,
                          fast ? DT_BF16 : DT_F32);
            if (rc2) return rc2;
            // x = x + CrossAtt(LN3(x), memory)   (decoder.py:109-119); fused path: LN3 in the FSMN kernel
            if (dffn && D == 512 && K == 11 && ldec == 5) {
                HIP_TRY(pfm_fsmn_ln_bf16in((const bf16*)Tdn, rowmap_plain(D), ntg, nb, L, D, P(Lr.fsmn), K, ldec, Xd, Xd,
                                           P(Lr.n3g), P(Lr.n3b), c.ln_eps, (bf16*)Xdn, s));
            } else {
                if (fast)
                    HIP_TRY(pfm_fsmn_bf16in((const bf16*)Tdn, rowmap_plain(D), ntg, nb, L, D, P(Lr.fsmn), K, ldec, Xd,
                                            Xd, nullptr, s));
                else
                    HIP_TRY(pfm_fsmn((const float*)Tdn, rowmap_plain(D), ntg, nb, L, D, P(Lr.fsmn), K, ldec, Xd, Xd,
                                     nullptr, s));
                HIP_TRY(pfm_layernorm(Xd, rowmap_plain(D), Mg, D, P(Lr.n3g), P(Lr.n3b), c.ln_eps, nullptr, 0, 1.f, Xdn,
                                      xdm, ndt, nullptr, plain, 0, s));
            }
            {
                GemmEpi e = epi_default();
                e.bias = P(Lr.bq);
                e.out = Qd; e.out_map = rowmap_plain(D); e.out_dtype = dt;
                HIP_TRY(gemmA(Xdn, false, W(Lr.wq), D, D, e));
            }
            if (kv_async && l % kv_lpg == 0 && l / kv_lpg < kv_groups)   // join the side stream (this layer group)
                HIP_TRY(hipStreamWaitEvent(s, kv_groups > 1 ? h->ev_kvg[l / kv_lpg] : h->ev_kv, 0));
            {
                const char* kvb = KVg + (size_t)l * 2 * D * esz;
                if (x3d)
                    HIP_TRY(rg.attn3((const float*)Qd, rowmap_plain(D), (const float*)kvb, rowmap_plain(nkv),
                                     (const float*)(kvb + (size_t)D * esz), rowmap_plain(nkv), (bf16*)Od, lg, nb, L, T));
                else
                    HIP_TRY(rg.attn(dt, Qd, rowmap_plain(D), kvb, rowmap_plain(nkv), kvb + (size_t)D * esz,
                                    rowmap_plain(nkv), fast ? nullptr : Od, D, fast ? (void*)Odb : nullptr, lg, nb, L, T));
            }
            {
                GemmEpi e = epi_default();
                e.bias = P(Lr.bo);
                e.res0 = Xd; e.ld_res0 = D;
                e.out = Xd; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
                if (dffn) {   // runs as phase 0 of the next FFN launch
                    op_from = l;
                } else {
                    HIP_TRY(gemmA(fast ? (const void*)Odb : (const void*)Od, false, W(Lr.wo), D, D, e));
                }
            }
        }
        // decoders3: x = FFN(LN1(x)), no residual (decoder.py:97-100 with self_attn = src_attn = None)
        int rc3 = ffn(c.dec_blocks, h->d3n1g, h->d3n1b, h->d3w1, h->d3b1, h->d3ng, h->d3nb, h->d3w2, Xd, h->dan_g,
                      h->dan_b, Xdn, ndt);
        if (rc3) return rc3;
        if (h->want_logits) {   // beam search (pfm_run_beam): the f32 logits [B][L][V] themselves
            GemmEpi e = epi_default();
            e.bias = P(h->out_b);
            e.out = h->logits.as<float>() + r0 * c.vocab_size; e.out_map = rowmap_plain(c.vocab_size);
            e.out_dtype = DT_F32;
            HIP_TRY(gemmA(Xdn, false, W(h->out_w), c.vocab_size, D, e));
        } else {   // output layer with fused row-argmax (logits never written)
            const int ntl = amax_tiles(dt, rowmap_plain(D), D, c.vocab_size, D, h, W(h->out_w));
            GemmEpi e = epi_default();
            e.bias = P(h->out_b);
            e.amax_val = h->amv.as<float>() + r0 * ntl; e.amax_idx = h->ami.as<int>() + r0 * ntl; e.n_tiles = ntl;
            e.out = nullptr;
            HIP_TRY(gemmA(Xdn, false, W(h->out_w), c.vocab_size, D, e));
        }
        return PFM_OK;
    };
    // the per-tile row maxima of every group -> token ids, one launch on the caller's stream after the join
    auto finish = [&]() -> int {
        if (L_cap > 0 && !h->want_logits) {
            const int ntl = amax_tiles(dt, rowmap_plain(D), D, c.vocab_size, D, h, W(h->out_w));
            HIP_TRY(pfm_argmax_reduce(h->amv.as<float>(), h->ami.as<int>(), ntl, (c.vocab_size + 63) / 64, B, L, ntok,
                                      L_cap, tokens, nullptr, st));
        }
        return PFM_OK;
    };
    // PFM_DEC_SUBBATCH=n: utterance groups on concurrent streams (default 2: with the fused decoder FFN kernels
    // the two groups overlap, 19.74 vs 19.90 ms/step in three interleaved rounds of tools/bench_ab.py; before
    // the FFN fusion they measured equal, 23.5-24.0 ms/step either way)
    const int ng = ngd;
    (void)Ml;
    if (ng == 1) {
        rc = dec_group(run, 0, B, 0);
        return rc ? rc : finish();
    }
    if (!h->ev_fork) HIP_TRY(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->ev_fork, st));
    for (int k = 0; k < ng; ++k) {
        if (!h->sub_st[k]) {
            HIP_TRY(hipStreamCreateWithFlags(&h->sub_st[k], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&h->ev_join[k], hipEventDisableTiming));
        }
        const int b0 = (int)((long long)B * k / ng), b1 = (int)((long long)B * (k + 1) / ng);
        if (b1 <= b0) continue;
        HIP_TRY(hipStreamWaitEvent(h->sub_st[k], h->ev_fork, 0));
        Run rk = run;
        rk.st = h->sub_st[k];
        rc = dec_group(rk, b0, b1 - b0, k);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(h->ev_join[k], h->sub_st[k]));
        HIP_TRY(hipStreamWaitEvent(st, h->ev_join[k], 0));
    }
    return finish();
}

int pfm_run_beam(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens, int B, int T,
                 int beam, float ctc_weight, float penalty, int nbest, int end_detect, int sos, int eos, int blank,
                 int32_t* tokens, int L_cap, int32_t* ntok_out, float* scores_out, float* alphas_out,
                 float* peaks_out) {
    pfm_knobs_refresh();
    if (!h || !feats || !lens || !tokens || !ntok_out || !scores_out) return fail(PFM_E_ARG, "pfm_run_beam: null argument");
    if (h->cfg.arch != PFM_ARCH_PARAFORMER || !h->cfg.ctc_head)
        return fail(PFM_E_STATE, "pfm_run_beam: needs a Paraformer handle with a CTC head (ctc_head = 1)");
    const int V = h->cfg.vocab_size;
    // BeamSearchPara(pre_beam_ratio 1.5, pre_beam_score_key "full"): pre-beam when int(1.5 beam) < V
    const int pre = (int)(1.5 * beam), P = pre < V ? pre : V;
    if (sos < 0 || sos >= V || eos < 0 || eos >= V || blank < 0 || blank >= V)
        return fail(PFM_E_ARG, "pfm_run_beam: sos / eos / blank outside the vocabulary");
    if (beam < 1 || beam > 16 || nbest < 1 || nbest > 16 || P > 64 || !(ctc_weight > 1e-5f) || L_cap < 0)
        return fail(PFM_E_ARG, "pfm_run_beam: need 1 <= beam <= 16, 1 <= nbest <= 16, ctc_weight > 1e-5, <= 64 candidates");
    CHECK_DEV("pfm_run_beam", h->device, {"feats", feats}, {"lens", lens}, {"tokens", tokens}, {"ntok", ntok_out},
              {"scores", scores_out}, {"alphas", alphas_out}, {"peaks", peaks_out});
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    int32_t* ntok_dev = nullptr;
    {   // encoder -> CIF -> decoder with the output layer writing f32 logits (pfm_run, want_logits)
        h->want_logits = true;
        h->last_L = 0;
        HIP_TRY(h->beam_is.ensure((size_t)B * sizeof(int32_t)));
        ntok_dev = h->beam_is.as<int32_t>();
        const int rc = pfm_run(h, stream, mode, feats, lens, B, T, ntok_dev, 0, ntok_dev, nullptr, alphas_out, peaks_out);
        h->want_logits = false;
        if (rc) return rc;
    }
    const int L = h->last_L;
    const int D = h->cfg.d_model;
    HIP_TRY(hipMemsetAsync(scores_out, 0, (size_t)B * nbest * sizeof(float), st));
    if (L < 1) {   // model.py:514-515: nothing decoded -> no hypotheses
        HIP_TRY(pfm_fill_i32(ntok_out, (long long)B * nbest, -1, st));
        return PFM_OK;
    }
    const bool fast = mode == PFM_MODE_FAST;
    const Run run(h, st, fast);
    // CTC log-probs of the encoder output (ctc.log_softmax, ctc/ctc.py:173-185): [B*T, V] f32
    const long long M = (long long)B * T;
    HIP_TRY(h->ctcx.ensure((size_t)M * V * sizeof(float)));
    {
        GemmEpi e = epi_default();
        e.bias = run.P(h->ctc_b);
        e.out = h->ctcx.p; e.out_map = rowmap_plain(V); e.out_dtype = DT_F32;
        const RowMap encmap = rowmap_seg(T, (long long)(T + 2) * D, D);
        const void* A = fast ? (const void*)(h->encpb.as<bf16>() + D) : (const void*)(h->encp.as<float>() + D);
        HIP_TRY(run.gemm(run.dt, A, encmap, run.W(h->ctc_w), D, (int)M, V, D, e));
    }
    HIP_TRY(pfm_logsoftmax_rows(h->ctcx.as<float>(), M, V, V, st));
    HIP_TRY(pfm_logsoftmax_rows(h->logits.as<float>(), (long long)B * L, V, V, st));   // decoder log_softmax
    // the search (ntok of the run: the device token counts behind pfm_run's ntok_out)
    const long long fsz = pfm_ctc_beam_fscratch(beam, P, T, L, V), isz = pfm_ctc_beam_iscratch(beam, nbest, L, P, V);
    // the device token counts (first B ints of beam_is) move behind the float scratch before beam_is is resized
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(h->beam_fs.ensure(((size_t)B * fsz + B) * sizeof(float)));
    int* ntk = (int*)(h->beam_fs.as<float>() + (size_t)B * fsz);
    HIP_TRY(hipMemcpyAsync(ntk, ntok_dev, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(h->beam_is.ensure((size_t)B * isz * sizeof(int32_t)));
    HIP_TRY(h->beam_fail.ensure(sizeof(unsigned)));
    HIP_TRY(pfm_ctc_beam(h->logits.as<float>(), L, h->ctcx.as<float>(), T, lens, ntk, B, V, beam, P, nbest,
                         ctc_weight, penalty, penalty != 0.f ? 1 : 0, end_detect, sos, eos, blank,
                         h->beam_fs.as<float>(), h->beam_is.as<int>(), tokens, L_cap, ntok_out, scores_out,
                         h->beam_fail.as<unsigned>(), st));
    HIP_TRY(hipStreamSynchronize(st));
    return beam_failed(h->beam_fail.as<unsigned>(), "pfm_run_beam");
}

int pfm_run_ctc(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens, int B, int T,
                const int32_t* query, int ban_token, int32_t* tokens, int L_cap, int32_t* ntok_out, float* enc_out,
                int32_t* frame_ids) {
    pfm_knobs_refresh();
    if (!h || !feats || !lens || !query || !tokens || !ntok_out) return fail(PFM_E_ARG, "pfm_run_ctc: null argument");
    if (B < 1 || T < 1 || L_cap < 0) return fail(PFM_E_ARG, "pfm_run_ctc: bad sizes");
    if (mode != PFM_MODE_EXACT && mode != PFM_MODE_FAST) return fail(PFM_E_ARG, "pfm_run_ctc: bad mode");
    if (h->cfg.arch != PFM_ARCH_SENSEVOICE) return fail(PFM_E_STATE, "pfm_run_ctc: handle is not a SenseVoice model");
    if (h->missing) return fail(PFM_E_STATE, "pfm_run_ctc: " + std::to_string(h->missing) + " weights not set");
    const pfm_config& c = h->cfg;
    constexpr int NQ = 4;   // [language, event, emotion, textnorm] (sense_voice/model.py:851-876)
    for (int i = 0; i < NQ; ++i)
        if (query[i] < 0 || query[i] >= c.n_embed) return fail(PFM_E_ARG, "pfm_run_ctc: query id out of range");
    if (ban_token >= c.vocab_size) return fail(PFM_E_ARG, "pfm_run_ctc: ban_token out of range");
    CHECK_DEV("pfm_run_ctc", h->device, {"feats", feats}, {"lens", lens}, {"tokens", tokens}, {"ntok", ntok_out},
              {"enc_out", enc_out}, {"frame_ids", frame_ids});
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    const int Tq = T + NQ;
    int rc = reserve(h, B, Tq);
    if (rc) return rc;
    const bool fast = mode == PFM_MODE_FAST;
    if (fast) { rc = ensure_bf16(h, st); if (rc) return rc; }
    else { rc = ensure_x6(h, st); if (rc) return rc; }
    if (h->prof_on && h->ev_used > 4096) prof_collect(h);
    const Run run(h, st, fast);
    const int D = c.d_model, I = c.input_size, V = c.vocab_size;
    const long long M = (long long)B * Tq;
    int* olen = h->olen.as<int>();
    // x = [embed(query) ; feats], lens + 4 (model.py:851-876)
    HIP_TRY(pfm_sv_input(feats, lens, h->w(h->embed), query, NQ, B, T, I, h->Xin.as<float>(), olen, st));
    // encoder: 50 SAN-M layers -> after_norm (f32, feeds the tp stack) -> 20 tp layers -> tp_norm
    // (SenseVoiceEncoderSmall.forward, model.py:553-585)
    {
        const FinalLN fin = {h->an_g, h->an_b, h->X2.p, rowmap_plain(D), DT_F32, nullptr, rowmap_plain(0), 0};
        rc = encoder_split(h, run, h->Xin.as<float>(), olen, B, Tq, 0, c.enc_blocks, h->X.as<float>(), fin);
        if (rc) return rc;
    }
    {
        const FinalLN fin = {h->tp_g, h->tp_b, h->Xf.p, rowmap_plain(D), run.dt, enc_out, rowmap_plain(D), DT_F32};
        rc = encoder_split(h, run, nullptr, olen, B, Tq, c.enc_blocks, c.enc_blocks + c.tp_blocks, h->X2.as<float>(),
                           fin);
        if (rc) return rc;
    }
    // CTC head (ctc.py:173-184) with fused row-argmax; ban_emo_unk (model.py:885-886) sets the banned
    // token's log-prob to -inf: a -inf bias entry excludes it from the argmax the same way
    const float* bias = run.P(h->ctc_b);
    if (ban_token >= 0) {
        if (h->ban_tok != ban_token || !h->ban_bias.p) {
            HIP_TRY(h->ban_bias.ensure((size_t)V * 4));
            HIP_TRY(hipMemcpyAsync(h->ban_bias.p, bias, (size_t)V * 4, hipMemcpyDeviceToDevice, st));
            const float ninf = -INFINITY;
            HIP_TRY(hipMemcpyAsync(h->ban_bias.as<float>() + ban_token, &ninf, 4, hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));   // the host source of the -inf entry is a stack value
            h->ban_tok = ban_token;
        }
        bias = h->ban_bias.as<float>();
    }
    const int ntl = amax_tiles(run.dt, rowmap_plain(D), D, V, D, h, run.W(h->ctc_w));
    {
        GemmEpi e = epi_default();
        e.bias = bias;
        e.amax_val = h->amv.as<float>(); e.amax_idx = h->ami.as<int>(); e.n_tiles = ntl;
        e.out = nullptr;
        HIP_TRY(run.gemm(run.dt, h->Xf.p, rowmap_plain(D), run.W(h->ctc_w), D, (int)M, V, D, e));
    }
    int* fid = frame_ids ? frame_ids : h->fids.as<int>();
    HIP_TRY(pfm_argmax_reduce(h->amv.as<float>(), h->ami.as<int>(), ntl, (V + 63) / 64, B, Tq, olen, Tq, fid, nullptr,
                              st));
    // unique_consecutive + drop blank (model.py:894-906)
    HIP_TRY(pfm_ctc_collapse(fid, Tq, olen, B, 0, L_cap, tokens, ntok_out, st));
    return PFM_OK;
}

// Run `body` on `st`, through a HIP graph of its launches when `use`: the first call of a shape runs eagerly
// (one-time launcher setup happens there), the second captures and every later one replays. A graph is rebuilt
// when the owner's workspace generation `gen()` moved since its capture; graphs are keyed by the calling
// thread's knob snapshot as well. `st` must not be the legacy null stream (it cannot be captured).
extern "C++" {
template <class G, class F>
int graphed(GraphCache& gc, const char* tag, std::array<int, 4> shape, bool use, hipStream_t st, G&& gen_of,
            F&& body) {
    if (!use) return body(st);
    const std::array<unsigned long long, 5> key = {(unsigned long long)shape[0], (unsigned long long)shape[1],
                                                   (unsigned long long)shape[2], (unsigned long long)shape[3],
                                                   pfm_knobs().sig};
    if (!gc.graphs.count(key) && gc.graphs.size() >= GraphCache::MAX) {   // evict the LRU entry
        auto lru = gc.graphs.begin();
        for (auto it = gc.graphs.begin(); it != gc.graphs.end(); ++it)
            if (it->second.last_use < lru->second.last_use) lru = it;
        if (lru->second.exec) (void)hipGraphExecDestroy(lru->second.exec);
        gc.graphs.erase(lru);
    }
    auto& g = gc.graphs[key];
    g.last_use = ++gc.use_clock;
    const unsigned long long gen = gen_of();
    static const bool log = getenv("PFM_STREAM_GRAPH_LOG") != nullptr;
    if (log)
        fprintf(stderr, "[%s graph] key %d/%d/%d/%d %s gen %llu/%llu seen %d (%zu graphs)\n", tag, shape[0], shape[1],
                shape[2], shape[3], g.exec && g.gen == gen ? "replay" : (g.bad || g.seen == 0 ? "eager" : "capture"),
                g.gen, gen, g.seen, gc.graphs.size());
    if (g.exec && g.gen == gen) {
        HIP_TRY(hipGraphLaunch(g.exec, st));
        return PFM_OK;
    }
    if (g.exec) { (void)hipGraphExecDestroy(g.exec); g.exec = nullptr; }
    if (g.bad || g.seen++ == 0) return body(st);
    HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    const int rc = body(st);
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(st, &graph);
    if (rc != PFM_OK || e != hipSuccess || gen_of() != gen) {   // run this call eagerly instead
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
        if (rc != PFM_OK) return rc;
        g.bad = e != hipSuccess;   // not capturable: this shape stays eager
        return body(st);
    }
    const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) {
        g.exec = nullptr;
        g.bad = true;
        (void)hipGetLastError();
        return body(st);
    }
    g.gen = gen;
    HIP_TRY(hipGraphLaunch(g.exec, st));
    return PFM_OK;
}
}  // extern "C++"

// CTTransformer.punc_forward's model (ct_transformer/model.py:70-79 forward): embedding * sqrt(d) + PE, the
// SAN-M blocks, after_norm, the punctuation head and its argmax; workspace reserved and weights converted already
static int punc_body(pfm_handle* h, hipStream_t st, bool fast, const int32_t* ids, const int32_t* lens, int B, int T,
                     int32_t* punc, float* logits) {
    const pfm_config& c = h->cfg;
    const int D = c.d_model;
    float* X = h->X.as<float>();
    // X = embed[ids] * sqrt(d) + PE: the encoder input AND layer 0's residual (input_size == d_model)
    HIP_TRY(pfm_punc_embed(ids, lens, B, T, h->w(h->embed), c.n_embed, h->pe.as<float>(), D, sqrtf((float)D), X, st));
    Run run(h, st, fast);
    run.fuse_fsmn = false;   // 32-wide heads: the fused FSMN epilogue lives in the d_k = 128 kernel
    run.raw_input = true;
    const FinalLN fin = {h->an_g, h->an_b, h->Xf.as<float>(), rowmap_plain(D), DT_F32, nullptr, rowmap_plain(D),
                         DT_BF16};
    const int rc = encoder_stack(run, X, lens, B, T, 0, c.enc_blocks, X, fin, enc_ws(h, 0));
    if (rc) return rc;
    HIP_TRY(pfm_punc_head(h->Xf.as<float>(), B, T, lens, h->w(h->ctc_w), h->w(h->ctc_b), c.vocab_size, D, punc,
                          logits, st));
    return PFM_OK;
}

static int punc_prepare(pfm_handle* h, hipStream_t st, bool fast, int B, int T) {
    int rc = reserve(h, B, T);
    if (rc) return rc;
    return fast ? ensure_bf16(h, st) : ensure_x6(h, st);
}

int pfm_run_punc(pfm_handle* h, void* stream, int mode, const int32_t* ids, const int32_t* lens, int B, int T,
                 int32_t* punc, float* logits) {
    pfm_knobs_refresh();
    if (!h || !ids || !lens || !punc) return fail(PFM_E_ARG, "pfm_run_punc: null argument");
    if (h->cfg.arch != PFM_ARCH_PUNC) return fail(PFM_E_STATE, "pfm_run_punc: handle is not a punctuation model");
    if (B < 1 || T < 1) return fail(PFM_E_ARG, "pfm_run_punc: bad sizes");
    if (mode != PFM_MODE_EXACT && mode != PFM_MODE_FAST) return fail(PFM_E_ARG, "pfm_run_punc: bad mode");
    if (h->missing) return fail(PFM_E_STATE, "pfm_run_punc: weights not set");
    CHECK_DEV("pfm_run_punc", h->device, {"ids", ids}, {"lens", lens}, {"punc", punc}, {"logits", logits});
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    const bool fast = mode == PFM_MODE_FAST;
    const int rc = punc_prepare(h, st, fast, B, T);
    if (rc) return rc;
    return punc_body(h, st, fast, ids, lens, B, T, punc, logits);
}

// One mini-sentence of the CT-Transformer text loop with host word ids in and host labels out (the per-call form
// CTTransformer.punc_forward is used in, model.py:277-316): one pinned staging copy each way around the model on
// the handle's own device buffers, so a caller's sequential loop costs one C call per sentence. The model's ~35
// launches run on the handle's own stream, ordered after the caller's queued work by one event; the call returns
// with that stream drained. Fast mode (PFM_PUNC_GRAPH, default 1): the sentence is padded to a multiple of 16 words and
// the launches replay from a HIP graph per padded length from its second call on (192 vs 207 us per 30-word call,
// 287 vs 295 at 200: the kernels' own latency dominates; labels identical to the unpadded call, tests/test_gpu_punc.py).
int pfm_run_punc_host(pfm_handle* h, void* stream, int mode, const int32_t* ids, int n, int32_t* punc) {
    pfm_knobs_refresh();
    if (!h || !ids || !punc || n < 1) return fail(PFM_E_ARG, "pfm_run_punc_host: null argument or n < 1");
    if (h->cfg.arch != PFM_ARCH_PUNC) return fail(PFM_E_STATE, "pfm_run_punc_host: handle is not a punctuation model");
    if (mode != PFM_MODE_EXACT && mode != PFM_MODE_FAST) return fail(PFM_E_ARG, "pfm_run_punc_host: bad mode");
    if (h->missing) return fail(PFM_E_STATE, "pfm_run_punc_host: weights not set");
    HIP_TRY(hipSetDevice(h->device));
    if (!h->punc_st) {
        HIP_TRY(hipStreamCreateWithFlags(&h->punc_st, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&h->punc_ev, hipEventDisableTiming));
    }
    HIP_TRY(hipEventRecord(h->punc_ev, (hipStream_t)stream));
    HIP_TRY(hipStreamWaitEvent(h->punc_st, h->punc_ev, 0));
    hipStream_t st = h->punc_st;
    const bool fast = mode == PFM_MODE_FAST;
    const bool use = fast && pfm_knobs().punc_graph && !h->prof_on;
    // with graphs (fast mode) the sentence is padded to a multiple of 16 words: every kernel of the chain reads the
    // length from the device (masked keys / FSMN rows, -1 labels beyond it) and computes each row alone, so the labels
    // are the unpadded call's, and the <= 16 padded shapes of a text loop replay from a handful of graphs
    const int Tp = use ? (n + 15) / 16 * 16 : n;
    if (h->punc_cap < Tp) {
        const int cap = std::max(Tp, 256);
        if (h->punc_pin) { HIP_TRY(hipStreamSynchronize(st)); HIP_TRY(hipHostFree(h->punc_pin)); h->punc_pin = nullptr; }
        HIP_TRY(hipHostMalloc((void**)&h->punc_pin, (size_t)(2 * cap + 1) * sizeof(int32_t), 0));
        HIP_TRY(h->punc_io.ensure((size_t)(2 * cap + 1) * sizeof(int32_t)));
        h->punc_cap = cap;
    }
    int rc = punc_prepare(h, st, fast, 1, Tp);
    if (rc) return rc;
    int32_t* pin = h->punc_pin;
    memcpy(pin, ids, (size_t)n * sizeof(int32_t));
    for (int i = n; i < Tp; ++i) pin[i] = 0;
    pin[Tp] = n;
    int32_t* dio = h->punc_io.as<int32_t>();
    HIP_TRY(hipMemcpyAsync(dio, pin, (size_t)(Tp + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
    rc = graphed(h->punc_graphs, "punc", {mode, Tp, 0, 0}, use, st, [h] { return h->buf_gen.load(); },
                 [&](hipStream_t s) { return punc_body(h, s, fast, dio, dio + Tp, 1, Tp, dio + Tp + 1, nullptr); });
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(pin + Tp + 1, dio + Tp + 1, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(punc, pin + Tp + 1, (size_t)n * sizeof(int32_t));
    return PFM_OK;
}

static int fbank_tables_build(DevBuf& dst) {
    std::vector<unsigned char> tab(pfm_fbank_table_bytes(), 0);
    float* melw = (float*)tab.data();
    int* lo = (int*)(tab.data() + 80 * 256 * 4);
    int* hi = lo + 80;
    float* window = (float*)(hi + 80);
    double* tw = (double*)(tab.data() + pfm_fbank_twoff());
    pfm_fbank_tables(melw, lo, hi, window, tw);
    HIP_TRY(dst.ensure(tab.size()));
    HIP_TRY(hipMemcpy(dst.p, tab.data(), tab.size(), hipMemcpyHostToDevice));
    return PFM_OK;
}

static int fbank_tables_ready(pfm_handle* h) {
    if (h->fb_tab_ready) return PFM_OK;
    std::vector<unsigned char> tab(pfm_fbank_table_bytes(), 0);
    float* melw = (float*)tab.data();
    int* lo = (int*)(tab.data() + 80 * 256 * 4);
    int* hi = lo + 80;
    float* window = (float*)(hi + 80);
    double* tw = (double*)(tab.data() + pfm_fbank_twoff());
    pfm_fbank_tables(melw, lo, hi, window, tw);
    HIP_TRY(h->fb_tab.ensure(tab.size()));
    HIP_TRY(hipMemcpy(h->fb_tab.p, tab.data(), tab.size(), hipMemcpyHostToDevice));
    h->fb_tab_ready = true;
    return PFM_OK;
}

int pfm_fbank_raw(pfm_handle* h, void* stream, const float* wav, const int32_t* nsamp, int B, int S_max, float* fb,
                  int N_cap) {
    if (!h || !wav || !nsamp || !fb) return fail(PFM_E_ARG, "pfm_fbank_raw: null argument");
    if (B < 1 || S_max < 1 || N_cap < 1) return fail(PFM_E_ARG, "pfm_fbank_raw: bad sizes");
    if (pfm_fbank_nframes(S_max) > N_cap) return fail(PFM_E_ARG, "pfm_fbank_raw: N_cap smaller than frames of S_max");
    CHECK_DEV("pfm_fbank_raw", h->device, {"wav", wav}, {"nsamp", nsamp}, {"fb", fb});
    HIP_TRY(hipSetDevice(h->device));
    int rc = fbank_tables_ready(h);
    if (rc) return rc;
    HIP_TRY(pfm_fbank_raw_launch(wav, nsamp, B, S_max, h->fb_tab.as<unsigned char>(), fb, N_cap, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_lfr_gather(void* stream, const float* frames, const int32_t* idx, int rows, int m, const float* cmvn,
                   float* out) {
    if (rows < 0 || m < 1 || (m * 80) % 4) return fail(PFM_E_ARG, "pfm_lfr_gather: bad sizes");
    if (rows > 0 && (!frames || !idx || !out)) return fail(PFM_E_ARG, "pfm_lfr_gather: null argument");
    if (rows > 0) CHECK_DEV("pfm_lfr_gather", -1, {"frames", frames}, {"idx", idx}, {"cmvn", cmvn}, {"out", out});
    HIP_TRY(pfm_lfr_gather_launch(frames, idx, rows, m, cmvn, out, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_fbank(pfm_handle* h, void* stream, const float* wav, const int32_t* nsamp, int B, int S_max,
              const float* cmvn, float* feats, int T_cap, int32_t* T_out) {
    pfm_knobs_refresh();
    if (!h || !wav || !nsamp || !feats || !T_out) return fail(PFM_E_ARG, "pfm_fbank: null argument");
    if (B < 1 || S_max < 1 || T_cap < 1) return fail(PFM_E_ARG, "pfm_fbank: bad sizes");
    if (pfm_fbank_frames(S_max) > T_cap) return fail(PFM_E_ARG, "pfm_fbank: T_cap smaller than LFR frames of S_max");
    CHECK_DEV("pfm_fbank", h->device, {"wav", wav}, {"nsamp", nsamp}, {"cmvn", cmvn}, {"feats", feats}, {"T_out", T_out});
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    int rc = fbank_tables_ready(h);
    if (rc) return rc;

    const int N_cap = std::max(1, pfm_fbank_nframes(S_max));
    HIP_TRY(h->fb_ws.ensure((size_t)B * N_cap * 80 * 4));
    HIP_TRY(pfm_fbank_launch(wav, nsamp, B, S_max, cmvn, h->fb_tab.as<unsigned char>(), h->fb_ws.as<float>(), N_cap,
                             feats, T_cap, T_out, st));
    return PFM_OK;
}

int pfm_profile(pfm_handle* h, int enable) {
    if (!h) return fail(PFM_E_ARG, "pfm_profile: null handle");
    prof_collect(h);
    for (int k = 0; k < 4; ++k) { h->prof_ms[k] = h->prof_fl[k] = h->prof_by[k] = 0; h->prof_n[k] = 0; }
    h->prof_on = enable != 0;
    return PFM_OK;
}

int pfm_profile_read(pfm_handle* h, int kc, double* ms, double* flops, double* bytes, int64_t* launches) {
    if (!h || kc < 0 || kc > 3) return fail(PFM_E_ARG, "pfm_profile_read: bad arguments");
    prof_collect(h);
    if (ms) *ms = h->prof_ms[kc];
    if (flops) *flops = h->prof_fl[kc];
    if (bytes) *bytes = h->prof_by[kc];
    if (launches) *launches = h->prof_n[kc];
    return PFM_OK;
}

// ---------------- single-op entry points ----------------
int pfm_op_gemm(void* stream, int dtype, const void* A, const void* Wt, const float* bias, const float* res, float* C,
                int M, int N, int K, int act) {
    pfm_knobs_refresh();
    if (!A || !Wt || !C) return fail(PFM_E_ARG, "pfm_op_gemm: null operand");
    if (M < 0 || N < 1 || K < 1) return fail(PFM_E_ARG, "pfm_op_gemm: bad sizes");
    if (dtype != DT_F32 && dtype != DT_BF16) return fail(PFM_E_ARG, "pfm_op_gemm: dtype must be PFM_F32 or PFM_BF16");
    if ((act & 2) && dtype != DT_BF16) return fail(PFM_E_ARG, "pfm_op_gemm: bf16 output needs bf16 operands");
    CHECK_DEV("pfm_op_gemm", -1, {"A", A}, {"W", Wt}, {"bias", bias}, {"res", res}, {"C", C});
    GemmEpi e = epi_default();
    e.bias = bias; e.relu = act & 1;
    if (res) { e.res0 = res; e.ld_res0 = N; }
    e.out = C; e.out_map = rowmap_plain(N); e.out_dtype = (act & 2) ? DT_BF16 : DT_F32;
    if (act & 4) {   // split weights: Wt = two bf16 planes [2][N][K] (fast mode's PFM_FAST_XW projections)
        if (dtype != DT_BF16 || K % 64) return fail(PFM_E_ARG, "pfm_op_gemm: split weights need bf16 and K % 64 == 0");
        e.x6_k = K; e.x6_ws = (long long)N * K; e.x6_terms = 2;
        HIP_TRY(pfm_gemm_bf16_256(A, rowmap_plain(K), Wt, K, M, N, 2 * K, e, (hipStream_t)stream));
        return PFM_OK;
    }
    HIP_TRY(gemm_dispatch(dtype, A, rowmap_plain(K), Wt, K, M, N, K, e, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_ln_gemm(void* stream, const float* X, const float* g, const float* b, float eps, const void* W,
                   const float* bias, const float* res, float* C, int M, int N, int act) {
    pfm_knobs_refresh();
    if (!X || !g || !b || !W || !C || M < 0 || N < 0) return fail(PFM_E_ARG, "pfm_op_ln_gemm: null operand or bad sizes");
    CHECK_DEV("pfm_op_ln_gemm", -1, {"X", X}, {"g", g}, {"b", b}, {"W", W}, {"bias", bias}, {"res", res}, {"C", C});
    const hipStream_t st = (hipStream_t)stream;
    GemmEpi e = epi_default();
    e.bias = bias; e.relu = act & 1;
    if (res) { e.res0 = res; e.ld_res0 = N; }
    e.out = C; e.out_map = rowmap_plain(N); e.out_dtype = (act & 2) ? DT_BF16 : DT_F32;
    constexpr int K = 512;
    if (pfm_gemm_skinny_ln_ok(X, rowmap_plain(K), W, K, M, N, K, e)) {
        HIP_TRY(pfm_gemm_skinny_ln(X, rowmap_plain(K), g, b, eps, W, K, M, N, e, st));
        return PFM_OK;
    }
    bf16* xn = nullptr;
    HIP_TRY(hipMallocAsync((void**)&xn, (size_t)std::max(M, 1) * K * sizeof(bf16), st));
    hipError_t er = pfm_layernorm(X, rowmap_plain(K), M, K, g, b, eps, nullptr, 0, 1.f, xn, rowmap_plain(K), DT_BF16,
                                  nullptr, rowmap_plain(0), 0, st);
    if (er == hipSuccess) er = gemm_dispatch(DT_BF16, xn, rowmap_plain(K), W, K, M, N, K, e, st);
    (void)hipFreeAsync(xn, st);
    HIP_TRY(er);
    return PFM_OK;
}

}  // extern "C"

// scratch device buffers of one single-op call, freed on every return path
struct OpScratch {
    std::vector<void*> ptrs;
    OpScratch() = default;
    OpScratch(const OpScratch&) = delete;
    OpScratch& operator=(const OpScratch&) = delete;
    ~OpScratch() { for (void* p : ptrs) (void)hipFree(p); }
    template <typename T> hipError_t alloc(T** p, size_t n) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T));
        if (e == hipSuccess) { ptrs.push_back(q); *p = (T*)q; }
        return e;
    }
};

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool all_aligned16(std::initializer_list<const void*> ps) {
    for (const void* p : ps) if (!aligned16(p)) return false;
    return true;
}

extern "C" {

int pfm_op_ffn(void* stream, const float* x, int M, const float* g2, const float* b2n, float eps, const float* W1,
               const float* b1, const float* W2, const float* b2, float* xo, const float* gn, const float* bn,
               void* xn) {
    pfm_knobs_refresh();
    if (!x || !xo || !W1 || !W2 || !g2 || !b2n || !b1 || !b2 || M < 0) return fail(PFM_E_ARG, "pfm_op_ffn: null operand");
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr)) return fail(PFM_E_ARG, "pfm_op_ffn: xn needs gn and bn");
    if (!all_aligned16({x, xo, g2, b2n, b1, b2, xn, gn, bn})) return fail(PFM_E_ARG, "pfm_op_ffn: operands must be 16-B aligned");
    CHECK_DEV("pfm_op_ffn", -1, {"x", x}, {"g2", g2}, {"b2n", b2n}, {"W1", W1}, {"b1", b1}, {"W2", W2}, {"b2", b2},
              {"xo", xo}, {"gn", gn}, {"bn", bn}, {"xn", xn});
    const hipStream_t st = (hipStream_t)stream;
    const size_t nw = (size_t)2048 * 512;
    OpScratch sc;
    bf16 *w1b, *w2b, *wp;
    HIP_TRY(sc.alloc(&w1b, nw));
    HIP_TRY(sc.alloc(&w2b, nw));
    HIP_TRY(sc.alloc(&wp, pfm_ffn_packed_elems()));
    HIP_TRY(pfm_f32_to_bf16(W1, w1b, (long long)nw, st));
    HIP_TRY(pfm_f32_to_bf16(W2, w2b, (long long)nw, st));
    const bool k2 = pfm_knobs().ffn_kernel == 2;
    HIP_TRY((k2 ? pfm_ffn2_pack : pfm_ffn_pack)(w1b, w2b, wp, st));
    HIP_TRY((k2 ? pfm_ffn2_fused : pfm_ffn_fused)(x, M, g2, b2n, eps, wp, b1, b2, xo, gn, bn, (bf16*)xn, st));
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

int pfm_op_ffn_op(void* stream, const void* o, const void* f, const float* Wo, const float* bo, const float* x, int M,
                  const float* g2, const float* b2n, float eps, const float* W1, const float* b1, const float* W2,
                  const float* b2, float* xo, const float* gn, const float* bn, void* xn) {
    pfm_knobs_refresh();
    if (!o || !f || !Wo || !bo || !xo || !W1 || !W2 || !g2 || !b2n || !b1 || !b2 || M < 0)
        return fail(PFM_E_ARG, "pfm_op_ffn_op: null operand");
    if ((xn != nullptr) != (gn != nullptr && bn != nullptr)) return fail(PFM_E_ARG, "pfm_op_ffn_op: xn needs gn and bn");
    if (!all_aligned16({o, f, bo, x, xo, g2, b2n, b1, b2, xn, gn, bn}))
        return fail(PFM_E_ARG, "pfm_op_ffn_op: operands must be 16-B aligned");
    CHECK_DEV("pfm_op_ffn_op", -1, {"o", o}, {"f", f}, {"Wo", Wo}, {"bo", bo}, {"x", x}, {"g2", g2}, {"b2n", b2n},
              {"W1", W1}, {"b1", b1}, {"W2", W2}, {"b2", b2}, {"xo", xo}, {"gn", gn}, {"bn", bn}, {"xn", xn});
    const hipStream_t st = (hipStream_t)stream;
    const size_t nw = (size_t)2048 * 512, no = (size_t)512 * 512, po = pfm_ffn_packed_o_elems();
    OpScratch sc;
    bf16 *w1b, *w2b, *wob, *wp;
    HIP_TRY(sc.alloc(&w1b, nw));
    HIP_TRY(sc.alloc(&w2b, nw));
    HIP_TRY(sc.alloc(&wob, no));
    HIP_TRY(sc.alloc(&wp, po + pfm_ffn_packed_elems()));
    HIP_TRY(pfm_f32_to_bf16(W1, w1b, (long long)nw, st));
    HIP_TRY(pfm_f32_to_bf16(W2, w2b, (long long)nw, st));
    HIP_TRY(pfm_f32_to_bf16(Wo, wob, (long long)no, st));
    const bool k2 = pfm_knobs().ffn_kernel == 2;
    HIP_TRY((k2 ? pfm_ffn2_pack_o : pfm_ffn_pack_o)(wob, wp, st));
    HIP_TRY((k2 ? pfm_ffn2_pack : pfm_ffn_pack)(w1b, w2b, wp + po, st));
    HIP_TRY((k2 ? pfm_ffn2_fused_op : pfm_ffn_fused_op)((const bf16*)o, (const bf16*)f, bo, x, M, g2, b2n, eps, wp, b1, b2, xo, gn, bn, (bf16*)xn,
                             st));
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

int pfm_op_ffn_op_qkv(void* stream, const void* o, const void* f, const float* Wo, const float* bo, const float* x, int M,
                      const float* g2, const float* b2n, float eps, const float* W1, const float* b1, const float* W2,
                      const float* b2, float* xo, const float* gn, const float* bn, const float* Wq, const float* bq,
                      void* qkv) {
    pfm_knobs_refresh();
    if (!o || !f || !Wo || !bo || !xo || !W1 || !W2 || !g2 || !b2n || !b1 || !b2 || !gn || !bn || !Wq || !bq || !qkv ||
        M < 0)
        return fail(PFM_E_ARG, "pfm_op_ffn_op_qkv: null operand");
    if (!all_aligned16({o, f, bo, x, xo, g2, b2n, b1, b2, gn, bn, bq, qkv}))
        return fail(PFM_E_ARG, "pfm_op_ffn_op_qkv: operands must be 16-B aligned");
    CHECK_DEV("pfm_op_ffn_op_qkv", -1, {"o", o}, {"f", f}, {"Wo", Wo}, {"bo", bo}, {"x", x}, {"g2", g2}, {"b2n", b2n},
              {"W1", W1}, {"b1", b1}, {"W2", W2}, {"b2", b2}, {"xo", xo}, {"gn", gn}, {"bn", bn}, {"Wq", Wq}, {"bq", bq},
              {"qkv", qkv});
    const hipStream_t st = (hipStream_t)stream;
    const size_t nw = (size_t)2048 * 512, no = (size_t)512 * 512, po = pfm_ffn_packed_o_elems(),
                 pfe = pfm_ffn_packed_elems();
    OpScratch sc;
    bf16 *w1b, *w2b, *wob, *wqb, *wp;
    HIP_TRY(sc.alloc(&w1b, nw));
    HIP_TRY(sc.alloc(&w2b, nw));
    HIP_TRY(sc.alloc(&wob, no));
    HIP_TRY(sc.alloc(&wqb, 3 * no));
    // PFM_FAST_XW: bit 4 = MODE 5 (the v rows of Wq as two bf16 planes), bit 8 = MODE 6 (Wo too)
    const bool xv = (pfm_knobs().fast_xw & 4) != 0, xop = (pfm_knobs().fast_xw & 8) != 0;
    const size_t pw = (xop ? 2 : 1) * po;
    HIP_TRY(sc.alloc(&wp, pw + pfe + (xv ? 4 : 3) * po));
    HIP_TRY(pfm_f32_to_bf16(W1, w1b, (long long)nw, st));
    HIP_TRY(pfm_f32_to_bf16(W2, w2b, (long long)nw, st));
    HIP_TRY(pfm_f32_to_bf16(Wo, wob, (long long)no, st));
    HIP_TRY(pfm_f32_to_bf16(Wq, wqb, (long long)(3 * no), st));
    HIP_TRY(pfm_ffn2_pack_o(wob, wp, st));
    bf16* pl;
    HIP_TRY(sc.alloc(&pl, 9 * no));
    if (xop) {
        HIP_TRY(pfm_split3_planes(Wo, pl, (long long)no, (long long)no, st));
        HIP_TRY(pfm_ffn2_pack_o(pl + no, wp + po, st));
    }
    HIP_TRY(pfm_ffn2_pack(w1b, w2b, wp + pw, st));
    HIP_TRY(pfm_ffn2_pack_qkv(wqb, wp + pw + pfe, st));
    if (xv) {
        HIP_TRY(pfm_split3_planes(Wq, pl, (long long)(3 * no), (long long)(3 * no), st));
        HIP_TRY(pfm_ffn2_pack_qkv_v(pl + 3 * no, wp + pw + pfe + 3 * po, st));
        HIP_TRY(pfm_ffn2_fused_op_qkv_xv((const bf16*)o, (const bf16*)f, bo, x, M, g2, b2n, eps, wp, b1, b2, xo, gn, bn,
                                         bq, (bf16*)qkv, xop, st));
    } else {
        HIP_TRY(pfm_ffn2_fused_op_qkv((const bf16*)o, (const bf16*)f, bo, x, M, g2, b2n, eps, wp, b1, b2, xo, gn, bn, bq,
                                      (bf16*)qkv, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

int pfm_op_ffn_dec(void* stream, const float* x, int M, const float* g1, const float* b1n, float eps, const float* W1,
                   const float* b1, const float* W2, const float* gF, const float* bF, float* xo, const float* gn,
                   const float* bn, void* xn, const void* o, const float* Wo, const float* bo) {
    pfm_knobs_refresh();
    if (!x || !W1 || !W2 || !g1 || !b1n || !b1 || !gF || !bF || !gn || !bn || !xn || M < 0)
        return fail(PFM_E_ARG, "pfm_op_ffn_dec: null operand");
    if (o && (!Wo || !bo || !xo)) return fail(PFM_E_ARG, "pfm_op_ffn_dec: o needs Wo, bo and xo");
    if (!all_aligned16({x, g1, b1n, b1, gF, bF, xo, gn, bn, xn, o, bo}))
        return fail(PFM_E_ARG, "pfm_op_ffn_dec: operands must be 16-B aligned");
    CHECK_DEV("pfm_op_ffn_dec", -1, {"x", x}, {"g1", g1}, {"b1n", b1n}, {"W1", W1}, {"b1", b1}, {"W2", W2}, {"gF", gF},
              {"bF", bF}, {"xo", xo}, {"gn", gn}, {"bn", bn}, {"xn", xn}, {"o", o}, {"Wo", Wo}, {"bo", bo});
    const hipStream_t st = (hipStream_t)stream;
    const size_t nw = (size_t)2048 * 512, no = (size_t)512 * 512, po = pfm_ffn_packed_o_elems();
    OpScratch sc;
    bf16 *w1b, *wob, *wp;
    float* cc;
    HIP_TRY(sc.alloc(&w1b, nw));
    HIP_TRY(sc.alloc(&wob, no));
    HIP_TRY(sc.alloc(&wp, po + pfm_ffn_packed_elems()));
    HIP_TRY(sc.alloc(&cc, (size_t)2 * 512));
    HIP_TRY(pfm_f32_to_bf16(W1, w1b, (long long)nw, st));
    if (o) {
        HIP_TRY(pfm_f32_to_bf16(Wo, wob, (long long)no, st));
        HIP_TRY(pfm_ffn_pack_o(wob, wp, st));
    }
    if (pfm_knobs().dec_ffn_fused >= 2) {   // k_ffn2.hip: 128-row tiles (2: the hidden split over two workgroups)
        bf16* wp2;
        float* part;
        unsigned* cnt;
        HIP_TRY(sc.alloc(&wp2, pfm_ffn2_dec_packed_elems()));
        HIP_TRY(sc.alloc(&part, pfm_ffn2_dec_scratch_floats(std::max(M, 1))));
        HIP_TRY(sc.alloc(&cnt, pfm_ffn2_dec_counters(std::max(M, 1))));
        HIP_TRY(hipMemsetAsync(cnt, 0, pfm_ffn2_dec_counters(std::max(M, 1)) * sizeof(unsigned), st));
        const bool split = pfm_knobs().dec_ffn_fused == 2;
        HIP_TRY(pfm_ffn2_pack_dec(w1b, W2, gF, o ? wob : nullptr, wp2, st, split));
        HIP_TRY(pfm_ffn_dec_consts(W2, gF, bF, cc, cc + 512, st));
        HIP_TRY(pfm_ffn2_fused_dec(x, M, g1, b1n, eps, wp2, b1, cc, cc + 512, xo, gn, bn, (bf16*)xn, (const bf16*)o, bo,
                                   split ? part : nullptr, split ? cnt : nullptr, st));
        HIP_TRY(hipStreamSynchronize(st));
        return PFM_OK;
    }
    HIP_TRY(pfm_ffn_pack_dec(w1b, W2, gF, bF, wp + po, cc, cc + 512, st));
    auto dec = pfm_ffn_fused_dec;
    if (o) {   // mode 3: x1 = x + o Wo^T + bo -> xo, then the FFN on x1 (x may alias xo)
        HIP_TRY(dec(x, M, g1, b1n, eps, wp, b1, cc, cc + 512, xo, gn, bn, (bf16*)xn, (const bf16*)o, bo, st));
    } else {
        HIP_TRY(dec(x, M, g1, b1n, eps, wp + po, b1, cc, cc + 512, xo, gn, bn, (bf16*)xn, nullptr, nullptr, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

int pfm_op_attention(void* stream, int dtype, const void* q, const void* k, const void* v, const int32_t* klen,
                     float* out, int B, int Tq, int Tk, int heads, float scale) {
    pfm_knobs_refresh();
    if (!q || !k || !v || !klen || !out || B < 0 || Tq < 0 || Tk < 0 || heads < 1)
        return fail(PFM_E_ARG, "pfm_op_attention: null operand or bad sizes");
    if (dtype != DT_F32 && dtype != DT_BF16) return fail(PFM_E_ARG, "pfm_op_attention: dtype must be PFM_F32 or PFM_BF16");
    CHECK_DEV("pfm_op_attention", -1, {"q", q}, {"k", k}, {"v", v}, {"klen", klen}, {"out", out});
    const int D = heads * 128;
    HIP_TRY(pfm_attention(dtype, q, rowmap_plain(D), k, rowmap_plain(D), v, rowmap_plain(D), out, D, nullptr, klen, B,
                          Tq, Tk, heads, 128, scale, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_layernorm(void* stream, const float* x, const float* g, const float* b, float* out, int M, int D,
                     float eps) {
    pfm_knobs_refresh();
    if (!x || !g || !b || !out || M < 0 || D < 1) return fail(PFM_E_ARG, "pfm_op_layernorm: null operand or bad sizes");
    CHECK_DEV("pfm_op_layernorm", -1, {"x", x}, {"gamma", g}, {"beta", b}, {"out", out});
    HIP_TRY(pfm_layernorm(x, rowmap_plain(D), M, D, g, b, eps, nullptr, 0, 1.f, out, rowmap_plain(D), DT_F32,
                          nullptr, rowmap_plain(0), 0, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_fsmn(void* stream, const float* v, const int32_t* len, const float* w, const float* res, float* out,
                int B, int T, int D, int K, int left) {
    pfm_knobs_refresh();
    if (!v || !len || !w || !out || B < 0 || T < 0 || D < 1 || K < 1 || left < 0)
        return fail(PFM_E_ARG, "pfm_op_fsmn: null operand or bad sizes");
    CHECK_DEV("pfm_op_fsmn", -1, {"v", v}, {"len", len}, {"w", w}, {"res", res}, {"out", out});
    HIP_TRY(pfm_fsmn(v, rowmap_plain(D), len, B, T, D, w, K, left, res, out, nullptr, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_layernorm_bf16(void* stream, const void* x, const float* g, const float* b, float* out, int M, int D,
                          float eps) {
    if (!x || !g || !b || !out || M < 0 || (D != 512 && D != 1024 && D != 2048))
        return fail(PFM_E_ARG, "pfm_op_layernorm_bf16: null operand or bad sizes (D 512 / 1024 / 2048)");
    CHECK_DEV("pfm_op_layernorm_bf16", -1, {"x", x}, {"gamma", g}, {"beta", b}, {"out", out});
    HIP_TRY(pfm_layernorm_bf16in((const bf16*)x, rowmap_plain(D), M, D, g, b, eps, out, rowmap_plain(D), DT_F32,
                                 (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_fsmn_bf16(void* stream, const void* v, const int32_t* len, const float* w, void* out, int B, int T, int D,
                     int K, int left) {
    if (!v || !len || !w || !out || B < 0 || T < 0 || D < 1 || K < 1 || left < 0)
        return fail(PFM_E_ARG, "pfm_op_fsmn_bf16: null operand or bad sizes");
    CHECK_DEV("pfm_op_fsmn_bf16", -1, {"v", v}, {"len", len}, {"w", w}, {"out", out});
    HIP_TRY(pfm_fsmn_bf16in((const bf16*)v, rowmap_plain(D), len, B, T, D, w, K, left, nullptr, nullptr, (bf16*)out,
                            (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_ctc_collapse(void* stream, const int32_t* ids, int64_t ld, const int32_t* olen, int B, int blank,
                        int32_t* tokens, int L_cap, int32_t* ntok) {
    if (!ids || !olen || !tokens || !ntok || B < 0 || L_cap < 0) return fail(PFM_E_ARG, "pfm_op_ctc_collapse: bad arguments");
    CHECK_DEV("pfm_op_ctc_collapse", -1, {"ids", ids}, {"olen", olen}, {"tokens", tokens}, {"ntok", ntok});
    HIP_TRY(pfm_ctc_collapse(ids, ld, olen, B, blank, L_cap, tokens, ntok, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_op_cif(void* stream, const float* alphas, const float* hidden, float* emb, float* peaks, int32_t* n_fire,
               int32_t* ntok, int B, int T, int D, int L_cap) {
    if (!alphas || !hidden || !emb || !peaks || !n_fire || !ntok || B < 0 || T < 0 || D < 1 || L_cap < 0)
        return fail(PFM_E_ARG, "pfm_op_cif: null operand or bad sizes");
    CHECK_DEV("pfm_op_cif", -1, {"alphas", alphas}, {"hidden", hidden}, {"emb", emb}, {"peaks", peaks},
              {"n_fire", n_fire}, {"ntok", ntok});
    HIP_TRY(pfm_cif_fire(alphas, hidden, rowmap_plain(D), B, T, D, L_cap, emb, peaks, n_fire, ntok,
                         (hipStream_t)stream));
    return PFM_OK;
}

int pfm_ctc_align(pfm_handle* h, void* stream, const float* enc, int B, int Tq, const int32_t* olens,
                  const int32_t* targets, int Lmax, const int32_t* tlens, int blank, int32_t* align) {
    pfm_knobs_refresh();
    if (!h || !enc || !olens || !align || (Lmax > 0 && (!targets || !tlens)) || B < 0 || Tq < 0 || Lmax < 0)
        return fail(PFM_E_ARG, "pfm_ctc_align: null argument or bad sizes");
    if (h->cfg.arch != PFM_ARCH_SENSEVOICE) return fail(PFM_E_STATE, "pfm_ctc_align: handle is not a SenseVoice model");
    if (h->missing) return fail(PFM_E_STATE, "pfm_ctc_align: weights not set");
    constexpr int NQ = 4;
    const int V = h->cfg.vocab_size, D = h->cfg.d_model, Tf = Tq - NQ;
    if (blank < 0 || blank >= V) return fail(PFM_E_ARG, "pfm_ctc_align: blank outside the vocabulary");
    if (2 * (2 * (long long)Lmax + 3) * 4 > 64 * 1024) return fail(PFM_E_ARG, "pfm_ctc_align: Lmax too large");
    if (B == 0 || Tf <= 0) return PFM_OK;
    CHECK_DEV("pfm_ctc_align", h->device, {"enc", enc}, {"olens", olens}, {"targets", Lmax > 0 ? targets : nullptr},
              {"tlens", Lmax > 0 ? tlens : nullptr}, {"align", align});
    HIP_TRY(hipSetDevice(h->device));
    const hipStream_t st = (hipStream_t)stream;
    const long long M = (long long)B * Tf;
    // CTC head logits of the speech frames (rows 4 .. Tq-1 of every utterance) in f32 (ctc.ctc_lo)
    OpScratch sc;
    float *logits, *mx, *inv;
    int* amax;
    unsigned char* bp;
    HIP_TRY(sc.alloc(&logits, (size_t)M * V));
    HIP_TRY(sc.alloc(&mx, (size_t)M));
    HIP_TRY(sc.alloc(&inv, (size_t)M));
    HIP_TRY(sc.alloc(&amax, (size_t)M));
    HIP_TRY(sc.alloc(&bp, (size_t)M * (2 * Lmax + 1)));
    GemmEpi e = epi_default();
    e.bias = h->w(h->ctc_b);
    e.out = logits; e.out_map = rowmap_plain(V); e.out_dtype = DT_F32;
    HIP_TRY(gemm_dispatch(DT_F32, enc + (size_t)NQ * D, rowmap_seg(Tf, (long long)Tq * D, D), h->w(h->ctc_w), D,
                          (int)M, V, D, e, st));
    HIP_TRY(pfm_emis_stats(logits, M, V, mx, inv, amax, st));
    HIP_TRY(pfm_ctc_align_run(logits, mx, inv, amax, B, Tf, V, blank, olens, targets, tlens, Lmax, bp, align, st));
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

int pfm_op_ctc_beam(void* stream, const float* am, int L, const float* x, int T, const int32_t* lens,
                    const int32_t* ntok, int B, int V, int beam, float ctc_weight, float penalty, int nbest,
                    int end_detect, int sos, int eos, int blank, int32_t* tokens, int L_cap, int32_t* ntok_out,
                    float* scores_out) {
    if (!am || !x || !lens || !ntok || !tokens || !ntok_out || !scores_out || B < 0 || L < 0 || T < 0 || V < 1)
        return fail(PFM_E_ARG, "pfm_op_ctc_beam: null argument or bad sizes");
    const int pre = (int)(1.5 * beam), P = pre < V ? pre : V;
    if (sos < 0 || sos >= V || eos < 0 || eos >= V || blank < 0 || blank >= V)
        return fail(PFM_E_ARG, "pfm_op_ctc_beam: sos / eos / blank outside the vocabulary");
    if (beam < 1 || beam > 16 || nbest < 1 || nbest > 16 || P > 64 || L_cap < 0)
        return fail(PFM_E_ARG, "pfm_op_ctc_beam: need 1 <= beam <= 16, 1 <= nbest <= 16, <= 64 candidates");
    if (B == 0) return PFM_OK;
    CHECK_DEV("pfm_op_ctc_beam", -1, {"am", am}, {"x", x}, {"lens", lens}, {"ntok", ntok}, {"tokens", tokens},
              {"ntok_out", ntok_out}, {"scores", scores_out});
    const hipStream_t st = (hipStream_t)stream;
    OpScratch sc;
    float* fs;
    int* is;
    HIP_TRY(sc.alloc(&fs, (size_t)B * pfm_ctc_beam_fscratch(beam, P, T, L, V)));
    HIP_TRY(sc.alloc(&is, (size_t)B * pfm_ctc_beam_iscratch(beam, nbest, L, P, V)));
    unsigned* fw;
    HIP_TRY(sc.alloc(&fw, 1));
    HIP_TRY(pfm_ctc_beam(am, L, x, T, lens, ntok, B, V, beam, P, nbest, ctc_weight, penalty, penalty != 0.f ? 1 : 0,
                         end_detect, sos, eos, blank, fs, is, tokens, L_cap, ntok_out, scores_out, fw, st));
    HIP_TRY(hipStreamSynchronize(st));
    return beam_failed(fw, "pfm_op_ctc_beam");
}

}  // extern "C"

// ============================================================================================
// Streaming Paraformer (include/pfm.h, pfm_streams_*): per-slot chunk caches in HBM.
// ============================================================================================
struct pfm_streams {
    std::atomic<unsigned long long> buf_gen{0};   // workspace generation of this object's DevBufs
    GenBind gen_bind_{&buf_gen};
    pfm_handle* h = nullptr;
    int slots = 0, cs[3] = {0, 10, 5}, elb = 0, dlb = 0, mode = PFM_MODE_EXACT;
    int C0 = 5, Ce = 0, Cd = 0;   // overlap rows, encoder / decoder K/V cache capacities (rows)
    DevBuf fcache;                // [slots][C0][I] f32   cache["encoder"]["feats"]
    DevBuf ekv;                   // [enc layers][slots][Ce][2d] operand dtype
    DevBuf dkv;                   // [dec layers][slots][Cd][2d] operand dtype
    DevBuf dfs;                   // [dec layers][slots][K-1][d] f32   decode_fsmn
    DevBuf chid, calpha;          // [slots][d], [slots] f32           cif_hidden / cif_alphas
    DevBuf prm;                   // per step: SPrm[n] | tw[n] | kle[n] | kld[n]
    DevBuf xin, kvbuf, kvw, pe;   // window input, gathered keys, decoder memory K|V, PE table
    int pe_T = 0;
    std::vector<int> start, cle, cld;   // host mirrors per slot
    unsigned char* hprm = nullptr;      // pinned host staging of the per-step parameters
    size_t hprm_cap = 0;
    int32_t* hntok = nullptr;
    int hntok_cap = 0;
    DevBuf fin, tok;                    // chunk rows [n][maxn][I] (graph-stable copy), tokens [n][L_cap]
    // HIP graphs of the two launch sequences of a step (encoder + CIF; decoder),
    // key: (phase, n, maxn, L * 4096 + L_cap, knob signature)
    GraphCache gc;
    hipStream_t cap = nullptr;          // work stream of every step: eager launches, graph capture and replay
    hipEvent_t ev_in = nullptr;
    GenUnbind gen_unbind_;
    // captured graphs stay valid while neither the handle's nor this object's workspace was reallocated
    unsigned long long gen() const { return h->buf_gen.load() + buf_gen.load(); }
    ~pfm_streams() {
        if (ev_in) (void)hipEventDestroy(ev_in);
        if (cap) (void)hipStreamDestroy(cap);
        if (hprm) (void)hipHostFree(hprm);
    }
};

// gathered attention keys of a step: the encoder's one layer at a time, the decoder's all layers at once
static size_t stream_kvbuf_bytes(const pfm_streams* s, int n, int Tw, int D, size_t es, int dec_layers) {
    const size_t enc = s->Ce ? (size_t)n * (s->Ce + Tw) : 0;
    const size_t dec = s->Cd ? (size_t)n * (s->Cd + Tw) * std::max(dec_layers, 1) : 0;
    return std::max(enc, dec) * 2 * D * es;
}

namespace {

// One streaming decoder pass (decoder.py:461-528 over n streams x L token rows): decoders with FFN ->
// causal FSMN (chunk cache) -> cross attention over [K/V cache ;] the window memory, decoders3, after_norm,
// output layer with fused argmax.
int stream_decoder(pfm_streams* s, const Run& r, int n, int Tw, int L, const SPrm* prm, const int* tw_d,
                   const int* kld_d, const int* ntok, int32_t* tokens, int L_cap, float* logits) {
    pfm_handle* h = s->h;
    const pfm_config& c = h->cfg;
    const hipStream_t st = r.st;
    const bool fast = r.fast;
    const int dt = r.dt, D = c.d_model, Fd = c.ffn, K = c.kernel_size, nkv = c.dec_blocks * 2 * D;
    const size_t es = fast ? 2 : 4;
    const long long Ml = (long long)n * L, Mw = (long long)n * Tw;
    const RowMap plain = rowmap_plain(0);
    float* Xd = h->Xd.as<float>();
    void* Xdn = h->Xdn.p;
    float* Hd = h->Hd.as<float>();
    void* Hdn = h->Hdn.p;
    float* Td = h->Td.as<float>();
    void* Tdn = h->Tdn.p;
    void* Qd = h->Qd.p;
    float* Od = h->Od.as<float>();
    bf16* Odb = h->Odb.as<bf16>();
    const float* encp = h->encp.as<float>();
    const bf16* encpb = h->encpb.as<bf16>();
    const RowMap encmap = rowmap_seg(Tw, (long long)(Tw + 2) * D, D);
    const int Lc = Tw + 2;
    HIP_TRY(pfm_rows_copy(Xd, (long long)L * D, h->emb.as<float>(), (long long)Lc * D, L * D, n, st));
    HIP_TRY(s->kvw.ensure((size_t)Mw * nkv * es));
    {   // memory K|V of every decoder layer from the window (rows i*Tw + t)
        GemmEpi e = epi_default();
        e.bias = r.P(h->bkv_all);
        e.out = s->kvw.p; e.out_map = rowmap_plain(nkv); e.out_dtype = dt;
        const void* A = fast ? (const void*)(encpb + D) : (const void*)(encp + D);
        HIP_TRY(r.gemm(dt, A, encmap, r.W(h->wkv_all), D, (int)Mw, nkv, D, e));
    }
    // pout == nullptr: the caller fuses the closing LayerNorm into its consumer (dec_fsmn_ln_stream_kernel)
    auto ffn = [&](const float* x, size_t lng, size_t lnb, size_t w1, size_t b1, size_t fng, size_t fnb, size_t w2,
                   float* out, size_t pg, size_t pb, void* pout, int pdt) -> int {
        GemmEpi e = epi_default();
        e.bias = r.P(b1); e.relu = 1;
        e.out = Hd; e.out_map = rowmap_plain(Fd); e.out_dtype = dt;
        HIP_TRY(r.ln_gemm(x, rowmap_plain(D), lng, lnb, Xdn, rowmap_plain(D), r.W(w1), D, (int)Ml, Fd, D, e));
        GemmEpi e2 = epi_default();
        e2.out = out; e2.out_map = rowmap_plain(D); e2.out_dtype = DT_F32;
        if (fast && pfm_gemm_skinny_ln2048_ok((const bf16*)Hd, rowmap_plain(Fd), r.W(w2), Fd, (int)Ml, D, Fd, e2)) {
            // the hidden's LayerNorm (2048 wide) in the w2 GEMM's A load
            ProfScope ps(h, st, PFM_K_GEMM, 2.0 * Ml * D * (double)Fd, (double)Ml * Fd * 2.0 + (double)D * Fd * 2.0 +
                                                                      (double)Ml * D * 4.0);
            HIP_TRY(pfm_gemm_skinny_ln2048((const bf16*)Hd, rowmap_plain(Fd), r.P(fng), r.P(fnb), c.ln_eps, r.W(w2), Fd,
                                           (int)Ml, D, e2, st));
        } else {
            if (fast)
                HIP_TRY(pfm_layernorm_bf16in((const bf16*)Hd, rowmap_plain(Fd), (int)Ml, Fd, r.P(fng), r.P(fnb), c.ln_eps,
                                             Hdn, rowmap_plain(Fd), dt, st));
            else
                HIP_TRY(pfm_layernorm(Hd, rowmap_plain(Fd), (int)Ml, Fd, r.P(fng), r.P(fnb), c.ln_eps, nullptr, 0, 1.f,
                                      Hdn, rowmap_plain(Fd), dt, nullptr, plain, 0, st));
            HIP_TRY(r.gemm(dt, Hdn, rowmap_plain(Fd), r.W(w2), Fd, (int)Ml, D, Fd, e2));
        }
        if (pout)
            HIP_TRY(pfm_layernorm(out, rowmap_plain(D), (int)Ml, D, r.P(pg), r.P(pb), c.ln_eps, nullptr, 0, 1.f, pout,
                                  rowmap_plain(D), pdt, nullptr, plain, 0, st));
        return PFM_OK;
    };
    const int Tk = s->Cd + Tw;
    // decoder look-back: the keys of every layer ([its K/V cache ; the window's memory K|V]) gathered in one launch
    // before the layers run (each layer's retain then rewrites only its own cache)
    const long long kv_ls = (long long)n * Tk * 2 * D;
    if (s->dlb > 0) {
        HIP_TRY(s->kvbuf.ensure(stream_kvbuf_bytes(s, n, Tw, D, es, c.dec_blocks)));
        HIP_TRY(pfm_kv_gather_layers(dt, s->dkv.p, (long long)s->slots * s->Cd * 2 * D, s->Cd, prm, n, 1, s->kvw.p, 2 * D,
                                     nkv, Tw, s->kvbuf.p, kv_ls, Tk, 2 * D, c.dec_blocks, st));
    }
    for (int l = 0; l < c.dec_blocks; ++l) {
        const DecLayer& Lr = h->dec[l];
        // fast mode: norm2 runs in the FSMN kernel's prologue (dec_fsmn_ln_stream_kernel)
        const bool fuse_n2 = fast && K == 11 && D == 512 && L <= 64;
        int rc = ffn(Xd, Lr.n1g, Lr.n1b, Lr.w1, Lr.b1, Lr.ng, Lr.nb, Lr.w2, Td, Lr.n2g, Lr.n2b, fuse_n2 ? nullptr : Tdn, dt);
        if (rc) return rc;
        float* dstate = s->dfs.as<float>() + (size_t)l * s->slots * (K - 1) * D;
        const hipError_t ef = fuse_n2 ? pfm_dec_fsmn_ln_stream(Td, r.P(Lr.n2g), r.P(Lr.n2b), c.ln_eps, r.P(Lr.fsmn), K,
                                                               dstate, prm, ntok, n, L, D, Xd, st)
                                      : hipErrorNotSupported;
        if (ef != hipErrorNotSupported) {
            HIP_TRY(ef);
        } else {
            if (fuse_n2)   // (unaligned vectors: the separate LayerNorm after all)
                HIP_TRY(pfm_layernorm(Td, rowmap_plain(D), (int)Ml, D, r.P(Lr.n2g), r.P(Lr.n2b), c.ln_eps, nullptr, 0, 1.f,
                                      Tdn, rowmap_plain(D), dt, nullptr, plain, 0, st));
            HIP_TRY(pfm_dec_fsmn_stream(dt, Tdn, r.P(Lr.fsmn), K, dstate, prm, ntok, n, L, D, Xd, st));
        }
        {
            GemmEpi e = epi_default();
            e.bias = r.P(Lr.bq);
            e.out = Qd; e.out_map = rowmap_plain(D); e.out_dtype = dt;
            HIP_TRY(r.ln_gemm(Xd, rowmap_plain(D), Lr.n3g, Lr.n3b, Xdn, rowmap_plain(D), r.W(Lr.wq), D, (int)Ml, D, D, e));
        }
        const char* kvl = (const char*)s->kvw.p + (size_t)l * 2 * D * es;
        if (s->dlb > 0) {
            void* cache = (char*)s->dkv.p + (size_t)l * s->slots * s->Cd * 2 * D * es;
            void* kb = (char*)s->kvbuf.p + (size_t)l * kv_ls * es;
            const hipError_t ea = fast ? r.attn_rt((const bf16*)Qd, rowmap_plain(D), kb, (bf16*)Odb, kld_d, n, L, Tk, prm, cache,
                                                   s->Cd, 0, 1, ntok)
                                       : hipErrorNotSupported;
            if (ea != hipErrorNotSupported) {
                HIP_TRY(ea);
            } else {
                const RowMap km = rowmap_seg(Tk, (long long)Tk * 2 * D, 2 * D);
                HIP_TRY(r.attn(dt, Qd, rowmap_plain(D), kb, km, (const char*)kb + (size_t)D * es, km,
                               fast ? nullptr : Od, D, fast ? (void*)Odb : nullptr, kld_d, n, L, Tk));
                HIP_TRY(pfm_kv_retain(dt, kb, Tk, prm, n, 1, 0, ntok, cache, s->Cd, 2 * D, st));
            }
        } else {
            HIP_TRY(r.attn(dt, Qd, rowmap_plain(D), kvl, rowmap_plain(nkv), kvl + (size_t)D * es, rowmap_plain(nkv),
                           fast ? nullptr : Od, D, fast ? (void*)Odb : nullptr, tw_d, n, L, Tw));
        }
        {
            GemmEpi e = epi_default();
            e.bias = r.P(Lr.bo);
            e.res0 = Xd; e.ld_res0 = D;
            e.out = Xd; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
            HIP_TRY(r.gemm(dt, fast ? (const void*)Odb : (const void*)Od, rowmap_plain(D), r.W(Lr.wo), D, (int)Ml, D,
                           D, e));
        }
    }
    int rc = ffn(Xd, h->d3n1g, h->d3n1b, h->d3w1, h->d3b1, h->d3ng, h->d3nb, h->d3w2, Xd, h->dan_g, h->dan_b, Xdn, dt);
    if (rc) return rc;
    if (logits) {   // CTC prefix beam (pfm_stream_step_beam): the f32 logits [n][L][V] themselves
        GemmEpi e = epi_default();
        e.bias = r.P(h->out_b);
        e.out = logits; e.out_map = rowmap_plain(c.vocab_size); e.out_dtype = DT_F32;
        HIP_TRY(r.gemm(dt, Xdn, rowmap_plain(D), r.W(h->out_w), D, (int)Ml, c.vocab_size, D, e));
        return PFM_OK;
    }
    const int ntl = amax_tiles(dt, rowmap_plain(D), D, c.vocab_size, D, h, r.W(h->out_w));
    GemmEpi e = epi_default();
    e.bias = r.P(h->out_b);
    e.amax_val = h->amv.as<float>(); e.amax_idx = h->ami.as<int>(); e.n_tiles = ntl;
    e.out = nullptr;
    HIP_TRY(r.gemm(dt, Xdn, rowmap_plain(D), r.W(h->out_w), D, (int)Ml, c.vocab_size, D, e));
    if (L_cap > 0)
        HIP_TRY(pfm_argmax_reduce(h->amv.as<float>(), h->ami.as<int>(), ntl, (c.vocab_size + 63) / 64, n, L, ntok,
                                  L_cap, tokens, nullptr, st));
    return PFM_OK;
}

template <class F>
int stream_graphed(pfm_streams* s, std::array<int, 4> shape, bool use, hipStream_t st, F&& body) {
    return graphed(s->gc, "stream", shape, use, st, [s] { return s->gen(); }, std::forward<F>(body));
}

int streams_zero(pfm_streams* s, hipStream_t st, int slot) {
    const pfm_config& c = s->h->cfg;
    const size_t D = c.d_model, I = c.input_size, K1 = c.kernel_size - 1;
    const size_t es = s->mode == PFM_MODE_FAST ? 2 : 4;
    HIP_TRY(hipMemsetAsync(s->fcache.as<float>() + (size_t)slot * s->C0 * I, 0, (size_t)s->C0 * I * 4, st));
    HIP_TRY(hipMemsetAsync(s->chid.as<float>() + (size_t)slot * D, 0, D * 4, st));
    HIP_TRY(hipMemsetAsync(s->calpha.as<float>() + slot, 0, 4, st));
    for (int l = 0; l < c.dec_blocks; ++l)
        HIP_TRY(hipMemsetAsync(s->dfs.as<float>() + ((size_t)l * s->slots + slot) * K1 * D, 0, K1 * D * 4, st));
    // K/V caches need no clearing: rows beyond cle / cld are never read
    (void)es;
    s->start[slot] = 0;
    s->cle[slot] = 0;
    s->cld[slot] = 0;
    return PFM_OK;
}

}  // namespace

extern "C" {

int pfm_streams_create(pfm_handle* h, int slots, const int32_t* chunk_size, int enc_look_back, int dec_look_back,
                       int mode, pfm_streams** out) {
    pfm_knobs_refresh();
    if (!h || !chunk_size || !out) return fail(PFM_E_ARG, "pfm_streams_create: null argument");
    *out = nullptr;
    const pfm_config& c = h->cfg;
    if (c.arch != PFM_ARCH_PARAFORMER) return fail(PFM_E_STATE, "pfm_streams_create: handle is not a Paraformer");
    if (c.dec_sanm_shift != 5 || c.kernel_size != 11)
        return fail(PFM_E_ARG, "pfm_streams_create: streaming needs the causal decoder FSMN (kernel 11, sanm_shfit 5)");
    if (slots < 1) return fail(PFM_E_ARG, "pfm_streams_create: slots must be >= 1");
    if (chunk_size[0] < 0 || chunk_size[1] < 1 || chunk_size[2] < 0 || chunk_size[0] + chunk_size[2] < 1 ||
        chunk_size[0] + chunk_size[1] + chunk_size[2] > 60)
        return fail(PFM_E_ARG, "pfm_streams_create: bad chunk_size");
    if (enc_look_back < 0 || dec_look_back < 0 || enc_look_back > 64 || dec_look_back > 64)
        return fail(PFM_E_ARG, "pfm_streams_create: look-back must be in [0, 64] (unbounded -1 is not supported)");
    if (mode != PFM_MODE_EXACT && mode != PFM_MODE_FAST) return fail(PFM_E_ARG, "pfm_streams_create: bad mode");
    HIP_TRY(hipSetDevice(h->device));
    std::unique_ptr<pfm_streams> s(new pfm_streams());
    s->h = h;
    s->slots = slots;
    for (int k = 0; k < 3; ++k) s->cs[k] = chunk_size[k];
    s->elb = enc_look_back;
    s->dlb = dec_look_back;
    s->mode = mode;
    s->C0 = chunk_size[0] + chunk_size[2];
    s->Ce = enc_look_back * chunk_size[1];
    s->Cd = dec_look_back * chunk_size[1];
    const size_t D = c.d_model, I = c.input_size, K1 = c.kernel_size - 1, es = mode == PFM_MODE_FAST ? 2 : 4;
    HIP_TRY(s->fcache.ensure((size_t)slots * s->C0 * I * 4));
    HIP_TRY(s->chid.ensure((size_t)slots * D * 4));
    HIP_TRY(s->calpha.ensure((size_t)slots * 4));
    HIP_TRY(s->dfs.ensure((size_t)std::max(c.dec_blocks, 1) * slots * K1 * D * 4));
    if (s->Ce) HIP_TRY(s->ekv.ensure((size_t)c.enc_blocks * slots * s->Ce * 2 * D * es));
    if (s->Cd) HIP_TRY(s->dkv.ensure((size_t)std::max(c.dec_blocks, 1) * slots * s->Cd * 2 * D * es));
    HIP_TRY(hipStreamCreateWithFlags(&s->cap, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming));
    s->start.assign(slots, 0);
    s->cle.assign(slots, 0);
    s->cld.assign(slots, 0);
    for (int k = 0; k < slots; ++k) {
        int rc = streams_zero(s.get(), nullptr, k);
        if (rc) return rc;
    }
    HIP_TRY(hipDeviceSynchronize());
    *out = s.release();
    return PFM_OK;
}

int pfm_streams_reset(pfm_streams* s, void* stream, const int32_t* slot_ids, int n) {
    if (!s || (n > 0 && !slot_ids)) return fail(PFM_E_ARG, "pfm_streams_reset: null argument");
    HIP_TRY(hipSetDevice(s->h->device));
    for (int k = 0; k < n; ++k) {
        if (slot_ids[k] < 0 || slot_ids[k] >= s->slots) return fail(PFM_E_ARG, "pfm_streams_reset: bad slot id");
        int rc = streams_zero(s, (hipStream_t)stream, slot_ids[k]);
        if (rc) return rc;
    }
    return PFM_OK;
}

}  // extern "C"

namespace {

// The CTC prefix beam of one streaming step (pfm_stream_step_beam)
struct StreamBeam {
    int beam, P, nbest, end_detect, sos, eos, blank;
    float ctc_weight, penalty;
    int32_t* ntok_hyp;   // [n][nbest]
    float* scores;       // [n][nbest]
};

int stream_step(pfm_streams* s, void* stream, int n, const int32_t* slot_ids, const float* feats, int Tn,
                const int32_t* nfeat, const int32_t* is_final, int32_t* tokens, int L_cap, int32_t* ntok_out,
                float* enc_out, float* alphas_out, const StreamBeam* sb) {
    pfm_handle* h = s->h;
    const pfm_config& c = h->cfg;
    if (h->missing) return fail(PFM_E_STATE, "pfm_stream_step: weights not set");
    int maxn = 0;
    std::vector<char> seen(s->slots, 0);
    for (int i = 0; i < n; ++i) {
        const int sl = slot_ids[i];
        if (sl < 0 || sl >= s->slots || seen[sl]) return fail(PFM_E_ARG, "pfm_stream_step: bad or repeated slot id");
        seen[sl] = 1;
        if (nfeat[i] < 0 || nfeat[i] > Tn) return fail(PFM_E_ARG, "pfm_stream_step: nfeat out of [0, Tn]");
        if (nfeat[i] == 0 && !is_final[i]) return fail(PFM_E_ARG, "pfm_stream_step: the tail chunk (nfeat 0) must be final");
        maxn = std::max(maxn, (int)nfeat[i]);
    }
    if (maxn > 0 && !feats) return fail(PFM_E_ARG, "pfm_stream_step: feats is null");
    HIP_TRY(hipSetDevice(h->device));
    // every launch of a step goes to the object's own stream, ordered after the caller's queued work (the
    // chunk rows, a reset) by one event; the step synchronises that stream before returning, so its outputs
    // are ready for any stream. (The caller's stream may be the legacy null stream, whose ordering with
    // graph launches on other streams was observed to be unreliable.)
    HIP_TRY(hipEventRecord(s->ev_in, (hipStream_t)stream));
    HIP_TRY(hipStreamWaitEvent(s->cap, s->ev_in, 0));
    hipStream_t st = s->cap;
    const bool fast = s->mode == PFM_MODE_FAST;
    const int D = c.d_model, I = c.input_size, C0 = s->C0;
    const int Tw = C0 + maxn;
    // the beam path writes whole hypotheses: check L_cap against the worst-case fire count (one per window row,
    // plus the final chunk's tail fire) before any stream state moves, so a refused step can be retried
    if (sb && L_cap < Tw + 1)
        return fail(PFM_E_ARG, "pfm_stream_step_beam: L_cap " + std::to_string(L_cap) + " below the window's " +
                                   std::to_string(Tw + 1) + " possible tokens");
    int rc = reserve(h, n, Tw + 2);
    if (rc) return rc;
    if (fast) { rc = ensure_bf16(h, st); if (rc) return rc; }
    else { rc = ensure_x6(h, st); if (rc) return rc; }
    // PE rows up to the furthest position of this step (grown by doubling)
    int need = 1;
    for (int i = 0; i < n; ++i) need = std::max(need, s->start[slot_ids[i]] + (int)nfeat[i]);
    if (need > s->pe_T) {
        const int T2 = std::max(need, std::max(2 * s->pe_T, 1024));
        std::vector<float> pe;
        make_pe(pe, T2, I);
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(s->pe.ensure(pe.size() * 4));
        HIP_TRY(hipMemcpy(s->pe.p, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
        s->pe_T = T2;
    }
    // every buffer this step touches is sized here, before any launch sequence that may be captured
    const size_t es = fast ? 2 : 4;
    const int nkv = c.dec_blocks * 2 * D;
    const size_t pb = (size_t)n * sizeof(SPrm), ib = (size_t)n * 4;
    HIP_TRY(s->prm.ensure(pb + 3 * ib));
    HIP_TRY(s->xin.ensure((size_t)n * Tw * I * 4));
    HIP_TRY(s->fin.ensure((size_t)n * std::max(maxn, 1) * I * 4));
    if (s->Ce || s->Cd) HIP_TRY(s->kvbuf.ensure(stream_kvbuf_bytes(s, n, Tw, D, es, c.dec_blocks)));
    if (c.dec_blocks > 0) HIP_TRY(s->kvw.ensure((size_t)n * Tw * nkv * es));
    HIP_TRY(s->tok.ensure((size_t)n * std::max(L_cap, 1) * 4));
    if (s->hntok_cap < n) {
        if (s->hntok) (void)hipHostFree(s->hntok);
        s->hntok = nullptr;
        HIP_TRY(hipHostMalloc((void**)&s->hntok, (size_t)n * 4, 0));
        s->hntok_cap = n;
    }
    if (s->hprm_cap < pb + 3 * ib) {
        if (s->hprm) (void)hipHostFree(s->hprm);
        s->hprm = nullptr;
        HIP_TRY(hipHostMalloc((void**)&s->hprm, pb + 3 * ib, 0));
        s->hprm_cap = pb + 3 * ib;
    }
    // per-stream parameters: SPrm[n] | tw[n] | kle[n] | kld[n] (pinned staging; the previous step's upload
    // has completed: every step synchronises the stream before returning)
    SPrm* hp = (SPrm*)s->hprm;
    int* htw = (int*)(s->hprm + pb);
    int* hkle = htw + n;
    int* hkld = hkle + n;
    for (int i = 0; i < n; ++i) {
        const int sl = slot_ids[i];
        SPrm p;
        p.slot = sl; p.nfeat = nfeat[i]; p.start = s->start[sl]; p.tw = C0 + nfeat[i]; p.fin = is_final[i] ? 1 : 0;
        p.cle = s->Ce ? s->cle[sl] : 0; p.cld = s->Cd ? s->cld[sl] : 0; p.pad = 0;
        hp[i] = p;
        htw[i] = p.tw;
        hkle[i] = p.cle + p.tw;
        hkld[i] = p.cld + p.tw;
    }
    HIP_TRY(hipMemcpyAsync(s->prm.p, s->hprm, pb + 3 * ib, hipMemcpyHostToDevice, st));
    const SPrm* prm = s->prm.as<SPrm>();
    const int* tw_d = (const int*)((const char*)s->prm.p + pb);
    const int* kle_d = tw_d + n;
    const int* kld_d = kle_d + n;
    // the chunk rows, re-pitched to maxn rows per stream in a buffer whose address a graph can keep
    float* fin = s->fin.as<float>();
    if (maxn > 0)
        HIP_TRY(hipMemcpy2DAsync(fin, (size_t)maxn * I * 4, feats, (size_t)Tn * I * 4, (size_t)maxn * I * 4, n,
                                 hipMemcpyDeviceToDevice, st));
    float* encp = h->encp.as<float>();
    bf16* encpb = h->encpb.as<bf16>();
    int* ntok = h->ntok.as<int>();
    const int Lc = Tw + 2;
    const RowMap encmap = rowmap_seg(Tw, (long long)(Tw + 2) * D, D);
    // HIP graphs replace the ~10 launches per encoder layer when no optional output is requested: kernels
    // read every per-step value from `prm`, so one graph per (n, maxn) replays any step of that shape
    const bool graphs = !enc_out && !alphas_out && !h->prof_on && pfm_knobs().stream_graph;
    const int V = c.vocab_size;
    if (sb) {   // the beam's f32 decoder / CTC log-probs, sized before any capture
        HIP_TRY(h->logits.ensure((size_t)n * L_cap * V * sizeof(float)));
        HIP_TRY(h->ctcx.ensure((size_t)n * Tw * V * sizeof(float)));
    }

    // ---- phase A: encoder window + SANMEncoderChunkOpt.forward_chunk (scama/encoder.py:456-499) +
    // CifPredictorV2.forward_chunk (cif_predictor.py:255-344) -> acoustic embeds, ntok on the device
    auto phaseA = [&](hipStream_t q) -> int {
        float* xin = s->xin.as<float>();
        HIP_TRY(pfm_stream_window(fin, maxn, prm, n, s->fcache.as<float>(), s->pe.as<float>(), I, C0, Tw,
                                  sqrtf((float)D), xin, q));
        HIP_TRY(pfm_stream_fcache(xin, prm, n, I, C0, Tw, s->fcache.as<float>(), q));
        Run run(h, q, fast);
        run.fuse_fsmn = false;
        run.raw_input = true;
        ChunkKV ck;
        if (s->Ce) {
            ck.cache = s->ekv.p;
            ck.layer_stride = (long long)s->slots * s->Ce * 2 * D;
            ck.C = s->Ce; ck.drop = s->cs[2]; ck.Tk = s->Ce + Tw;
            ck.buf = s->kvbuf.p; ck.prm = prm; ck.klen = kle_d;
            run.ck = &ck;
        }
        HIP_TRY(pfm_pad_rows_zero(encp, fast ? encpb : nullptr, n, Tw, D, q));
        const FinalLN finln = {h->an_g, h->an_b, encp + D, encmap, DT_F32, fast ? (void*)(encpb + D) : nullptr,
                               encmap, DT_BF16};
        int rc2 = encoder_stack(run, xin, tw_d, n, Tw, 0, c.enc_blocks, h->X.as<float>(), finln, enc_ws(h, 0));
        if (rc2) return rc2;
        HIP_TRY(pfm_stream_mask_rows(encp, fast ? encpb : nullptr, prm, n, Tw, D, q));
        GemmEpi e = epi_default();
        e.bias = run.P(h->cif_b); e.relu = 1;
        e.out = h->Hc.p; e.out_map = rowmap_plain(D); e.out_dtype = DT_F32;
        const void* A = fast ? (const void*)encpb : (const void*)encp;
        HIP_TRY(run.gemm(run.dt, A, rowmap_seg(Tw, (long long)(Tw + 2) * D, D), run.W(h->cif_w), 3 * D, n * Tw, D,
                         3 * D, e));
        HIP_TRY(pfm_cif_chunk(h->Hc.as<float>(), run.P(h->cif_ow), run.P(h->cif_ob), encp, prm, n, Tw, D, s->cs[0],
                              s->cs[0] + s->cs[1], c.smooth_factor, c.noise_threshold, c.tail_threshold,
                              c.cif_threshold, s->chid.as<float>(), s->calpha.as<float>(), h->emb.as<float>(), Lc,
                              ntok, alphas_out, q));
        return PFM_OK;
    };
    rc = stream_graphed(s, {0, n, maxn, 0}, graphs, st, phaseA);
    if (rc) return rc;
    if (enc_out)
        HIP_TRY(hipMemcpy2DAsync(enc_out, (size_t)Tw * D * 4, encp + D, (size_t)(Tw + 2) * D * 4, (size_t)Tw * D * 4, n,
                                 hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(ntok_out, ntok, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(s->hntok, ntok, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    int L = 0;
    for (int i = 0; i < n; ++i) L = std::max(L, (int)s->hntok[i]);
    // host mirrors of the caches (the device caches were advanced by the kernels above / below)
    for (int i = 0; i < n; ++i) {
        const int sl = slot_ids[i];
        const int tw = C0 + nfeat[i];
        s->start[sl] += nfeat[i] ? nfeat[i] : C0;
        if (s->Ce) s->cle[sl] = std::min(s->Ce, s->cle[sl] + tw - s->cs[2]);
        if (s->Cd && s->hntok[i] > 0) s->cld[sl] = std::min(s->Cd, s->cld[sl] + tw);
    }
    if (L < 1 || c.dec_blocks < 1) {   // model.py:490-491: nothing to decode
        const long long nb = sb ? sb->nbest : 1;
        if (L_cap > 0) HIP_TRY(pfm_fill_i32(tokens, n * nb * L_cap, -1, st));
        if (sb) {
            HIP_TRY(pfm_fill_i32(sb->ntok_hyp, n * nb, -1, st));
            HIP_TRY(hipMemsetAsync(sb->scores, 0, (size_t)(n * nb) * sizeof(float), st));
        }
        HIP_TRY(hipStreamSynchronize(st));
        return PFM_OK;
    }
    if (sb) {   // model.py:510-519: BeamSearchPara per stream on its window's CTC log-probs and decoder log-probs
        if (L > L_cap) return fail(PFM_E_ARG, "pfm_stream_step_beam: L_cap below the chunk's token count");
        {
            Run run(h, st, fast);
            int rc2 = stream_decoder(s, run, n, Tw, L, prm, tw_d, kld_d, ntok, nullptr, 0, h->logits.as<float>());
            if (rc2) return rc2;
            // ctc.log_softmax of the window (encoder_out[i, :encoder_out_lens[i]], lens = the window rows)
            GemmEpi e = epi_default();
            e.bias = run.P(h->ctc_b);
            e.out = h->ctcx.p; e.out_map = rowmap_plain(V); e.out_dtype = DT_F32;
            const void* A = fast ? (const void*)(encpb + D) : (const void*)(encp + D);
            HIP_TRY(run.gemm(run.dt, A, encmap, run.W(h->ctc_w), D, n * Tw, V, D, e));
        }
        HIP_TRY(pfm_logsoftmax_rows(h->ctcx.as<float>(), (long long)n * Tw, V, V, st));
        HIP_TRY(pfm_logsoftmax_rows(h->logits.as<float>(), (long long)n * L, V, V, st));
        HIP_TRY(hipMemsetAsync(sb->scores, 0, (size_t)n * sb->nbest * sizeof(float), st));
        const long long fsz = pfm_ctc_beam_fscratch(sb->beam, sb->P, Tw, L, V);
        const long long isz = pfm_ctc_beam_iscratch(sb->beam, sb->nbest, L, sb->P, V);
        HIP_TRY(h->beam_fs.ensure((size_t)n * fsz * sizeof(float)));
        HIP_TRY(h->beam_is.ensure((size_t)n * isz * sizeof(int32_t)));
        HIP_TRY(h->beam_fail.ensure(sizeof(unsigned)));
        HIP_TRY(pfm_ctc_beam(h->logits.as<float>(), L, h->ctcx.as<float>(), Tw, tw_d, ntok, n, V, sb->beam, sb->P,
                             sb->nbest, sb->ctc_weight, sb->penalty, sb->penalty != 0.f ? 1 : 0, sb->end_detect, sb->sos,
                             sb->eos, sb->blank, h->beam_fs.as<float>(), h->beam_is.as<int>(), tokens, L_cap,
                             sb->ntok_hyp, sb->scores, h->beam_fail.as<unsigned>(), st));
        HIP_TRY(hipStreamSynchronize(st));
        return beam_failed(h->beam_fail.as<unsigned>(), "pfm_stream_step_beam");
    }
    // ---- phase B: ParaformerSANMDecoder.forward_chunk (decoder.py:461-528) + greedy argmax, tokens into
    // the step's token buffer
    int32_t* tk = s->tok.as<int32_t>();
    auto phaseB = [&](hipStream_t q) -> int {
        if (L_cap > 0) HIP_TRY(pfm_fill_i32(tk, (long long)n * L_cap, -1, q));
        Run run(h, q, fast);
        return stream_decoder(s, run, n, Tw, L, prm, tw_d, kld_d, ntok, tk, L_cap, nullptr);
    };
    rc = stream_graphed(s, {1, n, maxn, L * 4096 + L_cap}, graphs, st, phaseB);
    if (rc) return rc;
    if (L_cap > 0) HIP_TRY(hipMemcpyAsync(tokens, tk, (size_t)n * L_cap * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return PFM_OK;
}

}  // namespace

extern "C" {

int pfm_stream_step(pfm_streams* s, void* stream, int n, const int32_t* slot_ids, const float* feats, int Tn,
                    const int32_t* nfeat, const int32_t* is_final, int32_t* tokens, int L_cap, int32_t* ntok_out,
                    float* enc_out, float* alphas_out) {
    pfm_knobs_refresh();
    if (!s || !slot_ids || !nfeat || !is_final || !tokens || !ntok_out)
        return fail(PFM_E_ARG, "pfm_stream_step: null argument");
    if (n < 1 || Tn < 0 || L_cap < 0) return fail(PFM_E_ARG, "pfm_stream_step: bad sizes");
    CHECK_DEV("pfm_stream_step", s->h->device, {"feats", feats}, {"tokens", tokens}, {"ntok", ntok_out},
              {"enc_out", enc_out}, {"alphas", alphas_out});
    return stream_step(s, stream, n, slot_ids, feats, Tn, nfeat, is_final, tokens, L_cap, ntok_out, enc_out,
                       alphas_out, nullptr);
}

int pfm_stream_step_beam(pfm_streams* s, void* stream, int n, const int32_t* slot_ids, const float* feats, int Tn,
                         const int32_t* nfeat, const int32_t* is_final, int beam, float ctc_weight, float penalty,
                         int nbest, int end_detect, int sos, int eos, int blank, int32_t* tokens, int L_cap,
                         int32_t* ntok_out, float* scores_out, int32_t* nfire) {
    pfm_knobs_refresh();
    if (!s || !slot_ids || !nfeat || !is_final || !tokens || !ntok_out || !scores_out)
        return fail(PFM_E_ARG, "pfm_stream_step_beam: null argument");
    if (n < 1 || Tn < 0 || L_cap < 1) return fail(PFM_E_ARG, "pfm_stream_step_beam: bad sizes");
    const pfm_config& c = s->h->cfg;
    if (!c.ctc_head) return fail(PFM_E_STATE, "pfm_stream_step_beam: the model has no CTC head (ctc_weight 0.0)");
    const int V = c.vocab_size;
    const int pre = (int)(1.5 * beam), P = pre < V ? pre : V;
    if (sos < 0 || sos >= V || eos < 0 || eos >= V || blank < 0 || blank >= V)
        return fail(PFM_E_ARG, "pfm_stream_step_beam: sos / eos / blank outside the vocabulary");
    if (beam < 1 || beam > 16 || nbest < 1 || nbest > 16 || P > 64 || !(ctc_weight > 1e-5f))
        return fail(PFM_E_ARG,
                    "pfm_stream_step_beam: need 1 <= beam <= 16, 1 <= nbest <= 16, ctc_weight > 1e-5, <= 64 candidates");
    CHECK_DEV("pfm_stream_step_beam", s->h->device, {"feats", feats}, {"tokens", tokens}, {"ntok", ntok_out},
              {"scores", scores_out}, {"nfire", nfire});
    StreamBeam sb;
    sb.beam = beam; sb.P = P; sb.nbest = nbest; sb.end_detect = end_detect; sb.sos = sos; sb.eos = eos;
    sb.blank = blank; sb.ctc_weight = ctc_weight; sb.penalty = penalty; sb.ntok_hyp = ntok_out;
    sb.scores = scores_out;
    // the CIF fire counts go to nfire (or a scratch the step owns)
    int32_t* nf = nfire;
    if (!nf) {
        HIP_TRY(s->h->beam_nf.ensure((size_t)n * sizeof(int32_t)));
        nf = s->h->beam_nf.as<int32_t>();
    }
    return stream_step(s, stream, n, slot_ids, feats, Tn, nfeat, is_final, tokens, L_cap, nf, nullptr, nullptr, &sb);
}

void pfm_streams_destroy(pfm_streams* s) {
    if (!s) return;
    (void)hipSetDevice(s->h->device);
    (void)hipDeviceSynchronize();
    if (s->hntok) (void)hipHostFree(s->hntok);
    delete s;
}

}  // extern "C"

// ============================================================================================
// FSMN-VAD encoder (include/pfm.h, pfm_vad_*): one stream, per-layer memory caches in HBM.
// ============================================================================================
struct pfm_vad {
    pfm_vad_config cfg;
    int device = 0;
    struct W { std::vector<int64_t> shape; size_t off = 0, numel = 0; bool set = false; };
    std::unordered_map<std::string, W> reg;
    size_t elems = 0;
    int missing = 0;
    DevBuf arena, cache, ctmp, h1, h2, pa, pb, o1, lg;
    DevBuf fb_tab;        // fbank tables of the object's own online frontend (pfm_vad_fbank_raw)
    bool fb_ready = false;
    int capT = 0;
    size_t add(const std::string& n, std::vector<int64_t> shape) {
        W w;
        w.shape = shape;
        w.numel = 1;
        for (auto d : shape) w.numel *= (size_t)d;
        w.off = elems;
        elems += (w.numel + 63) & ~size_t(63);
        reg[n] = w;
        ++missing;
        return w.off;
    }
    float* p(const std::string& n) { return arena.as<float>() + reg[n].off; }
};

extern "C" {

void pfm_vad_config_default(pfm_vad_config* c) {
    c->input_dim = 400; c->input_affine_dim = 140; c->fsmn_layers = 4; c->linear_dim = 250; c->proj_dim = 128;
    c->lorder = 20; c->output_affine_dim = 140; c->output_dim = 248;
}

int pfm_vad_create(const pfm_vad_config* c, int device, pfm_vad** out) {
    if (!c || !out) return fail(PFM_E_ARG, "pfm_vad_create: null argument");
    *out = nullptr;
    if (c->input_dim < 1 || c->input_affine_dim < 1 || c->fsmn_layers < 0 || c->linear_dim < 1 || c->proj_dim < 1 ||
        c->lorder < 1 || c->output_affine_dim < 1 || c->output_dim < 1)
        return fail(PFM_E_ARG, "pfm_vad_create: bad dims");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(PFM_E_ARG, "pfm_vad_create: bad device index");
    HIP_TRY(hipSetDevice(device));
    std::unique_ptr<pfm_vad> v(new pfm_vad());
    v->cfg = *c;
    v->device = device;
    const int64_t I = c->input_dim, A = c->input_affine_dim, Lin = c->linear_dim, P = c->proj_dim, L = c->lorder,
                  OA = c->output_affine_dim, O = c->output_dim;
    v->add("encoder.in_linear1.linear.weight", {A, I});
    v->add("encoder.in_linear1.linear.bias", {A});
    v->add("encoder.in_linear2.linear.weight", {Lin, A});
    v->add("encoder.in_linear2.linear.bias", {Lin});
    for (int i = 0; i < c->fsmn_layers; ++i) {
        const std::string p = "encoder.fsmn." + std::to_string(i);
        v->add(p + ".linear.linear.weight", {P, Lin});
        v->add(p + ".fsmn_block.conv_left.weight", {P, 1, L, 1});
        v->add(p + ".affine.linear.weight", {Lin, P});
        v->add(p + ".affine.linear.bias", {Lin});
    }
    v->add("encoder.out_linear1.linear.weight", {OA, Lin});
    v->add("encoder.out_linear1.linear.bias", {OA});
    v->add("encoder.out_linear2.linear.weight", {O, OA});
    v->add("encoder.out_linear2.linear.bias", {O});
    HIP_TRY(v->arena.ensure(v->elems * 4));
    HIP_TRY(hipMemset(v->arena.p, 0, v->arena.bytes));
    const size_t nc = (size_t)std::max(c->fsmn_layers, 1) * std::max(L - 1, (int64_t)1) * P;
    HIP_TRY(v->cache.ensure(nc * 4));
    HIP_TRY(v->ctmp.ensure((size_t)std::max(L - 1, (int64_t)1) * P * 4));
    HIP_TRY(hipMemset(v->cache.p, 0, v->cache.bytes));
    *out = v.release();
    return PFM_OK;
}

int pfm_vad_set_weight(pfm_vad* v, const char* name, const void* host_ptr, int dtype, const int64_t* shape, int ndim) {
    if (!v || !name || !host_ptr || (ndim > 0 && !shape)) return fail(PFM_E_ARG, "pfm_vad_set_weight: null argument");
    if (dtype != PFM_F32) return fail(PFM_E_ARG, "pfm_vad_set_weight: weights are f32");
    auto it = v->reg.find(name);
    if (it == v->reg.end()) return fail(PFM_E_ARG, std::string("pfm_vad_set_weight: unknown key ") + name);
    auto& w = it->second;
    if ((int)w.shape.size() != ndim) return fail(PFM_E_ARG, std::string("pfm_vad_set_weight: rank of ") + name);
    for (int i = 0; i < ndim; ++i)
        if (shape[i] != w.shape[i]) return fail(PFM_E_ARG, std::string("pfm_vad_set_weight: shape of ") + name);
    HIP_TRY(hipSetDevice(v->device));
    HIP_TRY(hipMemcpy(v->arena.as<float>() + w.off, host_ptr, w.numel * 4, hipMemcpyHostToDevice));
    if (!w.set) { w.set = true; --v->missing; }
    return PFM_OK;
}

int pfm_vad_missing_weights(pfm_vad* v) { return v ? v->missing : -1; }

int pfm_vad_reset(pfm_vad* v, void* stream) {
    if (!v) return fail(PFM_E_ARG, "pfm_vad_reset: null argument");
    HIP_TRY(hipSetDevice(v->device));
    HIP_TRY(hipMemsetAsync(v->cache.p, 0, v->cache.bytes, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_vad_run(pfm_vad* v, void* stream, const float* feats, int T, float* p_sil, float* probs) {
    pfm_knobs_refresh();
    if (!v || (T > 0 && (!feats || !p_sil))) return fail(PFM_E_ARG, "pfm_vad_run: null argument");
    if (T < 0) return fail(PFM_E_ARG, "pfm_vad_run: bad T");
    if (v->missing) return fail(PFM_E_STATE, "pfm_vad_run: weights not set");
    if (T == 0) return PFM_OK;
    const pfm_vad_config& c = v->cfg;
    CHECK_DEV("pfm_vad_run", v->device, {"feats", feats}, {"p_sil", p_sil}, {"probs", probs});
    HIP_TRY(hipSetDevice(v->device));
    hipStream_t st = (hipStream_t)stream;
    if (T > v->capT) {
        HIP_TRY(hipStreamSynchronize(st));
        const size_t t = (size_t)T;
        HIP_TRY(v->h1.ensure(t * std::max(c.input_affine_dim, c.output_affine_dim) * 4));
        HIP_TRY(v->h2.ensure(t * c.linear_dim * 4));
        HIP_TRY(v->pa.ensure(t * c.proj_dim * 4));
        HIP_TRY(v->pb.ensure(t * c.proj_dim * 4));
        HIP_TRY(v->o1.ensure(t * c.linear_dim * 4));
        HIP_TRY(v->lg.ensure(t * c.output_dim * 4));
        v->capT = T;
    }
    float* h1 = v->h1.as<float>();
    float* h2 = v->h2.as<float>();
    float* pa = v->pa.as<float>();
    float* pb = v->pb.as<float>();
    float* o1 = v->o1.as<float>();
    // in_linear1 -> in_linear2 -> ReLU (encoder.py:264-266)
    HIP_TRY(pfm_vad_dense(feats, c.input_dim, T, c.input_dim, v->p("encoder.in_linear1.linear.weight"),
                          v->p("encoder.in_linear1.linear.bias"), c.input_affine_dim, 0, h1, c.input_affine_dim, st));
    HIP_TRY(pfm_vad_dense(h1, c.input_affine_dim, T, c.input_affine_dim, v->p("encoder.in_linear2.linear.weight"),
                          v->p("encoder.in_linear2.linear.bias"), c.linear_dim, 1, h2, c.linear_dim, st));
    // FSMN stack: linear (no bias) -> memory block with cache -> affine -> ReLU (BasicBlock.forward :105-117)
    const int Lm1 = std::max(c.lorder - 1, 1);
    for (int i = 0; i < c.fsmn_layers; ++i) {
        const std::string p = "encoder.fsmn." + std::to_string(i);
        HIP_TRY(pfm_vad_dense(h2, c.linear_dim, T, c.linear_dim, v->p(p + ".linear.linear.weight"), nullptr, c.proj_dim,
                              0, pa, c.proj_dim, st));
        HIP_TRY(pfm_vad_fsmn(pa, T, c.proj_dim, v->cache.as<float>() + (size_t)i * Lm1 * c.proj_dim, v->ctmp.as<float>(),
                             v->p(p + ".fsmn_block.conv_left.weight"), c.lorder, pb, st));
        HIP_TRY(pfm_vad_dense(pb, c.proj_dim, T, c.proj_dim, v->p(p + ".affine.linear.weight"),
                              v->p(p + ".affine.linear.bias"), c.linear_dim, 1, o1, c.linear_dim, st));
        std::swap(h2, o1);
    }
    // out_linear1 -> out_linear2 -> softmax (encoder.py:268-272)
    HIP_TRY(pfm_vad_dense(h2, c.linear_dim, T, c.linear_dim, v->p("encoder.out_linear1.linear.weight"),
                          v->p("encoder.out_linear1.linear.bias"), c.output_affine_dim, 0, h1, c.output_affine_dim, st));
    HIP_TRY(pfm_vad_dense(h1, c.output_affine_dim, T, c.output_affine_dim, v->p("encoder.out_linear2.linear.weight"),
                          v->p("encoder.out_linear2.linear.bias"), c.output_dim, 0, v->lg.as<float>(), c.output_dim,
                          st));
    HIP_TRY(pfm_vad_softmax(v->lg.as<float>(), T, c.output_dim, p_sil, probs, st));
    return PFM_OK;
}

int pfm_vad_frame_energy(pfm_vad* v, void* stream, const float* wav, int nsamp, int frame_len, int frame_shift,
                         float* energy) {
    if (!v || nsamp < 0 || frame_len < 1 || frame_len > 2048 || frame_shift < 1)
        return fail(PFM_E_ARG, "pfm_vad_frame_energy: bad arguments (1 <= frame_len <= 2048, frame_shift >= 1)");
    const int nf = nsamp >= frame_len ? (nsamp - frame_len) / frame_shift + 1 : 0;
    if (nf == 0) return PFM_OK;
    if (!wav || !energy) return fail(PFM_E_ARG, "pfm_vad_frame_energy: null argument");
    CHECK_DEV("pfm_vad_frame_energy", v->device, {"wav", wav}, {"energy", energy});
    HIP_TRY(hipSetDevice(v->device));
    HIP_TRY(pfm_vad_frame_energy(wav, nf, frame_len, frame_shift, energy, (hipStream_t)stream));
    return PFM_OK;
}

int pfm_vad_fbank_raw(pfm_vad* v, void* stream, const float* wav, const int32_t* nsamp, int B, int S_max, float* fb,
                      int N_cap) {
    if (!v || !wav || !nsamp || !fb) return fail(PFM_E_ARG, "pfm_vad_fbank_raw: null argument");
    if (B < 1 || S_max < 1 || N_cap < 1) return fail(PFM_E_ARG, "pfm_vad_fbank_raw: bad sizes");
    if (pfm_fbank_nframes(S_max) > N_cap) return fail(PFM_E_ARG, "pfm_vad_fbank_raw: N_cap smaller than frames of S_max");
    CHECK_DEV("pfm_vad_fbank_raw", v->device, {"wav", wav}, {"nsamp", nsamp}, {"fb", fb});
    HIP_TRY(hipSetDevice(v->device));
    if (!v->fb_ready) {
        int rc = fbank_tables_build(v->fb_tab);
        if (rc) return rc;
        v->fb_ready = true;
    }
    HIP_TRY(pfm_fbank_raw_launch(wav, nsamp, B, S_max, v->fb_tab.as<unsigned char>(), fb, N_cap, (hipStream_t)stream));
    return PFM_OK;
}

void pfm_vad_destroy(pfm_vad* v) {
    if (!v) return;
    (void)hipSetDevice(v->device);
    (void)hipDeviceSynchronize();
    delete v;
}

}  // extern "C"

