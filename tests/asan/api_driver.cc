// Drives the C-ABI of libpfm_hip (include/pfm.h) with its host code built under AddressSanitizer +
// UndefinedBehaviorSanitizer (tests/test_host_sanitize.py builds pfm_api.hip / vad_detector.hip with
// -Xarch_host -fsanitize=address,undefined and links them with the library's other objects).
//
//   api_driver cpu               argument validation of every entry point; pfm_create's config checks; the host
//                                VAD detector; no device needed (pfm_create stops at the device query)
//   api_driver gpu <model.bin>   the same, then a tiny model end to end on device 0: weight upload with the host
//                                re-layouts (Conv1d, FSMN taps), reserve, fast / exact / beam runs on a ragged
//                                batch, profiling, the ops on small device buffers, streams, teardown
//
// model.bin (written by the test): "PFMW", the pfm_config struct, then per tensor u32 name length, name, u32 ndim,
// i64 shape[ndim], f32 data. A second file <model.bin>.stream holds a streaming (dec_sanm_shift 5) model.
// Prints "ok <check>" per check; any failed expectation prints "error <check> ..." and exits 1; any sanitizer
// report aborts (-fno-sanitize-recover).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "pfm.h"

static int g_fail = 0;

static void expect(bool ok, const char* what, const std::string& detail = "") {
    if (ok) {
        printf("ok %s\n", what);
    } else {
        printf("error %s %s (last error: %s)\n", what, detail.c_str(), pfm_last_error());
        g_fail = 1;
    }
}
static void expect_rc(int rc, int want, const char* what) {
    expect(rc == want, what, "rc " + std::to_string(rc) + " want " + std::to_string(want));
    if (rc < 0) expect(pfm_last_error() && pfm_last_error()[0] != 0, "error message set");
}
// a refusal: any PFM_E_* code, with a message
static void expect_err(int rc, const char* what) {
    expect(rc < 0, what, "rc " + std::to_string(rc) + " want an error");
    if (rc < 0) expect(pfm_last_error() && pfm_last_error()[0] != 0, "error message set");
}

// ---- argument validation: every entry point refuses null / out-of-range arguments with a PFM_E_* code
static void validation() {
    pfm_config c;
    pfm_config_default(&c);
    expect(c.d_model == 512 && c.heads == 4 && c.enc_blocks == 50 && c.vocab_size == 8404, "config_default");
    pfm_config s;
    pfm_config_sensevoice(&s);
    expect(s.arch == PFM_ARCH_SENSEVOICE && s.ln_eps < 2e-5f, "config_sensevoice");
    pfm_config p;
    pfm_config_punc(&p);
    expect(p.arch == PFM_ARCH_PUNC, "config_punc");

    pfm_handle* h = nullptr;
    expect_rc(pfm_create(nullptr, 0, &h), PFM_E_ARG, "create null cfg");
    expect_rc(pfm_create(&c, 0, nullptr), PFM_E_ARG, "create null out");
    struct Bad { const char* what; void (*edit)(pfm_config&); };
    const Bad bad[] = {
        {"create heads 0", [](pfm_config& x) { x.heads = 0; }},
        {"create heads 3", [](pfm_config& x) { x.heads = 3; }},
        {"create head dim 64", [](pfm_config& x) { x.heads = 8; }},
        {"create input 561", [](pfm_config& x) { x.input_size = 561; }},
        {"create ffn 4096", [](pfm_config& x) { x.ffn = 4096; }},
        {"create enc_blocks 0", [](pfm_config& x) { x.enc_blocks = 0; }},
        {"create dec_blocks -1", [](pfm_config& x) { x.dec_blocks = -1; }},
        {"create vocab 0", [](pfm_config& x) { x.vocab_size = 0; }},
        {"create arch 7", [](pfm_config& x) { x.arch = 7; }},
        {"create cif order", [](pfm_config& x) { x.cif_l_order = 2; }},
        {"create ctc_head 2", [](pfm_config& x) { x.ctc_head = 2; }},
        {"create punc classes", [](pfm_config& x) { pfm_config_punc(&x); x.vocab_size = 100; }},
        {"create sensevoice n_embed", [](pfm_config& x) { pfm_config_sensevoice(&x); x.n_embed = 0; }},
    };
    for (const Bad& b : bad) {
        pfm_config x = c;
        b.edit(x);
        expect_rc(pfm_create(&x, 0, &h), PFM_E_ARG, b.what);
        expect(h == nullptr, "create leaves out null");
    }
    expect_err(pfm_create(&c, -1, &h), "create device -1");   // (no device here: the device query fails first)

    int64_t shp[2] = {512, 512};
    float one = 0.f;
    int32_t i1 = 1, tok[4];
    float f4[4];
    expect_err(pfm_set_weight(nullptr, "x", &one, PFM_F32, shp, 2), "set_weight null handle");
    expect_err(pfm_set_weight_device(nullptr, "x", &one, PFM_F32, shp, 2, nullptr), "set_weight_device null handle");
    expect(pfm_missing_weights(nullptr) == -1, "missing_weights null");
    expect_err(pfm_reserve(nullptr, 1, 1), "reserve null");
    expect_rc(pfm_run(nullptr, nullptr, PFM_MODE_FAST, f4, &i1, 1, 1, tok, 4, tok, nullptr, nullptr, nullptr),
              PFM_E_ARG, "run null handle");
    expect_err(pfm_run_beam(nullptr, nullptr, 0, f4, &i1, 1, 1, 4, 0.3f, 0.f, 1, 0, 1, 2, 0, tok, 4, tok, f4, nullptr,
                           nullptr), "run_beam null handle");
    expect_err(pfm_run_ctc(nullptr, nullptr, 0, f4, &i1, 1, 1, tok, -1, tok, 4, tok, nullptr, nullptr), "run_ctc null handle");
    expect_err(pfm_run_punc(nullptr, nullptr, 0, tok, &i1, 1, 1, tok, nullptr), "run_punc null handle");
    expect_err(pfm_run_punc_host(nullptr, nullptr, 0, tok, 1, tok), "run_punc_host null handle");
    expect_err(pfm_ctc_align(nullptr, nullptr, f4, 1, 5, &i1, tok, 1, &i1, 0, tok), "ctc_align null");
    expect_err(pfm_profile(nullptr, 1), "profile null");
    double d;
    int64_t n64;
    expect_err(pfm_profile_read(nullptr, 0, &d, &d, &d, &n64), "profile_read null");
    pfm_destroy(nullptr);
    expect(true, "destroy null");

    pfm_streams* st = nullptr;
    const int32_t cs[3] = {0, 10, 5};
    expect_err(pfm_streams_create(nullptr, 1, cs, 4, 1, PFM_MODE_FAST, &st), "streams_create null");
    expect_err(pfm_streams_reset(nullptr, nullptr, &i1, 1), "streams_reset null");
    expect_err(pfm_stream_step(nullptr, nullptr, 1, &i1, f4, 1, &i1, &i1, tok, 4, tok, nullptr, nullptr), "stream_step null");
    expect_err(pfm_stream_step_beam(nullptr, nullptr, 1, &i1, f4, 1, &i1, &i1, 4, 0.3f, 0.f, 1, 0, 1, 2, 0, tok, 4, tok,
                                   f4, tok), "stream_step_beam null");
    pfm_streams_destroy(nullptr);
    expect(true, "streams_destroy null");

    expect_err(pfm_fbank(nullptr, nullptr, f4, &i1, 1, 1, f4, f4, 1, tok), "fbank null");
    expect(pfm_lfr_frames(16000) == 17 && pfm_lfr_frames(1 << 26) > 0, "lfr_frames");

}

// ---- the single-op entry points: null operands and bad sizes are refused with PFM_E_ARG before any launch (a
// launch failure would be PFM_E_HIP). Host pointers stand in for device operands; every entry point also refuses a
// host address before launching (check_dev in pfm_api.hip), so this runs on the GPU too.
static void op_validation() {
    float f4[4];
    int32_t i1 = 1, tok[4];
    expect_rc(pfm_op_gemm(nullptr, PFM_F32, nullptr, f4, nullptr, nullptr, f4, 1, 1, 1, 0), PFM_E_ARG, "op_gemm null A");
    expect_rc(pfm_op_gemm(nullptr, PFM_F32, f4, f4, nullptr, nullptr, f4, -1, 1, 1, 0), PFM_E_ARG, "op_gemm M -1");
    expect_rc(pfm_op_gemm(nullptr, 9, f4, f4, nullptr, nullptr, f4, 1, 1, 1, 0), PFM_E_ARG, "op_gemm dtype");
    expect_rc(pfm_op_ln_gemm(nullptr, nullptr, f4, f4, 1e-5f, f4, nullptr, nullptr, f4, 1, 1, 0), PFM_E_ARG, "op_ln_gemm null");
    expect_rc(pfm_op_ffn(nullptr, nullptr, 1, f4, f4, 1e-5f, f4, f4, f4, f4, f4, nullptr, nullptr, nullptr), PFM_E_ARG, "op_ffn null");
    expect_rc(pfm_op_ffn_op(nullptr, nullptr, f4, f4, f4, nullptr, 1, f4, f4, 1e-5f, f4, f4, f4, f4, f4, nullptr,
                            nullptr, nullptr), PFM_E_ARG, "op_ffn_op null");
    expect_rc(pfm_op_ffn_op_qkv(nullptr, nullptr, f4, f4, f4, nullptr, 1, f4, f4, 1e-5f, f4, f4, f4, f4, f4, f4, f4,
                                f4, f4, f4), PFM_E_ARG, "op_ffn_op_qkv null");
    expect_rc(pfm_op_ffn_dec(nullptr, nullptr, 1, f4, f4, 1e-5f, f4, f4, f4, f4, f4, f4, f4, f4, f4, nullptr, nullptr,
                             nullptr), PFM_E_ARG, "op_ffn_dec null");
    expect_rc(pfm_op_attention(nullptr, PFM_F32, nullptr, f4, f4, &i1, f4, 1, 1, 1, 4, 1.f), PFM_E_ARG, "op_attention null");
    expect_rc(pfm_op_layernorm(nullptr, nullptr, f4, f4, f4, 1, 4, 1e-5f), PFM_E_ARG, "op_layernorm null");
    expect_rc(pfm_op_fsmn(nullptr, nullptr, &i1, f4, nullptr, f4, 1, 1, 4, 3, 1), PFM_E_ARG, "op_fsmn null");
    expect_rc(pfm_op_layernorm_bf16(nullptr, nullptr, f4, f4, f4, 1, 512, 1e-5f), PFM_E_ARG, "op_layernorm_bf16 null");
    expect_rc(pfm_op_fsmn_bf16(nullptr, nullptr, &i1, f4, f4, 1, 1, 4, 3, 1), PFM_E_ARG, "op_fsmn_bf16 null");
    expect_rc(pfm_op_cif(nullptr, nullptr, f4, f4, f4, tok, tok, 1, 1, 4, 4), PFM_E_ARG, "op_cif null");
    expect_rc(pfm_op_ctc_collapse(nullptr, nullptr, 4, &i1, 1, 0, tok, 4, tok), PFM_E_ARG, "op_ctc_collapse null");
    expect_rc(pfm_op_ctc_beam(nullptr, nullptr, 1, f4, 1, &i1, &i1, 1, 4, 4, 0.3f, 0.f, 1, 0, 1, 2, 0, tok, 4, tok, f4),
              PFM_E_ARG, "op_ctc_beam null");
    expect_rc(pfm_op_ctc_beam(nullptr, f4, 1, f4, 1, &i1, &i1, 1, 4, 99, 0.3f, 0.f, 1, 0, 1, 2, 0, tok, 4, tok, f4),
              PFM_E_ARG, "op_ctc_beam beam 99");

}

static void vad_validation() {
    float f4[4], one = 0.f;
    int64_t shp[2] = {512, 512};
    // VAD: the device model's entry points and the host detector
    pfm_vad_config vc;
    pfm_vad_config_default(&vc);
    pfm_vad* v = nullptr;
    expect_err(pfm_vad_create(nullptr, 0, &v), "vad_create null");
    expect_err(pfm_vad_set_weight(nullptr, "x", &one, PFM_F32, shp, 2), "vad_set_weight null");
    expect(pfm_vad_missing_weights(nullptr) == -1, "vad_missing null");
    expect_err(pfm_vad_reset(nullptr, nullptr), "vad_reset null");
    expect_err(pfm_vad_run(nullptr, nullptr, f4, 1, f4, nullptr), "vad_run null");
    expect_err(pfm_vad_frame_energy(nullptr, nullptr, f4, 4, 400, 160, f4), "vad_frame_energy null");
    pfm_vad_destroy(nullptr);
    pfm_vad_opts o;
    pfm_vad_opts_default(&o);
    pfm_vad_detector* det = nullptr;
    expect_err(pfm_vad_detector_create(nullptr, &det), "vad_detector_create null");
    expect_rc(pfm_vad_detector_create(&o, &det), PFM_OK, "vad_detector_create");
    pfm_vad_detector_destroy(det);
    pfm_vad_detector_destroy(nullptr);
}

// ---- model file
struct Tensor { std::string name; std::vector<int64_t> shape; std::vector<float> data; };
struct Model { pfm_config cfg; std::vector<Tensor> ts; };

static bool load_model(const char* path, Model& m) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    char magic[4];
    bool ok = fread(magic, 1, 4, f) == 4 && memcmp(magic, "PFMW", 4) == 0 && fread(&m.cfg, sizeof(m.cfg), 1, f) == 1;
    uint32_t n = 0;
    ok = ok && fread(&n, 4, 1, f) == 1;
    for (uint32_t i = 0; ok && i < n; ++i) {
        Tensor t;
        uint32_t len = 0, nd = 0;
        ok = fread(&len, 4, 1, f) == 1 && len < 4096;
        if (!ok) break;
        t.name.resize(len);
        ok = fread(&t.name[0], 1, len, f) == len && fread(&nd, 4, 1, f) == 1 && nd <= 8;
        if (!ok) break;
        t.shape.resize(nd);
        ok = fread(t.shape.data(), 8, nd, f) == nd;
        size_t numel = 1;
        for (int64_t s : t.shape) numel *= (size_t)s;
        t.data.resize(numel);
        ok = ok && fread(t.data.data(), 4, numel, f) == numel;
        m.ts.push_back(std::move(t));
    }
    fclose(f);
    return ok;
}

#define HCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("error hip %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <class T> static T* dev_upload(const std::vector<T>& v) {
    T* p = nullptr;
    HCK(hipMalloc(&p, std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (!v.empty()) HCK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}
template <class T> static std::vector<T> dev_download(const T* p, size_t n) {
    std::vector<T> v(n);
    HCK(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
    return v;
}

static pfm_handle* create_and_load(const Model& m, const char* tag) {
    pfm_handle* h = nullptr;
    expect_rc(pfm_create(&m.cfg, 0, &h), PFM_OK, tag);
    if (!h) return nullptr;
    expect(pfm_missing_weights(h) > 0, "missing before upload");
    int bad = 0;
    for (const Tensor& t : m.ts)
        bad += pfm_set_weight(h, t.name.c_str(), t.data.data(), PFM_F32, t.shape.data(), (int)t.shape.size()) != PFM_OK;
    expect(bad == 0, "set_weight all", std::to_string(bad) + " refused");
    expect(pfm_missing_weights(h) == 0, "missing after upload");
    // refusals after creation: unknown key, rank / shape mismatch, dtype
    const Tensor& t0 = m.ts[0];
    std::vector<int64_t> sh = t0.shape;
    expect_rc(pfm_set_weight(h, "no.such.key", t0.data.data(), PFM_F32, sh.data(), (int)sh.size()), PFM_E_NAME,
              "set_weight unknown key");
    expect_rc(pfm_set_weight(h, t0.name.c_str(), t0.data.data(), PFM_F32, sh.data(), (int)sh.size() + 1), PFM_E_ARG,
              "set_weight rank mismatch");
    sh[0] += 1;
    expect_rc(pfm_set_weight(h, t0.name.c_str(), t0.data.data(), PFM_F32, sh.data(), (int)sh.size()), PFM_E_ARG,
              "set_weight shape mismatch");
    expect_rc(pfm_set_weight(h, t0.name.c_str(), t0.data.data(), PFM_BF16, t0.shape.data(), (int)t0.shape.size()),
              PFM_E_ARG, "set_weight dtype");
    // the device-pointer upload path re-lays the same tensors out on the device
    int badd = 0;
    for (const Tensor& t : m.ts) {
        float* d = dev_upload(t.data);
        badd += pfm_set_weight_device(h, t.name.c_str(), d, PFM_F32, t.shape.data(), (int)t.shape.size(), nullptr) !=
                PFM_OK;
        HCK(hipFree(d));
    }
    expect(badd == 0, "set_weight_device all", std::to_string(badd) + " refused");
    return h;
}

// ---- host memory where the ABI wants device memory: every entry point returns PFM_E_ARG naming the operand and
// launches nothing (before round 6 such a call faulted the GPU). One host operand per call, the rest valid device
// buffers; afterwards the handle still decodes (the refused lookups leave no sticky HIP error behind).
static void expect_host_refused(int rc, const char* what, const char* operand) {
    expect_rc(rc, PFM_E_ARG, what);
    expect(strstr(pfm_last_error(), operand) != nullptr, "refusal names the operand", pfm_last_error());
}
static void host_pointer_refusals(pfm_handle* h, const Model& m, float* dfe, int32_t* dln, int32_t* dtok,
                                  int32_t* dnt, int B, int T, int L_cap) {
    const int D = m.cfg.input_size, dm = m.cfg.d_model;
    std::vector<float> hfe((size_t)B * T * D, 0.f);
    std::vector<int32_t> hln(B, T), htok((size_t)B * L_cap), hnt(B);
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_FAST, hfe.data(), dln, B, T, dtok, L_cap, dnt, nullptr, nullptr,
                                nullptr), "run host feats", "feats");
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, hln.data(), B, T, dtok, L_cap, dnt, nullptr, nullptr,
                                nullptr), "run host lens", "lens");
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, htok.data(), L_cap, dnt, nullptr, nullptr,
                                nullptr), "run host tokens", "tokens");
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_EXACT, dfe, dln, B, T, dtok, L_cap, hnt.data(), nullptr, nullptr,
                                nullptr), "run host ntok", "ntok");
    std::vector<float> henc((size_t)B * T * dm);
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, dtok, L_cap, dnt, henc.data(), nullptr,
                                nullptr), "run host enc_out", "enc_out");
    // pinned host memory is host memory too (the kernels would read it over PCIe; the ABI takes device buffers)
    float* pinned = nullptr;
    HCK(hipHostMalloc((void**)&pinned, hfe.size() * sizeof(float), 0));
    expect_host_refused(pfm_run(h, nullptr, PFM_MODE_FAST, pinned, dln, B, T, dtok, L_cap, dnt, nullptr, nullptr,
                                nullptr), "run pinned feats", "feats");
    HCK(hipHostFree(pinned));
    if (m.cfg.ctc_head) {
        std::vector<float> hsc((size_t)B * 2);
        expect_host_refused(pfm_run_beam(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, 4, 0.3f, 0.f, 2, 0, 1, 2, 0, dtok,
                                         L_cap, dnt, hsc.data(), nullptr, nullptr), "run_beam host scores", "scores");
    }
    // single ops: device buffers big enough for the shapes below, one operand on the host
    const int M = 64, N = 64, K = 64, hd = 4 * 128, Bq = 1, Tq = 8;
    std::vector<float> zf((size_t)std::max(M * K, Bq * Tq * hd), 0.f);
    std::vector<int32_t> zi(64, 1);
    float* da = dev_upload(zf);
    float* dw = dev_upload(zf);
    float* dc = dev_upload(zf);
    int32_t* di = dev_upload(zi);
    expect_host_refused(pfm_op_gemm(nullptr, PFM_F32, zf.data(), dw, nullptr, nullptr, dc, M, N, K, 0), "op_gemm host A", "'A'");
    expect_host_refused(pfm_op_gemm(nullptr, PFM_F32, da, dw, nullptr, nullptr, zf.data(), M, N, K, 0), "op_gemm host C", "'C'");
    expect_host_refused(pfm_op_attention(nullptr, PFM_F32, zf.data(), da, da, di, dc, Bq, Tq, Tq, 4, 1.f),
                        "op_attention host q", "'q'");
    expect_host_refused(pfm_op_attention(nullptr, PFM_F32, da, da, da, zi.data(), dc, Bq, Tq, Tq, 4, 1.f),
                        "op_attention host klen", "klen");
    expect_host_refused(pfm_op_layernorm(nullptr, da, dw, dw, zf.data(), 8, 64, 1e-5f), "op_layernorm host out", "out");
    expect_host_refused(pfm_op_fsmn(nullptr, zf.data(), di, dw, nullptr, dc, 1, 8, 64, 3, 1), "op_fsmn host v", "'v'");
    expect_host_refused(pfm_op_cif(nullptr, da, zf.data(), dc, dc, di, di, 1, 8, 4, 4), "op_cif host hidden", "hidden");
    expect_host_refused(pfm_op_ctc_collapse(nullptr, zi.data(), 8, di, 1, 0, di, 4, di), "op_ctc_collapse host ids", "ids");
    expect_host_refused(pfm_op_ctc_beam(nullptr, zf.data(), 2, da, 4, di, di, 1, 8, 2, 0.3f, 0.f, 1, 0, 1, 2, 0, di, 4,
                                        di, dc), "op_ctc_beam host am", "'am'");
    std::vector<int32_t> hns(1, 400);
    expect_host_refused(pfm_fbank(h, nullptr, da, hns.data(), 1, 400, nullptr, dc, 8, di), "fbank host nsamp", "nsamp");
    expect_host_refused(pfm_fbank(h, nullptr, zf.data(), di, 1, 400, nullptr, dc, 8, di), "fbank host wav", "wav");
    HCK(hipFree(da)); HCK(hipFree(dw)); HCK(hipFree(dc)); HCK(hipFree(di));
    // the handle still runs after the refusals
    expect_rc(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, dtok, L_cap, dnt, nullptr, nullptr, nullptr), PFM_OK,
              "run after host-pointer refusals");
    HCK(hipDeviceSynchronize());
}

static void offline(const Model& m) {
    pfm_handle* h = create_and_load(m, "create offline model");
    if (!h) return;
    const int B = 3, T = 41, D = m.cfg.input_size, L_cap = 24;
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> feats((size_t)B * T * D);
    for (float& x : feats) x = nd(rng);
    const std::vector<int32_t> lens = {T, 17, 1};
    float* dfe = dev_upload(feats);
    int32_t* dln = dev_upload(lens);
    int32_t *dtok, *dnt;
    float *dal, *dpk, *denc;
    HCK(hipMalloc(&dtok, (size_t)B * 16 * L_cap * 4));
    HCK(hipMalloc(&dnt, (size_t)B * 16 * 4));
    HCK(hipMalloc(&dal, (size_t)B * (T + 1) * 4));
    HCK(hipMalloc(&dpk, (size_t)B * (T + 1) * 4));
    HCK(hipMalloc(&denc, (size_t)B * T * m.cfg.d_model * 4));
    expect_rc(pfm_reserve(h, 0, T), PFM_E_ARG, "reserve B 0");
    expect_rc(pfm_reserve(h, 8, 64), PFM_OK, "reserve");
    std::vector<int32_t> first;
    for (int mode : {PFM_MODE_EXACT, PFM_MODE_FAST, PFM_MODE_EXACT}) {
        expect_rc(pfm_run(h, nullptr, mode, dfe, dln, B, T, dtok, L_cap, dnt, denc, dal, dpk), PFM_OK,
                  mode == PFM_MODE_FAST ? "run fast" : "run exact");
        HCK(hipDeviceSynchronize());
        auto nt = dev_download(dnt, B);
        auto tk = dev_download(dtok, (size_t)B * L_cap);
        bool sane = true;
        for (int b = 0; b < B; ++b) {
            sane &= nt[b] >= 0;
            for (int l = 0; l < L_cap; ++l) {
                const int t = tk[(size_t)b * L_cap + l];
                sane &= l < std::min(nt[b], L_cap) ? (t >= 0 && t < m.cfg.vocab_size) : t == -1;
            }
        }
        expect(sane, "run outputs in range");
        if (mode == PFM_MODE_EXACT) {
            if (first.empty()) first = tk;
            else expect(first == tk, "exact run deterministic");
        }
    }
    // bad calls on a live handle
    expect_rc(pfm_run(h, nullptr, 5, dfe, dln, B, T, dtok, L_cap, dnt, nullptr, nullptr, nullptr), PFM_E_ARG,
              "run bad mode");
    expect_rc(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, 0, T, dtok, L_cap, dnt, nullptr, nullptr, nullptr),
              PFM_E_ARG, "run B 0");
    expect_rc(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, dtok, -1, dnt, nullptr, nullptr, nullptr), PFM_E_ARG,
              "run L_cap -1");
    // growth past the reservation (B 5 x T 90): the workspace is re-sized on demand
    {
        const int B2 = 5, T2 = 90;
        std::vector<float> f2((size_t)B2 * T2 * D);
        for (float& x : f2) x = nd(rng);
        std::vector<int32_t> l2 = {T2, 3, 45, 90, 2};
        float* d2 = dev_upload(f2);
        int32_t* dl2 = dev_upload(l2);
        int32_t *t2, *n2;
        HCK(hipMalloc(&t2, (size_t)B2 * L_cap * 4));
        HCK(hipMalloc(&n2, B2 * 4));
        expect_rc(pfm_run(h, nullptr, PFM_MODE_FAST, d2, dl2, B2, T2, t2, L_cap, n2, nullptr, nullptr, nullptr), PFM_OK,
                  "run beyond reservation");
        HCK(hipFree(d2)); HCK(hipFree(dl2)); HCK(hipFree(t2)); HCK(hipFree(n2));
    }
    if (m.cfg.ctc_head) {
        const int nbest = 2;
        float* dsc;
        HCK(hipMalloc(&dsc, (size_t)B * nbest * 4));
        for (int mode : {PFM_MODE_EXACT, PFM_MODE_FAST})
            expect_rc(pfm_run_beam(h, nullptr, mode, dfe, dln, B, T, 4, 0.3f, 0.f, nbest, 0, 1, 2, 0, dtok, L_cap, dnt,
                                   dsc, dal, dpk), PFM_OK, "run_beam");
        expect_rc(pfm_run_beam(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, 0, 0.3f, 0.f, nbest, 0, 1, 2, 0, dtok, L_cap,
                               dnt, dsc, nullptr, nullptr), PFM_E_ARG, "run_beam beam 0");
        auto nt = dev_download(dnt, (size_t)B * nbest);
        bool sane = true;
        for (int x : nt) sane &= x >= -1;
        expect(sane, "run_beam counts");
        HCK(hipFree(dsc));
    }
    host_pointer_refusals(h, m, dfe, dln, dtok, dnt, B, T, L_cap);
    expect_rc(pfm_profile(h, 1), PFM_OK, "profile on");
    expect_rc(pfm_run(h, nullptr, PFM_MODE_FAST, dfe, dln, B, T, dtok, L_cap, dnt, nullptr, nullptr, nullptr), PFM_OK,
              "run profiled");
    double ms = 0, fl = 0, by = 0;
    int64_t nl = 0;
    expect_rc(pfm_profile_read(h, 0, &ms, &fl, &by, &nl), PFM_OK, "profile_read");
    expect_rc(pfm_profile_read(h, 99, &ms, &fl, &by, &nl), PFM_E_ARG, "profile_read bad class");
    expect_rc(pfm_profile(h, 0), PFM_OK, "profile off");
    HCK(hipFree(dfe)); HCK(hipFree(dln)); HCK(hipFree(dtok)); HCK(hipFree(dnt));
    HCK(hipFree(dal)); HCK(hipFree(dpk)); HCK(hipFree(denc));
    pfm_destroy(h);
    expect(true, "destroy offline");
}

static void streaming(const Model& m) {
    pfm_handle* h = create_and_load(m, "create streaming model");
    if (!h) return;
    const int32_t cs[3] = {0, 10, 5};
    pfm_streams* s = nullptr;
    expect_rc(pfm_streams_create(h, 2, cs, -1, 1, PFM_MODE_FAST, &s), PFM_E_ARG, "streams_create look_back -1");
    expect_rc(pfm_streams_create(h, 2, cs, 4, 1, PFM_MODE_EXACT, &s), PFM_OK, "streams_create");
    if (!s) { pfm_destroy(h); return; }
    const int n = 2, Tn = 10, D = m.cfg.input_size, L_cap = 16;
    std::mt19937 rng(11);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> f((size_t)n * Tn * D);
    int32_t *dtok, *dnt;
    HCK(hipMalloc(&dtok, (size_t)n * 4 * L_cap * 4));
    HCK(hipMalloc(&dnt, (size_t)n * 4 * 4));
    float* dsc;
    HCK(hipMalloc(&dsc, (size_t)n * 4 * 4));
    const int32_t slots[2] = {0, 1};
    for (int chunk = 0; chunk < 4; ++chunk) {
        for (float& x : f) x = nd(rng);
        float* df = dev_upload(f);
        const int32_t nfeat[2] = {Tn, chunk == 3 ? 0 : 7};
        const int32_t fin[2] = {chunk == 3, chunk == 3};
        expect_rc(pfm_stream_step(s, nullptr, n, slots, df, Tn, nfeat, fin, dtok, L_cap, dnt, nullptr, nullptr), PFM_OK,
                  "stream_step");
        HCK(hipFree(df));
    }
    {
        const int32_t nfeat[2] = {Tn, Tn};
        const int32_t fin[2] = {0, 0};
        expect_host_refused(pfm_stream_step(s, nullptr, n, slots, f.data(), Tn, nfeat, fin, dtok, L_cap, dnt, nullptr,
                                            nullptr), "stream_step host feats", "feats");
    }
    const int32_t dup[2] = {1, 1};
    expect_rc(pfm_streams_reset(s, nullptr, slots, 2), PFM_OK, "streams_reset");
    const int32_t three[3] = {0, 1, 5};
    expect_rc(pfm_streams_reset(s, nullptr, three, 3), PFM_E_ARG, "streams_reset bad slot id");
    {
        float* df = dev_upload(f);
        const int32_t nfeat[2] = {Tn, Tn};
        const int32_t fin[2] = {0, 0};
        expect_rc(pfm_stream_step(s, nullptr, n, dup, df, Tn, nfeat, fin, dtok, L_cap, dnt, nullptr, nullptr),
                  PFM_E_ARG, "stream_step duplicate slot");
        if (m.cfg.ctc_head)
            expect_rc(pfm_stream_step_beam(s, nullptr, n, slots, df, Tn, nfeat, fin, 4, 0.3f, 0.f, 2, 0, 1, 2, 0,
                                           dtok, L_cap, dnt, dsc, nullptr), PFM_OK, "stream_step_beam");
        HCK(hipFree(df));
    }
    pfm_streams_destroy(s);
    HCK(hipFree(dtok)); HCK(hipFree(dnt)); HCK(hipFree(dsc));
    pfm_destroy(h);
    expect(true, "destroy streaming");
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: api_driver cpu | gpu model.bin\n");
        return 2;
    }
    validation();
    vad_validation();
    op_validation();
    if (!strcmp(argv[1], "gpu")) {
        if (argc < 3) return 2;
        Model m, ms;
        expect(load_model(argv[2], m), "load model file");
        if (!m.ts.empty()) offline(m);
        const std::string sp = std::string(argv[2]) + ".stream";
        if (load_model(sp.c_str(), ms) && !ms.ts.empty()) streaming(ms);
    }
    printf(g_fail ? "FAILED\n" : "PASSED\n");
    return g_fail;
}
