/*
 * pfm.h — C ABI of libpfm_hip.so, the MI355X (gfx950) Paraformer inference path.
 *
 * This is the drop-in boundary for the hot path of funasr.auto.AutoModel.generate():
 * everything under Paraformer.inference (funasr/models/paraformer/model.py:443-596) from the
 * fbank tensor to the per-utterance argmax token ids runs behind these entry points. The
 * host side (funasr_amd/, Python) keeps AutoModel's input handling, batching, tokenizer and
 * result-dict contract. Plain C types only: pointers, sizes, status codes.
 *
 * Conventions
 *  - Return 0 (PFM_OK) on success, a negative PFM_E_* code on failure; pfm_last_error()
 *    returns a thread-local message for the last failing call on this thread. No C++
 *    exception crosses the ABI.
 *  - All tensor arguments of pfm_run / pfm_fbank / pfm_op_* are caller-owned DEVICE
 *    memory on the handle's device, row-major, and are consumed/produced in order on the
 *    caller's `stream` (a hipStream_t; NULL = default stream).
 *  - A handle owns its weights and workspace; it is not re-entrant (one call at a time per
 *    handle); distinct handles may be used from distinct threads. One handle per device.
 */
#ifndef PFM_H_
#define PFM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFM_ABI_VERSION 5

enum pfm_status {
    PFM_OK = 0,
    PFM_E_ARG = -1,      /* bad argument / shape */
    PFM_E_HIP = -2,      /* HIP runtime error */
    PFM_E_STATE = -3,    /* call out of order (e.g. run before all weights set) */
    PFM_E_NOMEM = -4,    /* device allocation failed */
    PFM_E_NAME = -5,     /* unknown weight name */
    PFM_E_DEVICE = -6    /* device-side failure reported by a kernel (e.g. the beam search's cross-workgroup
                            arrival barrier timed out): the outputs of the call are not valid */
};

enum pfm_dtype { PFM_F32 = 0, PFM_BF16 = 1 };

/* Numerics mode of pfm_run.
 *  EXACT: every GEMM and the attention as split-bf16 x6 MFMA (each f32 operand split into
 *         three bf16 planes x = x0+x1+x2, the six products above 2^-24 relative summed in
 *         f32 — f32-equivalent contractions; PFM_EXACT_X6=0 selects v_mfma_f32_32x32x2_f32),
 *         softmax / LayerNorm / CIF in f32 (f64 reductions) — the token-ID parity mode.
 *  FAST : bf16 MFMA operands with f32 accumulation; f32 residual stream, LayerNorm,
 *         softmax statistics and CIF — the throughput mode.                              */
enum pfm_mode { PFM_MODE_EXACT = 0, PFM_MODE_FAST = 1 };

/* Model family of a handle.
 *  PARAFORMER : SAN-M encoder + CIF predictor + SAN-M NAR decoder (funasr/models/paraformer/model.py)
 *  SENSEVOICE : SenseVoiceSmall — 4 query rows + SAN-M encoder + tp encoder + CTC head
 *               (funasr/models/sense_voice/model.py:445-950); decoder / predictor fields ignored */
enum pfm_arch { PFM_ARCH_PARAFORMER = 0, PFM_ARCH_SENSEVOICE = 1, PFM_ARCH_PUNC = 2 };

/* Model dimensions; mirrors encoder_conf / decoder_conf / predictor_conf of
 * funasr/models/paraformer/template.yaml:8-66 (Paraformer-large defaults via
 * pfm_config_default; SenseVoiceSmall via pfm_config_sensevoice). */
typedef struct pfm_config {
    int32_t input_size;      /* 560 = 80 mel x lfr_m 7 */
    int32_t d_model;         /* 512 */
    int32_t heads;           /* 4 (d_k must be 128) */
    int32_t ffn;             /* 2048 */
    int32_t enc_blocks;      /* 50 (encoders0 + 49 encoders) */
    int32_t dec_blocks;      /* 16 (att_layer_num == num_blocks) */
    int32_t kernel_size;     /* 11, FSMN depthwise kernel */
    int32_t enc_sanm_shift;  /* 0 */
    int32_t dec_sanm_shift;  /* 0 */
    int32_t vocab_size;      /* 8404 */
    int32_t cif_l_order;     /* 1 */
    int32_t cif_r_order;     /* 1 */
    float cif_threshold;     /* 1.0 */
    float tail_threshold;    /* 0.45 */
    float smooth_factor;     /* 1.0 */
    float noise_threshold;   /* 0.0 */
    float ln_eps;            /* 1e-12 (Paraformer, transformer/layer_norm.py:24); 1e-5 (SenseVoice) */
    int32_t arch;            /* pfm_arch */
    int32_t tp_blocks;       /* SenseVoice: 20 tp_encoders (sense_voice/model.py:529-540) */
    int32_t n_embed;         /* SenseVoice: 16 rows of the query Embedding (model.py:646-648) */
    int32_t ctc_head;        /* Paraformer: 1 = the model carries ctc.ctc_lo (trained with ctc_weight > 0,
                                paraformer/model.py:95-100, 147-150), needed by pfm_run_beam; else 0 */
} pfm_config;

typedef struct pfm_handle pfm_handle;

/* Paraformer-large defaults. */
void pfm_config_default(pfm_config* cfg);

/* SenseVoiceSmall defaults: d 512, 4 heads, FFN 2048, 50 + 20 blocks, vocab 25055, eps 1e-5. */
void pfm_config_sensevoice(pfm_config* cfg);

/* Create a handle on HIP device `device`. Replaces the model construction of
 * AutoModel.build_model (funasr/auto/auto_model.py:176-293). */
int pfm_create(const pfm_config* cfg, int device, pfm_handle** out);

/* Upload one parameter, addressed by its reference state_dict key
 * (e.g. "encoder.encoders.3.self_attn.linear_q_k_v.weight") with its
 * reference shape. `host_ptr` is host memory of `dtype` (PFM_F32). Replaces
 * load_pretrained_model (funasr/train_utils/load_pretrained_model.py:14-47).
 * Keys that are unused at inference (decoder.embed.0.weight) are accepted and ignored. */
int pfm_set_weight(pfm_handle* h, const char* name, const void* host_ptr, int dtype,
                   const int64_t* shape, int ndim);

/* Same contract as pfm_set_weight with the tensor already in device memory of the handle's GPU
 * (e.g. a slice of the flat buffer a data-parallel rank received by RCCL broadcast, so the weights
 * never round-trip through the host). Copies on `stream` (a hipStream_t; NULL = default stream) and
 * returns after the copy completed, so the caller may reuse its buffer. */
int pfm_set_weight_device(pfm_handle* h, const char* name, const void* dev_ptr, int dtype,
                          const int64_t* shape, int ndim, void* stream);

/* Number of required weights still missing (0 when pfm_run may be called). */
int pfm_missing_weights(const pfm_handle* h);

/* Pre-size the workspace for batches up to B utterances of up to T LFR frames
 * (pfm_run grows it on demand otherwise; growing is not stream-capturable). */
int pfm_reserve(pfm_handle* h, int B, int T);

/* Paraformer inference on an fbank batch — the body of Paraformer.inference for
 * data_type="fbank" (paraformer/model.py:464-565): SAN-M encoder, CIF predictor, SAN-M
 * decoder and the greedy argmax.
 *   feats   [B, T, input_size] f32, frames t >= lens[b] ignored (padding)
 *   lens    [B] int32 valid LFR frames per utterance (1..T)
 *   tokens  [B, L_cap] int32 out: argmax token id of decoder position l < ntok[b]
 *           (blank/sos/eos NOT removed; -1 beyond ntok[b] or when ntok[b] > L_cap)
 *   ntok    [B] int32 out: predicted token count round(token_num) (model.py:513)
 * Optional outputs (NULL to skip):
 *   enc_out [B, T, d_model] f32 encoder output (after after_norm)
 *   alphas  [B, T+1] f32 CIF weights after tail processing (cif_predictor.py:346-370)
 *   peaks   [B, T+1] f32 CIF fire values (cif_peak)
 * The call synchronises `stream` once (to read max(ntok), which sizes the decoder). */
int pfm_run(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens,
            int B, int T, int32_t* tokens, int L_cap, int32_t* ntok, float* enc_out,
            float* alphas, float* peaks);

/* Paraformer inference with the joint decoder + CTC prefix beam search — Paraformer.inference with
 * decoding_ctc_weight > 0 (paraformer/model.py:396-441, 530-565): BeamSearchPara
 * (paraformer/search.py:35-451) over the decoder log-probs with the CTCPrefixScorer
 * (transformer/scorers/ctc.py:10-80, ctc_prefix_score.py:255-337) and the LengthBonus scorer, pre-beam
 * int(1.5 beam) candidates, end detection (metrics/common.py:18-46) when end_detect != 0
 * (maxlenratio == 0). Handle: Paraformer with ctc_head = 1. Runs the encoder / CIF / decoder of pfm_run,
 * then the CTC head, both log_softmaxes and the search itself on the device (one workgroup per utterance).
 *   beam 1..16, nbest 1..16 (the reference returns sorted(ended_hyps)[:nbest], which may hold more than beam
 *   hypotheses), ctc_weight > 1e-5 (weights["ctc"]), penalty (weights["length_bonus"]),
 *   sos / eos / blank ids of the model (blank is also the CTC blank)
 *   tokens    [B, nbest, L_cap] int32 out: token ids of the n-th best ended hypothesis, sos / eos / blank
 *             removed (model.py:553-565)
 *   ntok_out  [B, nbest] int32 out: number of those ids (may exceed L_cap: truncated), -1 = no hypothesis
 *   scores_out[B, nbest] f32 out: the hypothesis score
 * Optional outputs (NULL to skip; ABI 4): alphas / peaks [B, T+1] f32, the CIF weights and fire values of the same
 * encoder pass (pfm_run's; what pred_timestamp needs, model.py:572-582).
 * Device scratch (held by the handle, grown on demand): per utterance the CTC log-probs transposed frame-contiguous
 * (V x T floats) plus the search state (~ 7 T beam P floats), i.e. about 4 B x B x V x T in total — 2.1 GB at B = 64,
 * T = 1000, V = 8404; an allocation failure returns PFM_E_HIP before any launch.
 * The call synchronises `stream`. */
int pfm_run_beam(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens, int B, int T,
                 int beam, float ctc_weight, float penalty, int nbest, int end_detect, int sos, int eos, int blank,
                 int32_t* tokens, int L_cap, int32_t* ntok_out, float* scores_out, float* alphas, float* peaks);

/* SenseVoiceSmall inference on an fbank batch — SenseVoiceSmall.inference for
 * data_type="fbank" (sense_voice/model.py:809-906) up to token_int: query rows, encoder,
 * tp encoder, ctc_lo, per-frame argmax (log_softmax is monotone), unique_consecutive and
 * blank removal. Handle must be PFM_ARCH_SENSEVOICE.
 *   feats   [B, T, input_size] f32; lens [B] int32 valid frames (1..T)
 *   query   4 HOST int32: embed rows [language, event, emotion, textnorm] prepended to every
 *           utterance (lid_dict / 1 / 2 / textnorm_dict of model.py:638-656)
 *   ban_token  vocabulary id excluded from the argmax (ban_emo_unk: 25009) or -1
 *   tokens  [B, L_cap] int32 out: collapsed CTC token ids (blank removed), -1 beyond ntok[b]
 *   ntok    [B] int32 out: tokens per utterance (may exceed L_cap: then tokens is truncated)
 * Optional outputs (NULL to skip):
 *   enc_out    [B, T+4, d_model] f32 encoder output (after tp_norm)
 *   frame_ids  [B, T+4] int32 per-frame argmax (-1 beyond lens[b] + 4)
 * No host synchronisation. */
int pfm_run_ctc(pfm_handle* h, void* stream, int mode, const float* feats, const int32_t* lens,
                int B, int T, const int32_t* query, int ban_token, int32_t* tokens, int L_cap,
                int32_t* ntok, float* enc_out, int32_t* frame_ids);

/* SenseVoice timestamps — the CTC forced alignment of SenseVoiceSmall.inference(output_timestamp=True)
 * (sense_voice/model.py:917-928, ctc_forced_align of sense_voice/utils/ctc_alignment.py:2-60): the CTC head's
 * softmax over each utterance's speech frames (rows 4 .. olens[b]-1 of enc), blank probability zeroed where the
 * blank is the frame's argmax, Viterbi over [blank, y1, blank, ..., yL, blank] summing those probabilities in
 * f32, back-pointers from the better of the last label / final blank. Handle: PFM_ARCH_SENSEVOICE.
 *   enc      [B, Tq, d_model] f32 device: pfm_run_ctc's enc_out (Tq = T + 4)
 *   olens    [B] int32 device: encoder_out_lens (lens + 4)
 *   targets  [B, Lmax] int32 device: token_int[4:] of each utterance; tlens [B] int32 device (0..Lmax)
 *   align    [B, Tq - 4] int32 out: label id of each speech frame's state (-1 beyond olens[b] - 4)
 * Lmax <= 8190. Synchronises `stream`. */
int pfm_ctc_align(pfm_handle* h, void* stream, const float* enc, int B, int Tq, const int32_t* olens,
                  const int32_t* targets, int Lmax, const int32_t* tlens, int blank, int32_t* align);

/* ---- CT-Transformer punctuation (PFM_ARCH_PUNC; funasr/models/ct_transformer/model.py:81-93) ----
 * Config: input_size = embed_unit, d_model = att_unit, heads (head width 32 or 64), ffn, enc_blocks,
 * kernel_size, vocab_size = number of punctuation classes (<= 64), n_embed = word vocabulary rows,
 * ln_eps. Weights: "embed.weight" [n_embed, input_size], the SANMEncoder keys "encoder.*",
 * "decoder.weight" [vocab_size, d_model], "decoder.bias". */
void pfm_config_punc(pfm_config* c);   /* the released punc_ct-transformer (vocab 272727, 4 x 256-wide) */

/* punc_forward + topk(1) for B word sequences (the reference runs one mini-sentence at a time):
 *   ids    [B, T] int32 device word ids; lens [B] int32 device
 *   punc   [B, T] int32 out: argmax punctuation class per word (-1 beyond lens)
 *   logits optional [B, T, vocab_size] f32 out (NULL to skip) */
int pfm_run_punc(pfm_handle* h, void* stream, int mode, const int32_t* ids, const int32_t* lens, int B, int T,
                 int32_t* punc, float* logits);

/* One mini-sentence with HOST word ids [n] in and HOST labels [n] out (CTTransformer.punc_forward as the text loop
 * calls it, model.py:277-316): the ids go to the handle's device buffers through pinned staging, pfm_run_punc runs,
 * the labels come back; synchronises `stream`. */
int pfm_run_punc_host(pfm_handle* h, void* stream, int mode, const int32_t* ids, int n, int32_t* punc);

/* ---- FSMN-VAD (fsmn_vad_streaming/encoder.py:200-279; model.py:350-360 ComputeScores) ----
 * One pfm_vad object = the FSMN encoder of one stream with its per-layer memory caches in HBM
 * (cache["encoder"]); the VAD state machine (model.py:493-916) runs on the host over the posteriors. */
typedef struct pfm_vad pfm_vad;
typedef struct pfm_vad_config {
    int32_t input_dim, input_affine_dim, fsmn_layers, linear_dim, proj_dim, lorder, output_affine_dim, output_dim;
} pfm_vad_config;
void pfm_vad_config_default(pfm_vad_config* c);   /* the released fsmn-vad: 400/140/4/250/128/20/140/248 */
int pfm_vad_create(const pfm_vad_config* c, int device, pfm_vad** out);
/* reference state_dict keys ("encoder.in_linear1.linear.weight", ...), f32 host data */
int pfm_vad_set_weight(pfm_vad* v, const char* name, const void* host_ptr, int dtype, const int64_t* shape, int ndim);
int pfm_vad_missing_weights(pfm_vad* v);
/* zero the FSMN caches: a new stream (init_cache) */
int pfm_vad_reset(pfm_vad* v, void* stream);
/* One chunk: feats [T, input_dim] f32 device (WavFrontendOnline LFR rows) -> p_sil [T] f32 device (softmax
 * posterior of pdf 0), probs optional [T, output_dim] (NULL to skip). The caches advance by the chunk. */
int pfm_vad_run(pfm_vad* v, void* stream, const float* feats, int T, float* p_sil, float* probs);
/* The VAD detection state machine (E2EVadModel, fsmn_vad_streaming/model.py:303-916): host code over the
 * per-frame silence posteriors (pfm_vad_run) and frame decibels; one detector per stream (init_cache).
 * Options: VADXOptions (model.py:49-117) used by the decision loop. */
typedef struct pfm_vad_opts {
    int32_t detect_mode, max_end_silence_time, max_start_silence_time, window_size_ms, sil_to_speech_time_thres,
        speech_to_sil_time_thres, do_extend, lookback_time_start_point, lookahead_time_end_point,
        max_single_segment_time, noise_frame_num_used_for_snr, frame_in_ms;
    double speech_2_noise_ratio, snr_thres, decibel_thres, speech_noise_thres, fe_prior_thres;
} pfm_vad_opts;
typedef struct pfm_vad_detector pfm_vad_detector;
void pfm_vad_opts_default(pfm_vad_opts* o);
int pfm_vad_detector_create(const pfm_vad_opts* o, pfm_vad_detector** out);
/* One forward() call (model.py:548-613): append the call's frame decibels (HOST f64, ComputeDecibel) and n
 * posteriors (HOST f32), run DetectCommonFrames / DetectLastFrames (is_final) over the n new frames and
 * write the segments this call outputs: segs [cap][2] HOST int32 ([beg_ms, end_ms]; -1 for an open end or
 * start when streaming), n_segs = their number (an error if > cap). No GPU work. */
int pfm_vad_detector_push(pfm_vad_detector* d, const double* decibel, int n_db, const float* p_sil, int n,
                          int is_final, int streaming, int32_t* segs, int cap, int32_t* n_segs);
void pfm_vad_detector_destroy(pfm_vad_detector* d);

/* ComputeDecibel's frame energies (fsmn_vad_streaming/model.py:326-348) of one waveform chunk: energy[f] =
 * sum_i wav[f * frame_shift + i]^2 over frame_len samples, f < (nsamp - frame_len) / frame_shift + 1, in float32 with
 * numpy's pairwise summation order (the values the reference's np.sum gives, bit for bit); the caller takes
 * 10 log10(energy + 1e-6). wav [nsamp] f32 device, energy [frames] f32 device out. frame_len <= 2048. */
int pfm_vad_frame_energy(pfm_vad* v, void* stream, const float* wav, int nsamp, int frame_len, int frame_shift,
                         float* energy);

/* pfm_fbank_raw on the VAD object (its online frontend runs without a model handle). */
int pfm_vad_fbank_raw(pfm_vad* v, void* stream, const float* wav, const int32_t* nsamp, int B, int S_max,
                      float* fb, int N_cap);
void pfm_vad_destroy(pfm_vad* v);

/* ---- Streaming Paraformer (ParaformerStreaming, paraformer_streaming/model.py:435-656) ----
 * A pfm_streams object holds `slots` independent streams whose chunk caches live in HBM:
 * the encoder input overlap (cache["encoder"]["feats"]), the per-layer encoder K/V look-back
 * cache (encoder_chunk_look_back), the CIF carry (cif_hidden / cif_alphas), the decoder FSMN
 * caches (decode_fsmn) and the decoder cross-attention K/V cache (decoder_chunk_look_back).
 * One pfm_stream_step advances any subset of slots by one chunk in a single batched pass —
 * the reference's generate_chunk (model.py:468-554) applied to each listed stream.
 * The handle must be a Paraformer whose config has dec_sanm_shift 5 (causal decoder FSMN).
 *   chunk_size      3 host ints [0, 10, 5] (chunk_size kwarg); chunk_size[0] + chunk_size[2]
 *                   rows of overlap, alphas beyond chunk_size[0] + chunk_size[1] masked
 *   enc_look_back   encoder_chunk_look_back >= 0 (-1, unbounded, is rejected)
 *   dec_look_back   decoder_chunk_look_back >= 0
 *   mode            PFM_MODE_EXACT / PFM_MODE_FAST for every step of this object
 * Replaces init_cache (model.py:435-466). */
typedef struct pfm_streams pfm_streams;
int pfm_streams_create(pfm_handle* h, int slots, const int32_t* chunk_size, int enc_look_back,
                       int dec_look_back, int mode, pfm_streams** out);

/* Reset slots to the init_cache state (zero caches, start_idx 0). slot_ids: n HOST ints. */
int pfm_streams_reset(pfm_streams* s, void* stream, const int32_t* slot_ids, int n);

/* One chunk for n streams (generate_chunk, greedy path):
 *   slot_ids  n HOST ints, distinct
 *   feats     [n, Tn, input_size] f32 device: the chunk's LFR+CMVN rows (WavFrontendOnline output)
 *   nfeat     n HOST ints, rows of feats per stream (<= Tn); 0 = the tail chunk (model.py:601-607:
 *             final call with < 960 samples; the encoder sees the cached overlap only)
 *   is_final  n HOST ints
 *   tokens    [n, L_cap] int32 out: argmax ids of the chunk's decoder rows (blank/sos/eos NOT
 *             removed), -1 beyond ntok
 *   ntok      [n] int32 out: CIF fires this chunk (0: the decoder did not run for that stream)
 * Optional (NULL to skip): enc_out [n, 5 + max(nfeat), d_model] f32 encoder window after
 * after_norm (rows >= window length zero); alphas [n, 5 + max(nfeat)] f32 chunk-masked CIF weights.
 * The step runs on the object's own HIP stream, ordered after the work already queued on `stream` (the
 * chunk rows), and returns with its outputs complete (the host needs max(ntok) to size the decoder).
 * Repeated shapes replay HIP graphs of the step's launch sequences when enc_out and alphas are NULL
 * (PFM_STREAM_GRAPH=0 disables). */
int pfm_stream_step(pfm_streams* s, void* stream, int n, const int32_t* slot_ids, const float* feats,
                    int Tn, const int32_t* nfeat, const int32_t* is_final, int32_t* tokens, int L_cap,
                    int32_t* ntok, float* enc_out, float* alphas);

/* One chunk for n streams with the joint decoder + CTC prefix beam search instead of the argmax: the
 * generate_chunk path of a ParaformerStreaming whose model has a CTC head (model_conf ctc_weight > 0)
 * decoding with decoding_ctc_weight > 0 (paraformer_streaming/model.py:510-521, beam search built by
 * Paraformer.init_beam_search, paraformer/model.py:396-441, per chunk as inference() at :567-575).
 * Per stream: BeamSearchPara over the chunk's decoder log-probs (its CIF fires) and the CTC log-probs
 * of its whole encoder window (encoder_out[i, :encoder_out_lens[i]], overlap + chunk rows).
 *   slot_ids .. is_final   as pfm_stream_step
 *   beam, ctc_weight, penalty, nbest, end_detect, sos, eos, blank   as pfm_run_beam
 *   tokens    [n, nbest, L_cap] int32 out: hypothesis tokens without sos / eos / blank
 *   ntok      [n, nbest] int32 out: tokens per hypothesis, -1 = none (the stream fired no token this
 *             chunk: the reference's generate_chunk returns [] for it)
 *   scores    [n, nbest] f32 out
 *   nfire     [n] int32 out (or NULL): CIF fires of the chunk
 * The stream caches advance exactly as in pfm_stream_step. Synchronous like pfm_stream_step. */
int pfm_stream_step_beam(pfm_streams* s, void* stream, int n, const int32_t* slot_ids, const float* feats,
                         int Tn, const int32_t* nfeat, const int32_t* is_final, int beam, float ctc_weight,
                         float penalty, int nbest, int end_detect, int sos, int eos, int blank,
                         int32_t* tokens, int L_cap, int32_t* ntok, float* scores, int32_t* nfire);

void pfm_streams_destroy(pfm_streams* s);

/* Kaldi fbank (80 mel, 25/10 ms, hamming, dither 0, snip_edges) -> LFR (7, 6) -> CMVN for a
 * batch of waveforms: WavFrontend.forward (funasr/frontends/wav_frontend.py:118-158).
 *   wav     [B, S_max] f32 samples in [-1, 1) (scaled by 32768 inside, upsacle_samples)
 *   nsamp   [B] int32 samples per utterance
 *   cmvn    [2, 560] f32 (AddShift row, Rescale row) as parsed by load_cmvn, or NULL
 *   feats   [B, T_cap, 560] f32 out, zero-padded;  T_out [B] int32 out: LFR frames
 * Requires d_model-independent state only; h may be any handle on the device. */
int pfm_fbank(pfm_handle* h, void* stream, const float* wav, const int32_t* nsamp, int B,
              int S_max, const float* cmvn, float* feats, int T_cap, int32_t* T_out);

/* Raw Kaldi fbank frames (no LFR / CMVN) for a batch of sample runs: the kaldi.fbank call of
 * WavFrontendOnline.forward_fbank (funasr/frontends/wav_frontend.py:336-364), which the online
 * frontend feeds with the samples it carries between chunks.
 *   wav [B, S_max] f32 in [-1, 1); nsamp [B] int32 device; fb [B, N_cap, 80] f32 out (rows beyond
 *   a run's frame count are zero); N_cap >= frames of S_max. */
int pfm_fbank_raw(pfm_handle* h, void* stream, const float* wav, const int32_t* nsamp, int B, int S_max,
                  float* fb, int N_cap);

/* Online LFR + CMVN (WavFrontendOnline.apply_lfr / apply_cmvn, wav_frontend.py:275-328): out row r
 * = concat_j frames[idx[r*m + j]] (j < m), then (x + shift) * scale when cmvn != NULL.
 *   frames [F, 80] f32 device; idx [rows * m] int32 device (host-computed from the splice cache and
 *   frame counts); cmvn [2, m*80] f32 device or NULL; out [rows, m*80] f32 device. */
int pfm_lfr_gather(void* stream, const float* frames, const int32_t* idx, int rows, int m,
                   const float* cmvn, float* out);

/* Host-side frame count helper: LFR frames for n samples (ceil(nfbank / 6)). */
int pfm_lfr_frames(int nsamp);

/* Thread-local message of the last error on this thread ("" if none). */
const char* pfm_last_error(void);

void pfm_destroy(pfm_handle* h);

/* ---- live kernel timing (bench / roofline) ----
 * pfm_profile(h, 1) resets and enables HIP-event bracketing of every launch pfm_run makes on
 * its stream; pfm_profile_read sums, per kernel class (0 = MFMA GEMM, 1 = attention,
 * 2 = everything else), the event-measured milliseconds, the ALGORITHMIC flops and bytes of
 * those launches and their count. Reading synchronises the recorded events. */
enum pfm_kclass { PFM_K_GEMM = 0, PFM_K_ATTN = 1, PFM_K_OTHER = 2,
                  PFM_K_FFN2 = 3 /* the dominant kernel alone: the encoder's fused layer launch (ffn2_kernel<4>:
                                    out-proj + LN2-FFN + LN1 + next QKV), also counted in PFM_K_GEMM */ };
int pfm_profile(pfm_handle* h, int enable);
int pfm_profile_read(pfm_handle* h, int kclass, double* ms, double* flops, double* bytes,
                     int64_t* launches);

/* ---- single-op entry points (kernel-level parity tests; same kernels pfm_run uses) ---- */

/* C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ res), dtype of A/W = PFM_F32 or PFM_BF16.
 * act bit 0: relu; act bit 1: C is bf16 (bf16 operands only; the fast-mode QKV / FFN1 output
 * form), otherwise C is f32; act bit 2: W is two bf16 planes [2][N][K], w = w0 + w1 (fast mode's split-weight
 * projections, PFM_FAST_XW; K % 64 == 0). */
int pfm_op_gemm(void* stream, int dtype, const void* A, const void* W, const float* bias,
                const float* res, float* C, int M, int N, int K, int act);

/* C[M,N] = act(bf16(LayerNorm(X) g + b) . W[N,512]^T + bias) (+ res) for f32 rows X [M, 512], W bf16: the fast-mode
 * LayerNorm -> projection pair of chunk-sized steps (<= 64 rows) in one kernel (LN1 -> QKV, LN2 -> FFN w1, the
 * decoder's LN -> w1 / q; sanm/encoder.py:114-145, paraformer/decoder.py:95-119); larger M runs the LayerNorm and
 * the GEMM separately. act as pfm_op_gemm. */
int pfm_op_ln_gemm(void* stream, const float* X, const float* g, const float* b, float eps, const void* W,
                   const float* bias, const float* res, float* C, int M, int N, int act);

/* Fused encoder feed-forward sub-layer (fast mode, bf16 MFMA, f32 accumulate / residual / statistics):
 *   x  = x + W2 relu(W1 LayerNorm2(x) + b1) + b2          -> xo [M, 512] f32 (may alias x)
 *   xn = LayerNorm_next(x) as bf16 [M, 512]               (optional: gn, bn, xn all non-null)
 * W1 f32 [2048, 512], W2 f32 [512, 2048] (torch Linear layout; converted to bf16 and packed per call).
 * Replaces EncoderLayerSANM's norm2 -> feed_forward -> residual (sanm/encoder.py:138-145,
 * transformer/positionwise_feed_forward.py:14-34) followed by the next layer's norm1 (encoder.py:114). */
int pfm_op_ffn(void* stream, const float* x, int M, const float* g2, const float* b2n, float eps, const float* W1,
               const float* b1, const float* W2, const float* b2, float* xo, const float* gn, const float* bn,
               void* xn);

/* Fused encoder sub-layer tail as the fast path runs it (k_ffn.hip, out-projection folded in front):
 *   x1 = o Wo^T + bo + f (+ x; x may be NULL: layer 0 has no residual)
 *   xo = x1 + W2 relu(W1 LN2(x1) + b1) + b2 ;  xn = LN_next(xo) as bf16 (optional: gn, bn, xn all or none)
 * o, f: bf16 [M, 512] (attention output, FSMN memory); x, xo: f32 [M, 512] (xo may alias x).
 * Replaces sanm/encoder.py:120-145 (linear_out + fsmn + residual, norm2, feed_forward, residual) and
 * transformer/positionwise_feed_forward.py:32-34. Weights f32 host layout [out][in] on the device; synchronous. */
int pfm_op_ffn_op(void* stream, const void* o, const void* f, const float* Wo, const float* bo, const float* x,
                  int M, const float* g2, const float* b2n, float eps, const float* W1, const float* b1,
                  const float* W2, const float* b2, float* xo, const float* gn, const float* bn, void* xn);

/* pfm_op_ffn_op followed by the next encoder layer's q|k|v projection in the same launch, as the fast path runs it
 * with the 128-row fused FFN (k_ffn2.hip MODE 4): x2 -> xo (f32) and qkv = LN1_next(x2) Wq^T + bq, bf16
 * [M, 1536] (Wq f32 [1536][512], bq [1536]; the next layer's attention.py:180-186 linear_q_k_v on its norm1).
 * With PFM_FAST_XW bit 4 set the v rows of Wq are used as two bf16 planes (MODE 5). Synchronous. */
int pfm_op_ffn_op_qkv(void* stream, const void* o, const void* f, const float* Wo, const float* bo, const float* x,
                      int M, const float* g2, const float* b2n, float eps, const float* W1, const float* b1,
                      const float* W2, const float* b2, float* xo, const float* gn, const float* bn, const float* Wq,
                      const float* bq, void* qkv);

/* Fused decoder feed-forward as the fast path runs it (k_ffn.hip DEC, LN_F folded through W2):
 *   x1 = x, or x + o Wo^T + bo when o is non-NULL (the previous block's cross-attention out-projection)
 *   y  = W2 LN_F(relu(W1 LN1(x1) + b1))  (w_2 has no bias) ;  xn = LN_next(y) bf16
 *   xo = x1 when o is non-NULL (may alias x), else y (optional)
 * Replaces sanm/positionwise_feed_forward.py:12-33 with paraformer/decoder.py:97-101 (norm1 -> feed_forward ->
 * norm2) and decoder.py:113-119 (src_attn linear_out + residual). Synchronous. */
int pfm_op_ffn_dec(void* stream, const float* x, int M, const float* g1, const float* b1n, float eps,
                   const float* W1, const float* b1, const float* W2, const float* gF, const float* bF,
                   float* xo, const float* gn, const float* bn, void* xn, const void* o, const float* Wo,
                   const float* bo);

/* Masked attention per (batch, head): q [B*Tq, heads*128], k/v [B*Tk, heads*128] of dtype,
 * klen [B] int32; out f32 [B*Tq, heads*128]. */
int pfm_op_attention(void* stream, int dtype, const void* q, const void* k, const void* v,
                     const int32_t* klen, float* out, int B, int Tq, int Tk, int heads,
                     float scale);

/* LayerNorm rows of x [M, D] f32 -> out [M, D] f32. */
int pfm_op_layernorm(void* stream, const float* x, const float* gamma, const float* beta,
                     float* out, int M, int D, float eps);

/* FSMN block: out = (res) + mask*(dwconv(mask*v) + mask*v); v/res/out [B*T, D]; w holds the
 * depthwise taps TRANSPOSED, [K, D] (fsmn_block.weight[d, 0, k] at w[k*D + d]). */
int pfm_op_fsmn(void* stream, const float* v, const int32_t* len, const float* w,
                const float* res, float* out, int B, int T, int D, int K, int left);

/* LayerNorm rows of bf16 x [M, D] (D in 512/1024/2048) -> out [M, D] f32 (fast-mode FFN hidden). */
int pfm_op_layernorm_bf16(void* stream, const void* x, const float* gamma, const float* beta, float* out,
                          int M, int D, float eps);

/* FSMN memory block on bf16 input v [B*T, D] -> bf16 out (fast-mode encoder form: no residual). */
int pfm_op_fsmn_bf16(void* stream, const void* v, const int32_t* len, const float* w, void* out, int B,
                     int T, int D, int K, int left);

/* CIF integrate-and-fire on tail-processed alphas [B, T+1] and hidden [B, T+1, D]
 * (row T zero): emb [B, L_cap, D], peaks [B, T+1], n_fire [B], ntok [B]. */
int pfm_op_cif(void* stream, const float* alphas, const float* hidden, float* emb, float* peaks,
               int32_t* n_fire, int32_t* ntok, int B, int T, int D, int L_cap);

/* Greedy CTC collapse of frame ids [B, ld] (first olen[b] valid): unique_consecutive then drop
 * `blank` -> tokens [B, L_cap] (-1 padded), ntok [B]. Same kernel pfm_run_ctc uses. */
int pfm_op_ctc_collapse(void* stream, const int32_t* ids, int64_t ld, const int32_t* olen, int B, int blank,
                        int32_t* tokens, int L_cap, int32_t* ntok);

/* The joint decoder + CTC prefix beam search of pfm_run_beam alone (k_beam.hip; BeamSearchPara,
 * paraformer/search.py:35-451, CTCPrefixScore, transformer/scorers/ctc_prefix_score.py:255-337) on given
 * log-probabilities: am [B, L, V] decoder log-probs (utterance b uses its first ntok[b] rows), x [B, T, V] CTC
 * log-probs (first lens[b] frames), device pointers. Arguments and outputs as pfm_run_beam (penalty != 0 adds
 * the LengthBonus scorer). Synchronises `stream`. */
int pfm_op_ctc_beam(void* stream, const float* am, int L, const float* x, int T, const int32_t* lens,
                    const int32_t* ntok, int B, int V, int beam, float ctc_weight, float penalty, int nbest,
                    int end_detect, int sos, int eos, int blank, int32_t* tokens, int L_cap, int32_t* ntok_out,
                    float* scores_out);

#ifdef __cplusplus
}
#endif
#endif /* PFM_H_ */
