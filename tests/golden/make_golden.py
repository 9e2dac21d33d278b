"""Generate golden vectors by running the REAL reference modules in the build container.

Run (build container only — /root/reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference package is imported from /root/reference with four audio/config IO
modules stubbed (kaldiio, librosa, torchaudio, omegaconf — none is on the fbank-input
path) and `funasr/__init__.py` bypassed. Weights come from
funasr_amd.weights (seed 0) loaded with strict load_state_dict; inputs are seeded
N(0,1) fbank tensors. Only inputs' seeds + outputs are stored (fixtures are data).

Outputs (tests/golden/*.npz):
  para_tiny.npz     enc 3 / dec 2 blocks, B=2 ragged: full encoder output, alphas,
                    peaks, token_num, acoustic embeds, decoder argmax, decoder logit rows.
  para_large_*.npz  Paraformer-large: token ids, token_num, alphas, encoder row slices
                    and per-utterance checksums, top-2 logit margins.
  lfr_cmvn.npz      reference apply_lfr / apply_cmvn / load_cmvn on seeded fbank.
  automodel_tiny.json  AutoModel.generate() result dicts (key/text) for the tiny config.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True


def install_stubs():
    pkg = types.ModuleType("funasr")
    pkg.__path__ = [f"{REF}/funasr"]
    sys.modules["funasr"] = pkg
    for n in ["kaldiio", "librosa", "torchaudio", "torchaudio.compliance", "torchaudio.compliance.kaldi"]:
        sys.modules[n] = types.ModuleType(n)
    sys.modules["torchaudio"].compliance = sys.modules["torchaudio.compliance"]
    sys.modules["torchaudio.compliance"].kaldi = sys.modules["torchaudio.compliance.kaldi"]
    oc = types.ModuleType("omegaconf")

    class DictConfig(dict):
        pass

    class ListConfig(list):
        pass

    oc.DictConfig, oc.ListConfig, oc.OmegaConf = DictConfig, ListConfig, None
    sys.modules["omegaconf"] = oc


install_stubs()
import torch  # noqa: E402

import funasr.models.paraformer.model  # noqa: E402,F401
import funasr.models.sanm.encoder  # noqa: E402,F401
import funasr.models.paraformer.decoder  # noqa: E402,F401
import funasr.models.paraformer.cif_predictor  # noqa: E402,F401
from funasr.register import tables  # noqa: E402

from funasr_amd.config import paraformer_large, paraformer_tiny  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.golden.inputs import fbank_input, token_list  # noqa: E402

CMVN = f"{REF}/runtime/triton_gpu/model_repo_paraformer_large_online/lfr_cmvn_pe/am.mvn"


def build_ref(cfg):
    kw = cfg.reference_kwargs()
    cls = tables.model_classes["Paraformer"]
    m = cls(encoder=kw["encoder"], encoder_conf=kw["encoder_conf"], decoder=kw["decoder"],
            decoder_conf=kw["decoder_conf"], predictor=kw["predictor"],
            predictor_conf=kw["predictor_conf"], input_size=cfg.input_size,
            vocab_size=cfg.vocab_size, ctc_weight=0.0, predictor_bias=1)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    m.load_state_dict(sd, strict=True)
    m.eval()
    return m


@torch.no_grad()
def run_ref(m, feats, lens):
    """Stage-by-stage reference run (what Paraformer.inference does for fbank input)."""
    x = torch.from_numpy(feats)
    ln = torch.from_numpy(lens.astype(np.int64))
    enc, olens = m.encode(x, ln)
    embeds, token_num, alphas, peak = m.calc_predictor(enc, olens)
    ntok = token_num.round().long()
    logp, _ = m.cal_decoder_with_predictor(enc, olens, embeds, ntok)
    res = m.inference(x, data_lengths=ln[:, None], key=[f"utt{i}" for i in range(len(lens))],
                      tokenizer=None, data_type="fbank", device="cpu")[0]
    tokens = [r["token_int"] for r in res]
    return dict(enc=enc.numpy(), enc_lens=olens.numpy(), embeds=embeds.numpy(),
                token_num=token_num.numpy(), alphas=alphas.numpy(), peak=peak.numpy(),
                ntok=ntok.numpy(), logp=logp.numpy(), tokens=tokens)


def pack_tokens(tokens):
    flat = np.array([t for ts in tokens for t in ts], dtype=np.int32)
    off = np.cumsum([0] + [len(t) for t in tokens]).astype(np.int32)
    return flat, off


def topk_rows(logp, ntok, k=5):
    """Per decoded position (utterance order): the k best ids (value desc, id asc) and their log-probs."""
    ids, vals = [], []
    for b in range(logp.shape[0]):
        t = torch.from_numpy(np.ascontiguousarray(logp[b, : ntok[b]]))
        v, i = torch.topk(t, k, dim=-1, sorted=True)
        ids.append(i.numpy().astype(np.int32))
        vals.append(v.numpy().astype(np.float32))
    return np.concatenate(ids), np.concatenate(vals)


def top2_margin(logp, ntok):
    out = []
    for b in range(logp.shape[0]):
        r = np.sort(logp[b, : ntok[b]], axis=-1)
        out.append(r[:, -1] - r[:, -2])
    return np.concatenate(out).astype(np.float32)


def save_tiny():
    cfg = paraformer_tiny()
    m = build_ref(cfg)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    r = run_ref(m, feats, lens)
    flat, off = pack_tokens(r["tokens"])
    # decoder logits of a few rows only (full logits are B*L*8404 floats)
    rows = np.stack([r["logp"][0, 0], r["logp"][0, int(r["ntok"][0]) - 1], r["logp"][1, 0]])
    np.savez_compressed(f"{HERE}/para_tiny.npz", seed=11, B=2, T=40, lens=lens,
                        enc=r["enc"], enc_lens=r["enc_lens"], embeds=r["embeds"],
                        token_num=r["token_num"], alphas=r["alphas"], peak=r["peak"], ntok=r["ntok"],
                        argmax=r["logp"].argmax(-1).astype(np.int32), logp_rows=rows,
                        tokens=flat, tokens_off=off, margin=top2_margin(r["logp"], r["ntok"]))
    print("tiny: ntok", r["ntok"], "tokens", [len(t) for t in r["tokens"]])


def save_large(m, name, seed, B, T, lens):
    feats, lens = fbank_input(seed=seed, B=B, T=T, lens=lens)
    r = run_ref(m, feats, lens)
    flat, off = pack_tokens(r["tokens"])
    enc = r["enc"]
    sl = []
    for b in range(B):
        n = int(lens[b])
        sl.append(enc[b, [0, 1, n // 2, n - 1]])
    valid = np.arange(T)[None, :] < lens[:, None]
    csum = np.array([enc[b][valid[b]].astype(np.float64).sum() for b in range(B)])
    csq = np.array([(enc[b][valid[b]].astype(np.float64) ** 2).sum() for b in range(B)])
    np.savez_compressed(f"{HERE}/{name}.npz", seed=seed, B=B, T=T, lens=lens,
                        enc_rows=np.stack(sl), enc_sum=csum, enc_sumsq=csq, enc_lens=r["enc_lens"],
                        token_num=r["token_num"], alphas=r["alphas"], peak=r["peak"], ntok=r["ntok"],
                        tokens=flat, tokens_off=off, margin=top2_margin(r["logp"], r["ntok"]))
    print(name, "ntok", r["ntok"], "min margin", top2_margin(r["logp"], r["ntok"]).min())


HEADLINE = {   # name: (seed, B, T, lens) — batches whose per-group row counts engage the fast path's fused
    # encoder FFN (OP mode), fused decoder FFN and the two-group concurrent dispatch (bench config C2 = b64)
    "para_large_b24": (6, 24, 500, [500 - 9 * i for i in range(24)]),
    "para_large_b64": (7, 64, 500, None),
}


def save_headline():
    """Paraformer-large reference run at the bench configuration (B=64 x T=500) and a B=24 ragged batch:
    token ids, the per-position decoder argmax (incl. special ids) and top-2 log-prob margins, token counts,
    alphas, three encoder rows per utterance and per-utterance encoder checksums."""
    m = build_ref(paraformer_large())
    for name, (seed, B, T, ln) in HEADLINE.items():
        feats, lens = fbank_input(seed=seed, B=B, T=T, lens=ln)
        r = run_ref(m, feats, lens)
        flat, off = pack_tokens(r["tokens"])
        enc = r["enc"]
        rows = np.stack([enc[b, [0, int(lens[b]) // 2, int(lens[b]) - 1]] for b in range(B)])
        valid = np.arange(T)[None, :] < lens[:, None]
        csum = np.array([enc[b][valid[b]].astype(np.float64).sum() for b in range(B)])
        csq = np.array([(enc[b][valid[b]].astype(np.float64) ** 2).sum() for b in range(B)])
        am = np.concatenate([r["logp"][b, : r["ntok"][b]].argmax(-1) for b in range(B)]).astype(np.int32)
        tid, tlp = topk_rows(r["logp"], r["ntok"])
        np.savez_compressed(f"{HERE}/{name}.npz", seed=seed, B=B, T=T, lens=lens, enc_rows=rows, enc_sum=csum,
                            enc_sumsq=csq, enc_lens=r["enc_lens"], token_num=r["token_num"], alphas=r["alphas"],
                            ntok=r["ntok"], tokens=flat, tokens_off=off, argmax=am,
                            margin=top2_margin(r["logp"], r["ntok"]), top_ids=tid, top_logp=tlp)
        mg = top2_margin(r["logp"], r["ntok"])
        print(name, "ntok mean", r["ntok"].mean(), "positions", len(mg), "min margin", mg.min(),
              "margins < 1e-3:", int((mg < 1e-3).sum()))


BEAM_CASES = {   # name: (large?, weight seed, fbank seed, B, T, lens, decoding_ctc_weight, beam_size, penalty, nbest
    #        [, + on the decoder output bias of eos: hypotheses end at many positions])
    "beam_tiny": (False, 4, 21, 3, 40, [40, 27, 9], 0.3, 3, 0.0, 2),
    "beam_tiny_pen": (False, 4, 22, 2, 40, [33, 40], 0.5, 4, 0.8, 3),
    "beam_large": (True, 0, 23, 2, 500, [500, 431], 0.3, 4, 0.0, 2),
    # nbest > beam: sorted(ended_hyps)[:nbest] collects ended hypotheses of every position (more than beam)
    "beam_tiny_nb": (False, 4, 24, 3, 40, [40, 31, 22], 0.01, 2, 0.0, 5, 8.0),
}


def save_beam_nb():
    save_beam(["beam_tiny_nb"])


def save_beam(only=None):
    """Paraformer with a CTC head (model_conf ctc_weight 0.3) decoded by the reference's joint decoder + CTC prefix
    beam search (Paraformer.inference with decoding_ctc_weight > 0: BeamSearchPara + CTCPrefixScorer +
    LengthBonus, paraformer/model.py:396-441, 530-565). Stores the n-best yseqs (sos ... eos) and scores from
    beam_search() itself and the token_int result dicts of inference()."""
    import dataclasses
    models = {}
    for name, case in BEAM_CASES.items():
        if only is not None and name not in only:
            continue
        large, wseed, fseed, B, T, ln, wctc, beam, pen, nbest = case[:10]
        eos_boost = case[10] if len(case) > 10 else 0.0
        cfg = dataclasses.replace(paraformer_large() if large else paraformer_tiny(), ctc_weight=0.3)
        kw = cfg.reference_kwargs()
        cls = tables.model_classes["Paraformer"]
        m = cls(encoder=kw["encoder"], encoder_conf=kw["encoder_conf"], decoder=kw["decoder"],
                decoder_conf=kw["decoder_conf"], predictor=kw["predictor"], predictor_conf=kw["predictor_conf"],
                input_size=cfg.input_size, vocab_size=cfg.vocab_size, ctc_weight=0.3, predictor_bias=1)
        w = make_weights(cfg, seed=wseed)
        if eos_boost:
            w["decoder.output_layer.bias"] = w["decoder.output_layer.bias"].copy()
            w["decoder.output_layer.bias"][cfg.eos] += eos_boost
        m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=True)
        m.eval()
        feats, lens = fbank_input(seed=fseed, B=B, T=T, lens=ln)
        x = torch.from_numpy(feats)
        l64 = torch.from_numpy(lens.astype(np.int64))
        toks = token_list(cfg.vocab_size)
        opts = dict(decoding_ctc_weight=wctc, beam_size=beam, penalty=pen, nbest=nbest, token_list=toks)
        with torch.no_grad():
            res = m.inference(x, data_lengths=l64[:, None], key=[f"utt{i}" for i in range(B)], tokenizer=None,
                              data_type="fbank", device="cpu", **opts)[0]
            enc, olens = m.encode(x, l64)
            embeds, token_num, alphas, peak = m.calc_predictor(enc, olens)
            ntok = token_num.round().long()
            logp, _ = m.cal_decoder_with_predictor(enc, olens, embeds, ntok)
            yseq, scores, owner = [], [], []
            for i in range(B):
                nb = m.beam_search(x=enc[i, : olens[i]], am_scores=logp[i, : ntok[i]], maxlenratio=0.0,
                                   minlenratio=0.0)[:nbest]
                for h in nb:
                    yseq.append(h.yseq.tolist())
                    scores.append(float(h.score))
                    owner.append(i)
        flat, off = pack_tokens(yseq)
        rflat, roff = pack_tokens([r["token_int"] for r in res])
        np.savez_compressed(f"{HERE}/{name}.npz", large=large, wseed=wseed, seed=fseed, B=B, T=T, lens=lens,
                            decoding_ctc_weight=wctc, beam_size=beam, penalty=pen, nbest=nbest, ntok=ntok.numpy(),
                            eos_boost=eos_boost,
                            enc_lens=olens.numpy(), yseq=flat, yseq_off=off, scores=np.array(scores, np.float32),
                            owner=np.array(owner, np.int32), result_tokens=rflat, result_off=roff)
        print(name, "ntok", ntok.tolist(), "hyps", len(yseq), "scores", [round(v, 3) for v in scores])


def save_lfr_cmvn():
    from funasr.frontends.wav_frontend import apply_cmvn, apply_lfr, load_cmvn
    cmvn = load_cmvn(CMVN).numpy()
    out = dict(cmvn=cmvn)
    rng = np.random.default_rng(5)
    for n in [1, 2, 5, 6, 7, 11, 12, 13, 83, 498]:
        fb = rng.standard_normal((n, 80)).astype(np.float32)
        lfr = apply_lfr(torch.from_numpy(fb.copy()), 7, 6)
        cm = apply_cmvn(lfr.clone(), torch.from_numpy(cmvn))
        out[f"in_{n}"] = fb
        out[f"lfr_{n}"] = lfr.numpy()
        out[f"cmvn_{n}"] = cm.numpy()
    np.savez_compressed(f"{HERE}/lfr_cmvn.npz", **out)
    print("lfr_cmvn saved")


def save_automodel_tiny():
    """AutoModel.generate() on the tiny config with a CharTokenizer: pins the result-dict contract."""
    import funasr.tokenizer.char_tokenizer  # noqa: F401
    import funasr.frontends.wav_frontend  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    cfg = paraformer_tiny()
    kw = cfg.reference_kwargs()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                   device="cpu", ncpu=4, disable_update=True, disable_pbar=True, disable_log=True,
                   tokenizer="CharTokenizer", tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)),
                   frontend="WavFrontend", frontend_conf=dict(fs=16000, window="hamming", n_mels=80,
                                                             frame_length=25, frame_shift=10, lfr_m=7,
                                                             lfr_n=6, dither=0.0, cmvn_file=CMVN),
                   **kw)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    am.model.load_state_dict(sd, strict=True)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens.astype(np.int32))[:, None],
                      data_type="fbank", key=["uttA", "uttB"])
    res = [{k: (v if not isinstance(v, np.ndarray) else v.tolist()) for k, v in r.items()} for r in res]
    with open(f"{HERE}/automodel_tiny.json", "w") as f:
        json.dump(res, f, ensure_ascii=False, indent=1)
    print("automodel:", [r["text"][:20] for r in res])


POSTPROC_CASES = [
    ["欢", "迎", "大", "家"], ["he@@", "llo", "world"], ["a", "b", "c"], ["i", "am", "o@@", "k"],
    ["你", "好", "hello", "世", "界"], ["<s>", "今", "天", "</s>", "<unk>"], ["12", "月", "3", "号"],
    ["g", "p", "u", "是", "a", "m", "d"], ["x", "<unk>", "y", "z"], ["don't", "stop"], ["@", "a"],
    ["中", "a@@", "b", "文"], ["!", "好"], [], ["<s>"], ["a", " ", "b"], ["hel@@", "lo"], ["A", "b", "C", "d@@", "e"],
]


def save_postprocess():
    from funasr.utils.postprocess_utils import sentence_postprocess
    out = []
    for toks in POSTPROC_CASES:
        sent, words = sentence_postprocess(list(toks))
        out.append({"tokens": toks, "sentence": sent, "words": words})
    with open(f"{HERE}/postprocess.json", "w") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print("postprocess cases", len(out))


def save_timestamps():
    """Reference ts_prediction_lfr6_standard + sentence_postprocess(words, time_stamp) on seeded
    synthetic CIF weights (both fire-search branches, '</s>', VAD offset, upsample rates)."""
    from funasr.utils.postprocess_utils import sentence_postprocess
    from funasr.utils.timestamp_tools import cif_wo_hidden, ts_prediction_lfr6_standard
    rng = np.random.default_rng(5)
    cases = []
    for ci, (T, ntok_extra, upsample, offset, eos) in enumerate([
            (40, 0, 1, 0, False), (83, 0, 1, 0, True), (200, 3, 1, 0, False), (501, 0, 1, 0, False),
            (501, -7, 1, 1230, False), (120, 0, 3, 0, False), (300, 2, 1, 0, True), (60, -1, 1, 0, False)]):
        a = (rng.random(T) * 0.6).astype(np.float32)
        a[rng.random(T) < 0.3] = 0.0
        peaks = cif_wo_hidden(torch.from_numpy(a)[None].clone(), 1.0 - 1e-4)[0].numpy()
        n_fire = int((peaks >= 1.0 - 1e-4).sum())
        nchar = max(1, n_fire - 1 + ntok_extra)
        chars = [f"t{i}" for i in range(nchar)] + (["</s>"] if eos else [])
        # the Paraformer call site passes (peaks, alphas) as (us_alphas, us_peaks)
        txt, ts = ts_prediction_lfr6_standard(torch.from_numpy(peaks.copy()), torch.from_numpy(a.copy()),
                                              list(chars), vad_offset=offset, upsample_rate=upsample)
        cases.append({"alphas": a.tolist(), "peaks": peaks.tolist(), "chars": chars, "vad_offset": offset,
                      "upsample_rate": upsample, "text": txt, "timestamp": ts})
    pp = []
    for toks in POSTPROC_CASES:
        spans = [[100 * i, 100 * i + 80] for i in range(len(toks))]
        try:
            sent, ts, words = sentence_postprocess(list(toks), spans)
        except Exception as e:   # noqa: BLE001 - record the reference's failure mode
            pp.append({"tokens": toks, "error": type(e).__name__})
            continue
        pp.append({"tokens": toks, "spans": spans, "sentence": sent, "timestamp": ts, "words": words})
    with open(f"{HERE}/timestamps.json", "w") as f:
        json.dump({"ts_prediction": cases, "postprocess_ts": pp}, f, ensure_ascii=False, indent=1)
    print("timestamp cases", len(cases), "postprocess_ts", len(pp))


def save_automodel_tiny_ts():
    """AutoModel.generate(..., pred_timestamp=True) on the tiny config: text + word timestamps."""
    import funasr.tokenizer.char_tokenizer  # noqa: F401
    import funasr.frontends.wav_frontend  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    cfg = paraformer_tiny()
    kw = cfg.reference_kwargs()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                   device="cpu", ncpu=4, disable_update=True, disable_pbar=True, disable_log=True,
                   tokenizer="CharTokenizer", tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)),
                   frontend="WavFrontend", frontend_conf=dict(fs=16000, window="hamming", n_mels=80,
                                                             frame_length=25, frame_shift=10, lfr_m=7,
                                                             lfr_n=6, dither=0.0, cmvn_file=CMVN),
                   **kw)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    am.model.load_state_dict(sd, strict=True)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens.astype(np.int32))[:, None],
                      data_type="fbank", key=["uttA", "uttB"], pred_timestamp=True)
    res = [{k: (v if not isinstance(v, np.ndarray) else v.tolist()) for k, v in r.items()} for r in res]
    with open(f"{HERE}/automodel_tiny_ts.json", "w") as f:
        json.dump(res, f, ensure_ascii=False, indent=1)
    print("automodel ts:", [(r["text"][:12], r["timestamp"][:2]) for r in res])


# ---------------------------------------------------------------- SenseVoiceSmall (config C4)
class _IdTokenizer:
    """decode(ids) -> "id id id": lets the reference's tokenizer.decode call return token_int."""

    def decode(self, ids):
        return " ".join(str(int(i)) for i in ids)


def build_sv_ref(cfg, bias_boost=None):
    import funasr.models.sense_voice.model  # noqa: F401
    kw = cfg.reference_kwargs()
    m = tables.model_classes["SenseVoiceSmall"](encoder=kw["encoder"], encoder_conf=kw["encoder_conf"],
                                                input_size=cfg.input_size, vocab_size=cfg.vocab_size)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    if bias_boost:
        b = sd["ctc.ctc_lo.bias"].clone()
        for tok, add in bias_boost.items():
            b[tok] += add
        sd["ctc.ctc_lo.bias"] = b
    m.load_state_dict(sd, strict=True)
    m.eval()
    return m


@torch.no_grad()
def run_sv_ref(m, feats, lens, **opts):
    """Reference SenseVoiceSmall.inference (data_type fbank) + hooks on encoder / ctc_lo outputs."""
    cap = {}
    h1 = m.encoder.register_forward_hook(lambda mod, i, o: cap.__setitem__("enc", o))
    h2 = m.ctc.ctc_lo.register_forward_hook(lambda mod, i, o: cap.__setitem__("logits", o))
    try:
        res, _ = m.inference(torch.from_numpy(feats.copy()), data_lengths=torch.from_numpy(lens.astype(np.int64)),
                             key=[f"utt{i}" for i in range(len(lens))], tokenizer=_IdTokenizer(),
                             data_type="fbank", device="cpu", **opts)
    finally:
        h1.remove()
        h2.remove()
    enc, olens = cap["enc"]
    logp = torch.log_softmax(cap["logits"], dim=2)
    if opts.get("ban_emo_unk"):
        logp[:, :, m.emo_dict["unk"]] = -float("inf")
    tokens = [[int(t) for t in r["text"].split()] for r in res]
    return dict(enc=enc.numpy(), enc_lens=olens.numpy(), logp=logp.numpy(), tokens=tokens,
                frame_ids=logp.argmax(-1).numpy().astype(np.int32))


def _frame_margin(logp, olens):
    out = []
    for b in range(logp.shape[0]):
        r = np.sort(logp[b, : olens[b]], axis=-1)
        out.append(r[:, -1] - r[:, -2])
    return np.concatenate(out).astype(np.float32)


def save_sv_tiny():
    """SenseVoice tiny (3 + 2 blocks): full encoder output; option / bias-boost variants pin the
    query rows, ban_emo_unk and the CTC collapse (blank-heavy frames)."""
    from funasr_amd.config import sense_voice_tiny
    cfg = sense_voice_tiny()
    feats, lens = fbank_input(seed=21, B=2, T=40, lens=[40, 27])
    out = dict(seed=21, B=2, T=40, lens=lens)
    m = build_sv_ref(cfg)
    r = run_sv_ref(m, feats, lens)
    flat, off = pack_tokens(r["tokens"])
    out.update(enc=r["enc"], enc_lens=r["enc_lens"], frame_ids=r["frame_ids"], tokens=flat, tokens_off=off,
               logp_rows=np.stack([r["logp"][0, 0], r["logp"][0, 5], r["logp"][1, 30]]),
               margin=_frame_margin(r["logp"], r["enc_lens"]))
    r = run_sv_ref(m, feats, lens, language="zh", use_itn=True)
    flat, off = pack_tokens(r["tokens"])
    out.update(zh_itn_tokens=flat, zh_itn_off=off, zh_itn_frame_ids=r["frame_ids"])
    # blank-heavy variant: bias of blank raised so roughly half the frames emit blank
    mb = build_sv_ref(cfg, bias_boost={0: 2.5})
    r = run_sv_ref(mb, feats, lens, language="en", text_norm="withitn")
    flat, off = pack_tokens(r["tokens"])
    out.update(blank_tokens=flat, blank_off=off, blank_frame_ids=r["frame_ids"],
               blank_margin=_frame_margin(r["logp"], r["enc_lens"]))
    # emo-unk variant: token 25009 dominates every frame unless banned
    me = build_sv_ref(cfg, bias_boost={25009: 50.0})
    r = run_sv_ref(me, feats, lens)
    out.update(emo_tokens=pack_tokens(r["tokens"])[0], emo_off=pack_tokens(r["tokens"])[1])
    r = run_sv_ref(me, feats, lens, ban_emo_unk=True)
    flat, off = pack_tokens(r["tokens"])
    out.update(ban_tokens=flat, ban_off=off, ban_frame_ids=r["frame_ids"])
    np.savez_compressed(f"{HERE}/sv_tiny.npz", **out)
    print("sv_tiny tokens", [len(t) for t in r["tokens"]], "blank frac",
          float((out["blank_frame_ids"] == 0).mean()), "emo", out["emo_tokens"][:6])


def save_sv_large():
    from funasr_amd.config import sense_voice_small
    m = build_sv_ref(sense_voice_small())
    for name, seed, B, T, ln in [("sv_large_ragged", 4, 3, 500, [500, 431, 83]), ("sv_large_c1", 5, 1, 83, [83])]:
        feats, lens = fbank_input(seed=seed, B=B, T=T, lens=ln)
        r = run_sv_ref(m, feats, lens)
        flat, off = pack_tokens(r["tokens"])
        enc, ol = r["enc"], r["enc_lens"]
        rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(B)])
        valid = np.arange(enc.shape[1])[None, :] < ol[:, None]
        csum = np.array([enc[b][valid[b]].astype(np.float64).sum() for b in range(B)])
        csq = np.array([(enc[b][valid[b]].astype(np.float64) ** 2).sum() for b in range(B)])
        np.savez_compressed(f"{HERE}/{name}.npz", seed=seed, B=B, T=T, lens=lens, enc_rows=rows, enc_sum=csum,
                            enc_sumsq=csq, enc_lens=ol, frame_ids=r["frame_ids"], tokens=flat, tokens_off=off,
                            margin=_frame_margin(r["logp"], ol))
        print(name, "tokens", [len(t) for t in r["tokens"]], "min margin", _frame_margin(r["logp"], ol).min())


SV_HEADLINE = {   # name: (seed, B, T, lens) — SenseVoiceSmall at BASELINE config C4 (B=64 x 500 frames, the bench's
    # SenseVoice leg) and a ragged 24-utterance batch; group rows B/2 x (T+4) >= 4096 engage the fused OP-FFN (LN 1e-5)
    "sv_large_b24": (8, 24, 500, [500 - 9 * i for i in range(24)]),
    "sv_large_b64": (9, 64, 500, None),
}


def save_sv_headline():
    """Reference SenseVoiceSmall.inference (sense_voice/model.py:809-906) at the C4 configuration: token ids, the
    per-frame CTC argmax with its top-2 margin and the top-3 ids / log-probs of every frame, encoder rows
    (0, 3, 4, n/2, n-1) and per-utterance sums / sums of squares of the encoder output."""
    from funasr_amd.config import sense_voice_small
    m = build_sv_ref(sense_voice_small())
    for name, (seed, B, T, ln) in SV_HEADLINE.items():
        feats, lens = fbank_input(seed=seed, B=B, T=T, lens=ln)
        r = run_sv_ref(m, feats, lens)
        flat, off = pack_tokens(r["tokens"])
        enc, ol = r["enc"], r["enc_lens"]
        rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(B)])
        valid = np.arange(enc.shape[1])[None, :] < ol[:, None]
        csum = np.array([enc[b][valid[b]].astype(np.float64).sum() for b in range(B)])
        csq = np.array([(enc[b][valid[b]].astype(np.float64) ** 2).sum() for b in range(B)])
        tid, tlp = topk_rows(r["logp"], ol, k=3)
        mg = _frame_margin(r["logp"], ol)
        np.savez_compressed(f"{HERE}/{name}.npz", seed=seed, B=B, T=T, lens=lens, enc_rows=rows, enc_sum=csum,
                            enc_sumsq=csq, enc_lens=ol, frame_ids=r["frame_ids"], tokens=flat, tokens_off=off,
                            margin=mg, top_ids=tid, top_logp=tlp)
        print(name, "tokens mean", np.mean([len(t) for t in r["tokens"]]), "frames", len(mg), "min margin", mg.min(),
              "margins < 1e-3:", int((mg < 1e-3).sum()))


def make_sv_bpe(path, vocab=300):
    """Tiny sentencepiece BPE model trained on seeded synthetic text (stands in for SenseVoice's
    chn_jpn_yue_eng_ko_spectok.bpe.model, which cannot be fetched offline)."""
    import io

    import sentencepiece as spm
    rng = np.random.default_rng(7)
    syll = ["ka", "to", "ri", "me", "su", "na", "lo", "pe", "di", "gu", "ba", "ze", "ho", "vi", "qu"]
    lines = [" ".join("".join(rng.choice(syll, size=rng.integers(1, 4))) for _ in range(rng.integers(4, 12)))
             for _ in range(3000)]
    model = io.BytesIO()
    spm.SentencePieceTrainer.train(sentence_iterator=iter(lines), model_writer=model, vocab_size=vocab,
                                   model_type="bpe", character_coverage=1.0, num_threads=1, normalization_rule_name="identity",
                                   minloglevel=2)
    with open(path, "wb") as f:
        f.write(model.getvalue())


def save_automodel_sv_tiny():
    """Reference AutoModel.generate() with SenseVoiceSmall (tiny, vocab 300) + SentencepiecesTokenizer:
    pins the SenseVoice result-dict contract (language / use_itn query rows, tokenizer.decode)."""
    import funasr.models.sense_voice.model  # noqa: F401
    import funasr.tokenizer.sentencepiece_tokenizer  # noqa: F401
    import funasr.frontends.wav_frontend  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    from funasr_amd.config import sense_voice_tiny
    bpe = f"{HERE}/sv_bpe.model"
    if not os.path.exists(bpe):
        make_sv_bpe(bpe)
    cfg = sense_voice_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    am = AutoModel(model="SenseVoiceSmall", model_conf={}, device="cpu", ncpu=4, disable_update=True,
                   disable_pbar=True, disable_log=True, tokenizer="SentencepiecesTokenizer",
                   tokenizer_conf=dict(bpemodel=bpe), frontend="WavFrontend",
                   frontend_conf=dict(fs=16000, window="hamming", n_mels=80, frame_length=25, frame_shift=10,
                                      lfr_m=7, lfr_n=6, dither=0.0, cmvn_file=CMVN),
                   encoder=kw["encoder"], encoder_conf=kw["encoder_conf"])
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    am.model.load_state_dict(sd, strict=True)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    out = {}
    for tag, opts in (("auto", {}), ("en_itn", dict(language="en", use_itn=True))):
        res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens.astype(np.int32)),
                          data_type="fbank", key=["uttA", "uttB"], batch_size=2, **opts)
        out[tag] = [{k: (v if not isinstance(v, np.ndarray) else v.tolist()) for k, v in r.items()} for r in res]
    with open(f"{HERE}/automodel_sv_tiny.json", "w") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print("automodel sv:", {k: [r["text"][:20] for r in v] for k, v in out.items()})


def save_sv_timestamps():
    """SenseVoice output_timestamp (model.py:917-945): (1) the reference ctc_forced_align on seeded emissions
    (repeated labels, blank-zeroed softmax rows); (2) reference SenseVoiceSmall.inference(output_timestamp=True)
    on the tiny config (vocab 300, sentencepiece tokenizer) one utterance per call, with the emission / targets /
    alignment the reference's own ctc_forced_align call saw and the result dicts."""
    import funasr.models.sense_voice.model as svm
    import funasr.tokenizer.sentencepiece_tokenizer  # noqa: F401
    from funasr.models.sense_voice.utils.ctc_alignment import ctc_forced_align
    from funasr_amd.config import sense_voice_tiny
    out = {}
    rng = np.random.default_rng(7)
    cases = [(30, 6, [3, 5, 5, 2, 4, 1]), (50, 9, [1, 2, 3, 4, 5, 6, 7, 8]), (12, 5, [4, 4, 4]), (8, 4, [2, 3, 1, 2])]
    for k, (T, V, tg) in enumerate(cases):
        e = torch.softmax(torch.from_numpy(rng.standard_normal((T, V)).astype(np.float32) * 2), -1)
        e[e.argmax(-1) == 0, 0] = 0
        a = ctc_forced_align(e[None].clone(), torch.tensor(tg)[None].long(), torch.tensor([T]).long(),
                             torch.tensor([len(tg)]).long())
        out[f"dp{k}_emis"], out[f"dp{k}_targets"], out[f"dp{k}_align"] = e.numpy(), np.array(tg), a[0].numpy()
    bpe = f"{HERE}/sv_bpe.model"
    if not os.path.exists(bpe):
        make_sv_bpe(bpe)
    tok = tables.tokenizer_classes["SentencepiecesTokenizer"](bpemodel=bpe)
    cfg = sense_voice_tiny(vocab_size=300)
    seen = []
    orig = svm.ctc_forced_align

    def spy(log_probs, targets, input_lengths, target_lengths, **kw):
        targets = targets.clone()
        e = log_probs[0].detach().clone().numpy()
        r = orig(log_probs, targets, input_lengths, target_lengths, **kw)
        seen.append((e, targets[0].numpy(), r[0].numpy()))
        return r

    svm.ctc_forced_align = spy
    results = []
    try:
        for bias, seed, T in ((None, 31, 40), ({0: 2.5}, 32, 60), ({0: 1.0}, 33, 25)):
            m = build_sv_ref(cfg, bias_boost=bias)
            feats, lens = fbank_input(seed=seed, B=1, T=T, lens=[T])
            res, _ = m.inference(torch.from_numpy(feats.copy()), data_lengths=torch.from_numpy(lens.astype(np.int64)),
                                 key=[f"utt{seed}"], tokenizer=tok, data_type="fbank", device="cpu",
                                 output_timestamp=True)
            r = res[0]
            results.append(dict(seed=seed, T=T, bias=bias and {str(k): v for k, v in bias.items()}, key=r["key"],
                                text=r["text"], timestamp=[[int(a), int(b)] for a, b in r["timestamp"]]))
    finally:
        svm.ctc_forced_align = orig
    for k, (e, tg, a) in enumerate(seen):
        out[f"sv{k}_emis"], out[f"sv{k}_targets"], out[f"sv{k}_align"] = e, tg, a
    np.savez_compressed(f"{HERE}/sv_timestamps.npz", **out)
    with open(f"{HERE}/sv_timestamps.json", "w") as f:
        json.dump(results, f, ensure_ascii=False, indent=1)
    print("sv timestamps:", [(r["text"][:20], len(r["timestamp"])) for r in results])


def save_automodel_tiny_bpe():
    """Reference AutoModel.generate() with Paraformer (tiny, vocab 300) + SentencepiecesTokenizer: pins the
    bpemodel branch of Paraformer.inference (text = tokens2text(ids2tokens(ids)), no sentence_postprocess,
    paraformer/model.py:567-586)."""
    import funasr.tokenizer.sentencepiece_tokenizer  # noqa: F401
    import funasr.frontends.wav_frontend  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    bpe = f"{HERE}/sv_bpe.model"
    if not os.path.exists(bpe):
        make_sv_bpe(bpe)
    cfg = paraformer_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                   device="cpu", ncpu=4, disable_update=True, disable_pbar=True, disable_log=True,
                   tokenizer="SentencepiecesTokenizer", tokenizer_conf=dict(bpemodel=bpe),
                   frontend="WavFrontend", frontend_conf=dict(fs=16000, window="hamming", n_mels=80,
                                                             frame_length=25, frame_shift=10, lfr_m=7,
                                                             lfr_n=6, dither=0.0, cmvn_file=CMVN),
                   **kw)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    am.model.load_state_dict(sd, strict=True)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens.astype(np.int32))[:, None],
                      data_type="fbank", key=["uttA", "uttB"])
    res = [{k: (v if not isinstance(v, np.ndarray) else v.tolist()) for k, v in r.items()} for r in res]
    with open(f"{HERE}/automodel_tiny_bpe.json", "w") as f:
        json.dump(res, f, ensure_ascii=False, indent=1)
    print("automodel bpe:", [r["text"][:40] for r in res])


def build_stream_ref(cfg):
    import funasr.models.scama.encoder  # noqa: F401
    import funasr.models.paraformer_streaming.model  # noqa: F401
    kw = cfg.reference_kwargs()
    m = tables.model_classes["ParaformerStreaming"](
        **{k: kw[k] for k in ("encoder", "encoder_conf", "decoder", "decoder_conf", "predictor", "predictor_conf")},
        input_size=cfg.input_size, vocab_size=cfg.vocab_size, ctc_weight=0.0, predictor_bias=1)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
    m.eval()
    return m


class _Recorder:
    """Wraps the reference encoder / predictor forward_chunk to keep each chunk's outputs."""

    def __init__(self, m):
        self.enc, self.alphas_in = [], []
        fe, fp = m.encoder.forward_chunk, m.predictor.forward_chunk

        def enc_chunk(*a, **k):
            r = fe(*a, **k)
            self.enc.append(r[0][0].detach().clone())
            return r

        def pred_chunk(hidden, cache=None, **k):
            return fp(hidden, cache=cache, **k)

        m.encoder.forward_chunk = enc_chunk
        m.predictor.forward_chunk = pred_chunk


def _stream_cache(m, elb, dlb):
    cache = {}
    m.init_cache(cache, chunk_size=[0, 10, 5], encoder_chunk_look_back=elb, decoder_chunk_look_back=dlb,
                 encoder_conf={"output_size": 512}, frontend_conf={"n_mels": 80, "lfr_m": 7})
    return cache


class _IdsTok:
    def ids2tokens(self, ids):
        return list(ids)


def save_stream():
    """ParaformerStreaming (tiny: enc 3 / dec 2) chunk-level goldens: seeded LFR+CMVN chunks of 10
    frames through the reference generate_chunk with its cache, for (encoder, decoder) look-back
    (0, 0) and (4, 1), ending in a short final chunk or in the tail chunk (cached overlap only).
    Then the waveform path: reference inference() over 600 ms sample chunks with WavFrontendOnline
    (kaldi.fbank patched to oracle/fbank_ref.fbank, the pinned fbank restatement)."""
    from funasr_amd.config import paraformer_streaming_tiny
    cfg = paraformer_streaming_tiny()
    m = build_stream_ref(cfg)
    rec = _Recorder(m)
    rng = np.random.default_rng(21)
    chunks = [rng.standard_normal((10, 560), dtype=np.float32) for _ in range(8)]
    last = rng.standard_normal((7, 560), dtype=np.float32)
    out = dict(seed=21, chunks=np.stack(chunks), last=last)
    for tag, (elb, dlb), tail in (("lb00", (0, 0), False), ("lb41", (4, 1), False), ("lb41_tail", (4, 1), True)):
        cache = _stream_cache(m, elb, dlb)
        rec.enc.clear()
        toks = []
        seq = chunks + ([None] if tail else [last])
        for i, x in enumerate(seq):
            fin = i == len(seq) - 1
            if x is None:
                cache["encoder"]["tail_chunk"] = True
                t = cache["encoder"]["feats"]
            else:
                t = torch.from_numpy(x.copy())[None]
            with torch.no_grad():
                toks.append(m.generate_chunk(t, torch.tensor([t.shape[1]]), key=["k"], tokenizer=_IdsTok(),
                                             cache=cache, is_final=fin, device="cpu"))
        flat, off = pack_tokens(toks)
        enc = [e.numpy() for e in rec.enc]
        out[f"{tag}_tokens"], out[f"{tag}_off"] = flat, off
        out[f"{tag}_enc"] = np.concatenate(enc)
        out[f"{tag}_enc_off"] = np.cumsum([0] + [e.shape[0] for e in enc]).astype(np.int32)
        print(tag, [len(t) for t in toks])
    np.savez_compressed(f"{HERE}/stream_tiny.npz", **out)

    # waveform path through the reference online frontend and inference()
    import funasr.frontends.wav_frontend as wf
    from oracle import fbank_ref
    from tests.golden.inputs import waveform

    def kfbank(w, **kw):
        return torch.from_numpy(fbank_ref.fbank(w[0].numpy().astype(np.float32) / np.float32(32768.0)))

    sys.modules["torchaudio.compliance.kaldi"].fbank = kfbank
    wf.kaldi.fbank = kfbank
    front = wf.WavFrontendOnline(cmvn_file=CMVN, fs=16000, window="hamming", n_mels=80, frame_length=25,
                                 frame_shift=10, lfr_m=7, lfr_n=6, dither=0.0)
    feats_log = []
    ff = front.forward

    def front_fwd(*a, **k):
        r = ff(*a, **k)
        feats_log.append(r[0][0].numpy().copy() if r[0].numel() else np.zeros((0, 560), np.float32))
        return r

    front.forward = front_fwd
    vocab = token_list(cfg.vocab_size)

    class Tok:
        def ids2tokens(self, ids):
            return [vocab[i] for i in ids]

    wout = {}
    for tag, n_total, calls in (("w1", 57600 + 2000, [9600] * 6 + [2000]), ("w2", 48000 + 500, [19200, 28800, 500])):
        wav = waveform(seed=31 if tag == "w1" else 32, n=n_total)
        cache = {}
        texts, feats_log[:] = [], []
        pos = 0
        for j, n in enumerate(calls):
            fin = j == len(calls) - 1
            with torch.no_grad():
                res, _ = m.inference([torch.from_numpy(wav[pos:pos + n].copy())], key=["s"], tokenizer=Tok(),
                                     frontend=front, cache=cache, is_final=fin, chunk_size=[0, 10, 5],
                                     encoder_chunk_look_back=4, decoder_chunk_look_back=1,
                                     encoder_conf={"output_size": 512}, frontend_conf={"n_mels": 80, "lfr_m": 7},
                                     device="cpu", data_type="sound")
            texts.append(res[0]["text"])
            pos += n
        wout[tag] = dict(seed=31 if tag == "w1" else 32, n=n_total, calls=calls, texts=texts,
                         feat_rows=[int(f.shape[0]) for f in feats_log])
        np.save(f"{HERE}/stream_{tag}_feats.npy", np.concatenate(feats_log).astype(np.float32))
        print(tag, texts, wout[tag]["feat_rows"])
    with open(f"{HERE}/stream_wave.json", "w") as f:
        json.dump(wout, f, ensure_ascii=False, indent=1)


STREAM_BEAM_CASES = {   # name: (encoder / decoder look-back, decoding_ctc_weight, beam_size, penalty, nbest, tail chunk)
    "sb_lb00": ((0, 0), 0.3, 3, 0.0, 1, False),
    "sb_lb41_nb": ((4, 1), 0.5, 4, 0.5, 3, True),
}


def save_stream_beam():
    """ParaformerStreaming with a CTC head (model_conf ctc_weight 0.3, tiny: enc 3 / dec 2) decoded per chunk by the
    reference's joint decoder + CTC prefix beam search (generate_chunk with self.beam_search built by
    init_beam_search, paraformer_streaming/model.py:510-552, 567-575). Chunk-level: seeded LFR+CMVN chunks of 10
    frames; per chunk the generate_chunk ids (every n-best hypothesis, concatenated) and, from beam_search() itself,
    the n-best yseqs and scores. Waveform-level: inference() over 600 ms sample chunks (kaldi.fbank patched to the
    pinned restatement) with decoding_ctc_weight, as the reference's own streaming entry builds the search."""
    import dataclasses
    from funasr_amd.config import paraformer_streaming_tiny
    import funasr.models.scama.encoder  # noqa: F401
    import funasr.models.paraformer_streaming.model  # noqa: F401
    cfg = dataclasses.replace(paraformer_streaming_tiny(), ctc_weight=0.3)
    kw = cfg.reference_kwargs()

    def build():
        m = tables.model_classes["ParaformerStreaming"](
            **{k: kw[k] for k in ("encoder", "encoder_conf", "decoder", "decoder_conf", "predictor", "predictor_conf")},
            input_size=cfg.input_size, vocab_size=cfg.vocab_size, ctc_weight=0.3, predictor_bias=1)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
        m.eval()
        return m

    toks = token_list(cfg.vocab_size)
    rng = np.random.default_rng(22)
    chunks = [rng.standard_normal((10, 560), dtype=np.float32) for _ in range(8)]
    last = rng.standard_normal((7, 560), dtype=np.float32)
    out = dict(seed=22, chunks=np.stack(chunks), last=last)
    for name, ((elb, dlb), wctc, beam, pen, nbest, tail) in STREAM_BEAM_CASES.items():
        m = build()
        m.init_beam_search(token_list=toks, decoding_ctc_weight=wctc, beam_size=beam, penalty=pen)
        m.nbest = nbest
        calls = []
        fwd = m.beam_search.forward

        def spy(*a, **k):
            r = fwd(*a, **k)
            calls[-1].append([(h.yseq.tolist(), float(h.score)) for h in r[:nbest]])
            return r

        m.beam_search.forward = spy
        cache = _stream_cache(m, elb, dlb)
        ids, hyps = [], []
        seq = chunks + ([None] if tail else [last])
        for i, x in enumerate(seq):
            fin = i == len(seq) - 1
            if x is None:
                cache["encoder"]["tail_chunk"] = True
                t = cache["encoder"]["feats"]
            else:
                t = torch.from_numpy(x.copy())[None]
            calls.append([])
            with torch.no_grad():
                ids.append(m.generate_chunk(t, torch.tensor([t.shape[1]]), key=["k"], tokenizer=_IdsTok(),
                                            cache=cache, is_final=fin, device="cpu", maxlenratio=0.0,
                                            minlenratio=0.0))
            hyps.append(calls[-1][0] if calls[-1] else [])
        flat, off = pack_tokens(ids)
        yseq = [y for hs in hyps for (y, _) in hs]
        yflat, yoff = pack_tokens(yseq)
        out[f"{name}_ids"], out[f"{name}_ids_off"] = flat, off
        out[f"{name}_yseq"], out[f"{name}_yseq_off"] = yflat, yoff
        out[f"{name}_scores"] = np.array([sc for hs in hyps for (_, sc) in hs], np.float32)
        out[f"{name}_nhyp"] = np.array([len(hs) for hs in hyps], np.int32)
        out[f"{name}_opts"] = np.array([elb, dlb, beam, nbest, int(tail)], np.int32)
        out[f"{name}_fopts"] = np.array([wctc, pen], np.float32)
        print(name, "chunk ids", [len(t) for t in ids], "hyps", [len(h) for h in hyps])
    np.savez_compressed(f"{HERE}/stream_beam_tiny.npz", **out)

    # waveform path: inference() builds the search from its kwargs (model.py:567-575)
    import funasr.frontends.wav_frontend as wf
    from oracle import fbank_ref
    from tests.golden.inputs import waveform

    def kfbank(w, **k):
        return torch.from_numpy(fbank_ref.fbank(w[0].numpy().astype(np.float32) / np.float32(32768.0)))

    sys.modules["torchaudio.compliance.kaldi"].fbank = kfbank
    wf.kaldi.fbank = kfbank
    front = wf.WavFrontendOnline(cmvn_file=CMVN, fs=16000, window="hamming", n_mels=80, frame_length=25,
                                 frame_shift=10, lfr_m=7, lfr_n=6, dither=0.0)

    class Tok:
        def ids2tokens(self, ids):
            return [toks[i] for i in ids]

    m = build()
    wav = waveform(seed=33, n=57600 + 2000)
    calls = [9600] * 6 + [2000]
    cache, texts, pos = {}, [], 0
    for j, n in enumerate(calls):
        with torch.no_grad():
            res, _ = m.inference([torch.from_numpy(wav[pos:pos + n].copy())], key=["s"], tokenizer=Tok(),
                                 frontend=front, cache=cache, is_final=j == len(calls) - 1, chunk_size=[0, 10, 5],
                                 encoder_chunk_look_back=4, decoder_chunk_look_back=1,
                                 encoder_conf={"output_size": 512}, frontend_conf={"n_mels": 80, "lfr_m": 7},
                                 device="cpu", data_type="sound", token_list=toks, decoding_ctc_weight=0.4,
                                 beam_size=3, nbest=2, penalty=0.0)
        texts.append(res[0]["text"])
        pos += n
    with open(f"{HERE}/stream_beam_wave.json", "w") as f:
        json.dump(dict(seed=33, n=57600 + 2000, calls=calls, texts=texts, decoding_ctc_weight=0.4, beam_size=3,
                       nbest=2), f, ensure_ascii=False, indent=1)
    print("wave", texts)


def save_stream_large():
    """ParaformerStreaming at Paraformer-large size, greedy (config C5's model), look-back 4 / 1, 24 seeded chunks
    of 10 rows + a final 4-row chunk through the reference generate_chunk: per chunk the token ids, and per decoded
    position the decoder's top-5 log-probs (cal_decoder_with_predictor_chunk, paraformer_streaming/model.py:427-433)
    for the fast-mode regret statistics (tests/fast_parity.py)."""
    from funasr_amd.config import paraformer_streaming
    cfg = paraformer_streaming()
    m = build_stream_ref(cfg)
    rows = []
    dec = m.cal_decoder_with_predictor_chunk

    def spy(*a, **k):
        r = dec(*a, **k)
        lp, n = r[0].detach(), int(r[1][0]) if r[1] is not None else r[0].shape[1]
        v, i = torch.topk(lp[0, :n], 5, dim=-1)
        rows.append((i.numpy().astype(np.int32), v.numpy().astype(np.float32)))
        return r

    m.cal_decoder_with_predictor_chunk = spy
    rng = np.random.default_rng(26)
    ns = [10] * 24 + [4]
    chunks = [rng.standard_normal((n, 560), dtype=np.float32) for n in ns]
    cache = _stream_cache(m, 4, 1)
    toks, ntok, top_ids, top_lp = [], [], [], []
    for i, x in enumerate(chunks):
        rows.clear()
        with torch.no_grad():
            t = m.generate_chunk(torch.from_numpy(x.copy())[None], torch.tensor([x.shape[0]]), key=["k"],
                                 tokenizer=_IdsTok(), cache=cache, is_final=i == len(chunks) - 1, device="cpu")
        toks.append(t)
        if rows:
            top_ids.append(rows[0][0])
            top_lp.append(rows[0][1])
            ntok.append(rows[0][0].shape[0])
        else:
            ntok.append(0)
    flat, off = pack_tokens(toks)
    np.savez_compressed(f"{HERE}/stream_large.npz", seed=26, ns=np.array(ns, np.int32), tokens=flat, tokens_off=off,
                        ntok=np.array(ntok, np.int32),
                        top_ids=np.concatenate(top_ids) if top_ids else np.zeros((0, 5), np.int32),
                        top_logp=np.concatenate(top_lp) if top_lp else np.zeros((0, 5), np.float32))
    print("stream large: tokens per chunk", [len(t) for t in toks], "positions", sum(ntok))


def save_stream_beam_large():
    """Config C5 as benched: ParaformerStreaming at Paraformer-large size with a CTC head (ctc_weight 0.3), chunk
    [0, 10, 5], look-back 4 / 1, decoded per chunk by the reference's joint decoder + CTC prefix beam search
    (generate_chunk, decoding_ctc_weight 0.3, beam 10, nbest 2; paraformer_streaming/model.py:510-552, 567-575) on
    six seeded LFR+CMVN-like chunks and a final tail chunk. Per chunk: generate_chunk's ids and, from beam_search()
    itself, the n-best yseqs and scores, plus the decoder's per-position argmax / top-2 margin (diagnostics)."""
    import dataclasses
    from funasr_amd.config import paraformer_streaming
    import funasr.models.scama.encoder  # noqa: F401
    import funasr.models.paraformer_streaming.model  # noqa: F401
    cfg = dataclasses.replace(paraformer_streaming(), ctc_weight=0.3)
    kw = cfg.reference_kwargs()
    m = tables.model_classes["ParaformerStreaming"](
        **{k: kw[k] for k in ("encoder", "encoder_conf", "decoder", "decoder_conf", "predictor", "predictor_conf")},
        input_size=cfg.input_size, vocab_size=cfg.vocab_size, ctc_weight=0.3, predictor_bias=1)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
    m.eval()
    toks = token_list(cfg.vocab_size)
    elb, dlb, wctc, beam, pen, nbest = 4, 1, 0.3, 10, 0.0, 2
    m.init_beam_search(token_list=toks, decoding_ctc_weight=wctc, beam_size=beam, penalty=pen)
    m.nbest = nbest
    calls = []
    fwd = m.beam_search.forward

    def spy(*a, **k):
        r = fwd(*a, **k)
        calls[-1].append([(h.yseq.tolist(), float(h.score)) for h in r[:nbest]])
        return r

    m.beam_search.forward = spy
    rng = np.random.default_rng(25)
    chunks = [rng.standard_normal((10, 560), dtype=np.float32) for _ in range(6)]
    cache = _stream_cache(m, elb, dlb)
    ids, hyps = [], []
    seq = chunks + [None]
    for i, x in enumerate(seq):
        fin = i == len(seq) - 1
        if x is None:
            cache["encoder"]["tail_chunk"] = True
            t = cache["encoder"]["feats"]
        else:
            t = torch.from_numpy(x.copy())[None]
        calls.append([])
        with torch.no_grad():
            ids.append(m.generate_chunk(t, torch.tensor([t.shape[1]]), key=["k"], tokenizer=_IdsTok(), cache=cache,
                                        is_final=fin, device="cpu", maxlenratio=0.0, minlenratio=0.0))
        hyps.append(calls[-1][0] if calls[-1] else [])
        print("chunk", i, "ids", len(ids[-1]), "hyps", [(len(y), round(sc, 3)) for y, sc in hyps[-1]], flush=True)
    flat, off = pack_tokens(ids)
    yseq = [y for hs in hyps for (y, _) in hs]
    yflat, yoff = pack_tokens(yseq)
    np.savez_compressed(f"{HERE}/stream_beam_large.npz", seed=25, chunks=np.stack(chunks), ids=flat, ids_off=off,
                        yseq=yflat, yseq_off=yoff, scores=np.array([sc for hs in hyps for (_, sc) in hs], np.float32),
                        nhyp=np.array([len(hs) for hs in hyps], np.int32),
                        opts=np.array([elb, dlb, beam, nbest, 1], np.int32), fopts=np.array([wctc, pen], np.float32))


PUNC_TEXTS = {
    "short": 12,            # CJK tokens only, one mini-sentence
    "mixed": 47,            # CJK + ASCII words (split_words keeps ASCII runs as one word; unknown -> <unk>)
    "long": 260,            # > 200 tokens: several mini-sentences, the carried cache and the comma cut-off rule
}


def punc_text(name: str, n: int, vocab) -> str:
    """Seeded text of n words from the synthetic token list (CJK tokens), with ASCII words mixed in."""
    rng = np.random.default_rng(abs(hash(name)) % 1000 if False else {"short": 1, "mixed": 2, "long": 3}[name])
    cjk = vocab[3:-1]
    words = []
    for i in range(n):
        if name == "mixed" and i % 5 == 3:
            words.append(" " + ["hello", "world", "FunASR", "ok", "GPU"][i % 5] + " ")
        else:
            words.append(cjk[int(rng.integers(len(cjk)))])
    return "".join(words).strip()


def save_punc():
    """CTTransformer (tiny: 2 SAN-M blocks, vocab 4000, widths of the released model) goldens: the
    reference inference() text / punc_array for seeded texts, and every punc_forward call it made
    (mini-sentence ids -> argmax punctuation ids, logits)."""
    import funasr.models.ct_transformer.model as ctm
    import funasr.models.sanm.encoder  # noqa: F401
    from funasr.tokenizer.char_tokenizer import CharTokenizer
    from funasr_amd.config import ct_transformer_tiny
    cfg = ct_transformer_tiny()
    m = tables.model_classes["CTTransformer"](**cfg.reference_kwargs())
    w = make_weights(cfg, 0)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=True)
    m.eval()
    vocab = token_list(cfg.vocab_size)
    tok = CharTokenizer(token_list=vocab, unk_symbol="<unk>")
    calls = []
    pf = m.punc_forward

    def rec(text, text_lengths, **kw):
        y, h = pf(text, text_lengths, **kw)
        calls.append((text[0].numpy().astype(np.int32).copy(), y[0].detach().numpy().copy()))
        return y, h

    m.punc_forward = rec
    out = {}
    arrays = {}
    for name, n in PUNC_TEXTS.items():
        text = punc_text(name, n, vocab)
        calls.clear()
        with torch.no_grad():
            res, _ = m.inference([text], key=[name], tokenizer=tok, device="cpu")
        out[name] = {"text_in": text, "text": res[0]["text"], "punc_array": res[0]["punc_array"].tolist(),
                     "n_calls": len(calls)}
        arrays[f"{name}_ids"] = np.concatenate([c[0] for c in calls])
        arrays[f"{name}_off"] = np.cumsum([0] + [len(c[0]) for c in calls]).astype(np.int32)
        arrays[f"{name}_logits"] = np.concatenate([c[1] for c in calls]).astype(np.float32)
        print(name, len(calls), res[0]["text"][:60])
    with open(f"{HERE}/punc.json", "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    np.savez_compressed(f"{HERE}/punc_tiny.npz", **arrays)


VAD_SIL_BIAS = 0.0      # added to out_linear2.bias[0] (the silence pdf) of the synthetic VAD weights
VAD_SIL_SCALE = -2000.0  # out_linear2.weight[0] scale


def vad_weights(cfg, seed=0, sil_bias=None, sil_scale=None):
    """Synthetic FSMN-VAD weights whose silence logit is amplified (row 0 of out_linear2 x VAD_SIL_SCALE) so
    that p(sil) separates the loud and quiet parts of the test signal around the speech/noise threshold
    (plain random weights give p(sil) ~ 1/248 everywhere: one all-speech segment)."""
    from funasr_amd.weights import vad_test_weights
    return vad_test_weights(cfg, seed, VAD_SIL_SCALE if sil_scale is None else sil_scale,
                            VAD_SIL_BIAS if sil_bias is None else sil_bias)


VAD_CASES = {   # name: (seed, seconds, gaps, calls (samples per inference call; None = one call))
    "v1": (51, 12.0, [(2.0, 4.0), (6.5, 7.7), (10.0, 12.0)], None),
    "v2": (52, 70.0, [(0.0, 1.5), (20.0, 23.0), (50.0, 52.5), (61.0, 62.0)], None),
}


def build_vad_ref(cfg, sil_bias=None, sil_scale=None):
    import funasr.models.fsmn_vad_streaming.encoder  # noqa: F401
    import funasr.models.fsmn_vad_streaming.model  # noqa: F401
    m = tables.model_classes["FsmnVADStreaming"](**cfg.reference_kwargs())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in vad_weights(cfg, 0, sil_bias, sil_scale).items()}, strict=True)
    m.eval()
    return m


def vad_frontend():
    import funasr.frontends.wav_frontend as wf
    from oracle import fbank_ref

    def kfbank(w, **kw):
        return torch.from_numpy(fbank_ref.fbank(w[0].numpy().astype(np.float32) / np.float32(32768.0)))

    sys.modules["torchaudio.compliance.kaldi"].fbank = kfbank
    wf.kaldi.fbank = kfbank
    return wf.WavFrontendOnline(cmvn_file=None, fs=16000, window="hamming", n_mels=80, frame_length=25,
                                frame_shift=10, lfr_m=5, lfr_n=1, dither=0.0)


def run_vad_ref(m, front, wav, calls=None):
    """FsmnVADStreaming.inference (offline: chunk_size 60000 ms) -> (segments, silence posteriors, decibels)."""
    scores, decib = [], []
    cs, cd = m.ComputeScores, m.ComputeDecibel

    def cscores(feats, cache={}):
        cs(feats, cache=cache)
        scores.append(cache["stats"].scores[0, -feats.shape[1]:, 0].numpy().copy())

    def cdecib(cache={}):
        n0 = len(cache["stats"].decibel)
        cd(cache=cache)
        decib.append(np.asarray(cache["stats"].decibel[n0:], np.float64))

    m.ComputeScores, m.ComputeDecibel = cscores, cdecib
    try:
        cache = {}
        with torch.no_grad():
            res, _ = m.inference([torch.from_numpy(wav.copy())], key=["v"], frontend=front, cache=cache,
                                 device="cpu", data_type="sound")
    finally:
        m.ComputeScores, m.ComputeDecibel = cs, cd
    return (res[0]["value"], np.concatenate(scores), np.concatenate(decib),
            np.cumsum([0] + [len(x) for x in scores]).astype(np.int32),
            np.cumsum([0] + [len(x) for x in decib]).astype(np.int32))


def save_vad():
    """FsmnVADStreaming goldens (released FSMN dims, synthetic weights, silence bias VAD_SIL_BIAS): the
    reference inference() segments [[beg_ms, end_ms], ...] of seeded waveforms with quiet gaps, plus the
    per-frame silence posteriors and decibels its state machine consumed."""
    from funasr_amd.config import fsmn_vad
    cfg = fsmn_vad()
    m = build_vad_ref(cfg)
    front = vad_frontend()
    out, arrays = {}, {}
    for name, (seed, sec, gaps, calls) in VAD_CASES.items():
        from tests.golden.inputs import vad_waveform
        wav = vad_waveform(seed, sec, gaps)
        segs, p0, db, p_off, d_off = run_vad_ref(m, front, wav, calls)
        arrays[f"{name}_p0_off"], arrays[f"{name}_db_off"] = p_off, d_off
        out[name] = dict(seed=seed, seconds=sec, gaps=gaps, segments=segs, sil_bias=VAD_SIL_BIAS)
        arrays[f"{name}_p0"] = p0.astype(np.float32)
        arrays[f"{name}_db"] = db.astype(np.float64)
        print(name, segs, "p0 mean", float(p0.mean()), "frames", len(p0))
    with open(f"{HERE}/vad.json", "w") as f:
        json.dump(out, f, indent=1)
    np.savez_compressed(f"{HERE}/vad.npz", **arrays)


def save_vad_pipeline():
    """Reference AutoModel(model=Paraformer tiny, vad_model=FsmnVADStreaming, punc_model=CTTransformer tiny)
    .generate(input=waveform): inference_with_vad (VAD segments -> sorted / batched ASR -> restored order ->
    joined text -> punctuation). Synthetic weights: make_weights seed 0 (ASR, punc), vad_test_weights (VAD)."""
    import funasr.tokenizer.char_tokenizer  # noqa: F401
    import funasr.frontends.wav_frontend as wf
    import funasr.models.ct_transformer.model  # noqa: F401
    import funasr.models.fsmn_vad_streaming.model  # noqa: F401
    import funasr.models.fsmn_vad_streaming.encoder  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    from funasr_amd.config import ct_transformer_tiny, fsmn_vad
    from funasr_amd.weights import vad_test_weights
    from tests.golden.inputs import vad_waveform

    _patch_kaldi_fbank_knf()   # both frontends (the VAD's WavFrontendOnline and the ASR WavFrontend)
    cfg, pcfg, vcfg = paraformer_tiny(), ct_transformer_tiny(), fsmn_vad()
    fconf = dict(fs=16000, window="hamming", n_mels=80, frame_length=25, frame_shift=10, dither=0.0)
    vad_kwargs = dict(model_conf={}, frontend="WavFrontendOnline", frontend_conf=dict(fconf, lfr_m=5, lfr_n=1),
                      disable_update=True, **vcfg.reference_kwargs())
    punc_kwargs = dict(model_conf={}, tokenizer="CharTokenizer",
                       tokenizer_conf=dict(token_list=token_list(pcfg.vocab_size), unk_symbol="<unk>"),
                       disable_update=True, **pcfg.reference_kwargs())
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                   device="cpu", ncpu=4, disable_update=True, disable_pbar=True, disable_log=True,
                   tokenizer="CharTokenizer", tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)),
                   frontend="WavFrontend", frontend_conf=dict(fconf, lfr_m=7, lfr_n=6, cmvn_file=CMVN),
                   vad_model="FsmnVADStreaming", vad_kwargs=vad_kwargs, punc_model="CTTransformer",
                   punc_kwargs=punc_kwargs, **cfg.reference_kwargs())
    am.model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, 0).items()}, strict=True)
    am.vad_model.load_state_dict({k: torch.from_numpy(v) for k, v in vad_test_weights(vcfg, 0).items()},
                                 strict=True)
    am.punc_model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(pcfg, 0).items()}, strict=True)
    out = {}
    calls = []   # per ASR batch of the pipeline: the decoder's per-position argmax, top-2 margin and token counts
    dec = am.model.cal_decoder_with_predictor

    def spy(*a, **k):
        r = dec(*a, **k)
        logp, ntok = r[0].detach(), a[3] if len(a) > 3 else k["pre_token_length"]
        top2 = torch.topk(logp, 2, dim=-1).values
        nt = [int(n) for n in ntok]
        calls.append(dict(ntok=nt,
                          argmax=[int(t) for b in range(len(nt)) for t in logp[b, : nt[b]].argmax(-1)],
                          margin=[float(x) for b in range(len(nt)) for x in (top2[b, : nt[b], 0] - top2[b, : nt[b], 1])]))
        return r

    am.model.cal_decoder_with_predictor = spy

    class GpuLikeCpu(str):
        """device "cpu" that does not compare equal to "cpu": inference_with_vad (auto_model.py:434-435) then keeps
        the duration-packed batches it builds for a GPU device instead of decoding one segment per call, while
        torch still runs on the CPU."""
        def __eq__(self, other):
            return False if other == "cpu" else str.__eq__(self, other)

        __hash__ = str.__hash__

    for name, bs, batched in (("v1", 300, False), ("v1_b4", 4, False), ("v1_batched", 300, True)):
        gj = VAD_CASES["v1"]
        wav = vad_waveform(gj[0], gj[1], gj[2])
        calls.clear()
        am.kwargs["device"] = GpuLikeCpu("cpu") if batched else "cpu"
        res = am.generate(input=wav, batch_size_s=bs)   # (a key= kwarg collides inside inference_with_vad)
        out[name] = dict(batch_size_s=bs, batched=batched, result=[{k: (v.tolist() if hasattr(v, "tolist") else v)
                                                   for k, v in r.items()} for r in res], asr_calls=list(calls))
        print(name, out[name]["result"][0]["text"][:80])
    with open(f"{HERE}/vad_pipeline.json", "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)


def _patch_kaldi_fbank_knf():
    """Route the reference WavFrontend's kaldi.fbank to the reference's own kaldi-native-fbank, compiled from its
    sources by oracle/Makefile (oracle/_ref/knf_fbank): torchaudio is absent here, and knf is the fbank of the
    reference's C++ runtime. Returns the patched function."""
    import funasr.frontends.wav_frontend as wf
    from tests.golden.make_fbank_golden import knf

    def kfbank(w, **kw):
        return torch.from_numpy(knf(w[0].numpy().astype(np.float32) / np.float32(32768.0)))

    sys.modules["torchaudio.compliance.kaldi"].fbank = kfbank
    wf.kaldi.fbank = kfbank
    return kfbank


WAV_LARGE_CASES = [("c1", 61, 16000 * 5), ("w3", 62, 16000 * 3 + 517), ("w7", 63, 16000 * 7 + 3001)]


def save_automodel_wav_large():
    """Config C1: Paraformer-large (seeded weights), a single 5 s wav through the reference
    AutoModel.generate() on the CPU (WavFrontend with CMVN, kaldi.fbank = compiled knf), one call per wav.
    Records the result dicts and the decoder's per-position argmax / top-2 margins (diagnostics)."""
    import funasr.tokenizer.char_tokenizer  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    from tests.golden.inputs import waveform
    _patch_kaldi_fbank_knf()
    cfg = paraformer_large()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                   device="cpu", ncpu=8, disable_update=True, disable_pbar=True, disable_log=True,
                   tokenizer="CharTokenizer", tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)),
                   frontend="WavFrontend", frontend_conf=dict(fs=16000, window="hamming", n_mels=80,
                                                             frame_length=25, frame_shift=10, lfr_m=7,
                                                             lfr_n=6, dither=0.0, cmvn_file=CMVN),
                   **cfg.reference_kwargs())
    am.model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
    calls = []
    dec = am.model.cal_decoder_with_predictor

    def spy(*a, **k):
        r = dec(*a, **k)
        logp, ntok = r[0].detach(), a[3] if len(a) > 3 else k["pre_token_length"]
        top2 = torch.topk(logp, 2, dim=-1).values
        n = int(ntok[0])
        calls.append(dict(ntok=n, argmax=[int(t) for t in logp[0, :n].argmax(-1)],
                          margin=[float(x) for x in (top2[0, :n, 0] - top2[0, :n, 1])]))
        return r

    am.model.cal_decoder_with_predictor = spy
    out = {}
    for name, seed, n in WAV_LARGE_CASES:
        calls.clear()
        res = am.generate(input=waveform(seed, n), key=[name])
        out[name] = dict(seed=seed, n=n, result=[{k: (v.tolist() if hasattr(v, "tolist") else v)
                                                  for k, v in r.items()} for r in res], decoder=calls[0])
        print(name, len(res[0]["text"]), "min margin", min(calls[0]["margin"] or [0]))
    with open(f"{HERE}/automodel_wav_large.json", "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)


def _read_tree(root):
    out = {}
    for dp, _, fns in os.walk(root):
        for fn in fns:
            full = os.path.join(dp, fn)
            with open(full, encoding="utf-8") as f:
                out[os.path.relpath(full, root)] = f.read()
    return out


def save_output_dir():
    """generate(..., output_dir=d) result files (funasr/utils/datadir_writer.py, paraformer/model.py:548-591,
    sense_voice/model.py:899-915): Paraformer tiny greedy over two generate() calls (the writer is created once per
    model, so the second call appends), Paraformer tiny + CTC head with the joint beam search and nbest=2
    ({1,2}best_recog), SenseVoice tiny (1best_recog/text, the un-postprocessed decode)."""
    import dataclasses
    import tempfile
    import funasr.tokenizer.char_tokenizer  # noqa: F401
    import funasr.tokenizer.sentencepiece_tokenizer  # noqa: F401
    import funasr.models.sense_voice.model  # noqa: F401
    import funasr.frontends.wav_frontend  # noqa: F401
    from funasr.auto.auto_model import AutoModel
    from funasr_amd.config import sense_voice_tiny
    front = dict(fs=16000, window="hamming", n_mels=80, frame_length=25, frame_shift=10, lfr_m=7, lfr_n=6,
                 dither=0.0, cmvn_file=CMVN)
    common = dict(device="cpu", ncpu=4, disable_update=True, disable_pbar=True, disable_log=True,
                  frontend="WavFrontend", frontend_conf=front)
    out = {}
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    x, ln = torch.from_numpy(feats), torch.from_numpy(lens.astype(np.int32))
    # (1) greedy, two calls
    cfg = paraformer_tiny()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), tokenizer="CharTokenizer",
                   tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), **common, **cfg.reference_kwargs())
    am.model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
    with tempfile.TemporaryDirectory() as d:
        am.generate(input=x, input_len=ln[:, None], data_type="fbank", key=["uttA", "uttB"], output_dir=d)
        am.generate(input=x[1:, :27], input_len=ln[1:, None], data_type="fbank", key=["uttC"], output_dir=d)
        am.model.writer.close()
        out["greedy"] = _read_tree(d)
    # (2) joint decoder + CTC prefix beam, nbest 2
    cfg = dataclasses.replace(paraformer_tiny(), ctc_weight=0.3)
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.3, predictor_bias=1), tokenizer="CharTokenizer",
                   tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), **common, **cfg.reference_kwargs())
    am.model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=4).items()}, strict=True)
    with tempfile.TemporaryDirectory() as d:
        res = am.generate(input=x, input_len=ln[:, None], data_type="fbank", key=["uttA", "uttB"], output_dir=d,
                          decoding_ctc_weight=0.3, beam_size=3, nbest=2)
        am.model.writer.close()
        out["beam"] = _read_tree(d)
        out["beam_results"] = [{k: v for k, v in r.items()} for r in res]
    # (3) SenseVoice
    bpe = f"{HERE}/sv_bpe.model"
    cfg = sense_voice_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    am = AutoModel(model="SenseVoiceSmall", model_conf={}, tokenizer="SentencepiecesTokenizer",
                   tokenizer_conf=dict(bpemodel=bpe), encoder=kw["encoder"], encoder_conf=kw["encoder_conf"], **common)
    am.model.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}, strict=True)
    with tempfile.TemporaryDirectory() as d:
        am.generate(input=x, input_len=ln, data_type="fbank", key=["uttA", "uttB"], batch_size=2, output_dir=d)
        am.model.writer.close()
        out["sensevoice"] = _read_tree(d)
    with open(f"{HERE}/output_dir.json", "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print({k: sorted(v) if isinstance(v, dict) else len(v) for k, v in out.items()})


if __name__ == "__main__" and len(sys.argv) > 1:
    torch.manual_seed(0)
    for part in sys.argv[1:]:
        globals()["save_" + part]()
elif __name__ == "__main__":
    torch.manual_seed(0)
    save_timestamps()
    save_automodel_tiny_ts()
    save_postprocess()
    torch.set_num_threads(8)
    save_lfr_cmvn()
    save_tiny()
    save_automodel_tiny()
    m = build_ref(paraformer_large())
    save_large(m, "para_large_ragged", seed=1, B=3, T=500, lens=[500, 431, 83])
    save_large(m, "para_large_c1", seed=2, B=1, T=83, lens=[83])
    save_large(m, "para_large_b4", seed=3, B=4, T=500, lens=[500, 500, 500, 500])
