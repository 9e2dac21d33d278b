"""SenseVoiceSmall (BASELINE config C4) through the C-ABI (pfm_run_ctc) against goldens captured
from the reference SenseVoiceSmall.inference (tests/golden/make_golden.py sv_tiny / sv_large).

EXACT mode (f32 MFMA): encoder rel-L2 <= 1e-5 (tiny, full tensors), row slices <= 1e-4 abs (large),
per-frame argmax identical wherever the reference's top-2 log-prob margin is >= 1e-4 (f32 rounding
of a different summation order can only flip closer frames), and token ids identical.
FAST mode (bf16 MFMA, f32 accumulate/residual): encoder rel-L2 <= 2e-2, frame agreement reported
and floored (random weights leave small CTC margins).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import sense_voice_small, sense_voice_tiny  # noqa: E402
from funasr_amd.runtime import PfmEngine, op_ctc_collapse  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.golden.inputs import fbank_input  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MARGIN = 1e-4


def _tok(g, flat="tokens", off="tokens_off"):
    o = g[off]
    return [g[flat][o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]


def _weights(cfg, boost=None):
    w = make_weights(cfg, seed=0)
    if boost:
        b = w["ctc.ctc_lo.bias"].copy()
        for t, a in boost.items():
            b[t] += np.float32(a)
        w["ctc.ctc_lo.bias"] = b
    return w


def _query(cfg, language="auto", use_itn=False, text_norm=None):
    if text_norm is None:
        text_norm = "withitn" if use_itn else "woitn"
    return [cfg.lid_dict.get(language, 0), 1, 2, cfg.textnorm_dict[text_norm]]


def _run(e, g, mode, **kw):
    x, l = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
    q = _query(e.cfg, **{k: v for k, v in kw.items() if k != "ban"})
    return e.run_ctc(torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda(), q, mode=mode,
                     ban_token=e.cfg.emo_unk if kw.get("ban") else -1, want_enc=True, want_frames=True)


def _tokens(r):
    toks, nt = r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy()
    return [toks[b, : nt[b]].tolist() for b in range(toks.shape[0])]


def _frames_close(fr, g_fr, lens, margin):
    """Frame argmax equal on every frame whose reference margin >= MARGIN; returns #close-call flips."""
    flips, k = 0, 0
    for b in range(len(lens)):
        n = int(lens[b]) + 4
        a, w = fr[b, :n], g_fr[b, :n]
        m = margin[k:k + n]
        k += n
        bad = a != w
        assert not np.any(bad & (m >= MARGIN)), (b, np.nonzero(bad & (m >= MARGIN))[0][:10])
        flips += int(bad.sum())
        assert np.all(fr[b, n:] == -1)
    return flips


@pytest.fixture(scope="module")
def sv():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = {}
    for name, cfg in (("tiny", sense_voice_tiny()), ("large", sense_voice_small())):
        e = PfmEngine(cfg, 0)
        e.load_state_dict(make_weights(cfg, seed=0))
        out[name] = e
    return out


def test_tiny_exact_full_tensors(sv):
    e = sv["tiny"]
    g = np.load(f"{GOLD}/sv_tiny.npz")
    r = _run(e, g, "exact")
    torch.cuda.synchronize()
    enc = r["enc"].cpu().numpy()
    for b, n in enumerate(g["enc_lens"]):
        d = enc[b, :n] - g["enc"][b, :n]
        assert np.linalg.norm(d) / np.linalg.norm(g["enc"][b, :n]) < 1e-5
    assert _frames_close(r["frame_ids"].cpu().numpy(), g["frame_ids"], g["lens"], g["margin"]) == 0
    assert _tokens(r) == _tok(g)
    r = _run(e, g, "exact", language="zh", use_itn=True)
    assert _tokens(r) == _tok(g, "zh_itn_tokens", "zh_itn_off")


def test_tiny_exact_blank_heavy_and_ban(sv):
    """Blank-dominated frames exercise the collapse; a +50 bias on <|unk|> emotion (25009) makes it every
    frame's argmax unless ban_emo_unk excludes it (model.py:885-886)."""
    cfg = sense_voice_tiny()
    g = np.load(f"{GOLD}/sv_tiny.npz")
    e = PfmEngine(cfg, 0)
    e.load_state_dict(_weights(cfg, {0: 2.5}))
    r = _run(e, g, "exact", language="en", text_norm="withitn")
    torch.cuda.synchronize()
    _frames_close(r["frame_ids"].cpu().numpy(), g["blank_frame_ids"], g["lens"], g["blank_margin"])
    assert _tokens(r) == _tok(g, "blank_tokens", "blank_off")
    e.load_state_dict(_weights(cfg, {25009: 50.0}))
    assert _tokens(_run(e, g, "exact")) == _tok(g, "emo_tokens", "emo_off")
    r = _run(e, g, "exact", ban=True)
    assert _tokens(r) == _tok(g, "ban_tokens", "ban_off")
    assert not np.any(r["frame_ids"].cpu().numpy() == 25009)
    r = _run(e, g, "fast", ban=True)
    assert not np.any(r["frame_ids"].cpu().numpy() == 25009)


@pytest.mark.parametrize("name", ["sv_large_ragged", "sv_large_c1"])
def test_large_exact(sv, name):
    e = sv["large"]
    g = np.load(f"{GOLD}/{name}.npz")
    r = _run(e, g, "exact")
    torch.cuda.synchronize()
    enc = r["enc"].cpu().numpy()
    ol = g["enc_lens"]
    rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(len(ol))])
    assert np.abs(rows - g["enc_rows"]).max() < 1e-4
    for b in range(len(ol)):
        s = enc[b, : int(ol[b])].astype(np.float64)
        assert abs((s ** 2).sum() - g["enc_sumsq"][b]) < 1e-5 * g["enc_sumsq"][b]
    flips = _frames_close(r["frame_ids"].cpu().numpy(), g["frame_ids"], g["lens"], g["margin"])
    print(f"{name}: exact-mode close-call frame flips {flips}")
    if flips == 0:
        assert _tokens(r) == _tok(g)


# ---------------------------------------------------------------- BASELINE config C4 itself
# sv_large_b64 = the bench's SenseVoice leg (B=64 x 500 frames), sv_large_b24 a ragged batch: reference runs
# (make_golden.py save_sv_headline). Group rows B/2 x 504 >= 4096 engage the fused out-projection + FFN kernel with
# SenseVoice's LayerNorm eps 1e-5 through all 70 layers (50 + the 20 tp layers), and the next layer's QKV fold.
SV_HEADLINE = ["sv_large_b24", "sv_large_b64"]
# fast-mode frame-decision bounds (tests/fast_parity.py; tools/fast_parity_calib.py, profiles/r04_fast_parity_calib.json):
# the default fast dispatch gives mean regret 9e-5 nat, flips at 2 % of the frames, 95-96 % of them to the reference's
# second-best id, max regret 0.024, none outside the top 3; a 0.1-nat perturbation of the CTC head bias gives mean
# regret 0.034 and 11 % of the frames outside the top 3
SV_FAST_BOUNDS = dict(mean_regret=1e-3, flip_frac=0.05, outside_frac=1e-3, max_regret=0.1, second_best=0.9)


def sv_fast_violations(st, bounds=SV_FAST_BOUNDS):
    bad = []
    for k in ("mean_regret", "flip_frac", "max_regret"):
        if st[k] >= bounds[k]:
            bad.append(f"{k} {st[k]:.4g} >= {bounds[k]}")
    if st["outside_topk"] >= bounds["outside_frac"] * st["positions"]:
        bad.append(f"{st['outside_topk']} frames outside the reference top 3")
    if st["second_best"] < bounds["second_best"]:
        bad.append(f"only {st['second_best']:.3f} of the flips to the second-best id")
    return bad


@pytest.mark.parametrize("name", SV_HEADLINE)
def test_headline_exact(sv, name):
    """EXACT mode at C4: per-frame CTC argmax identical wherever the reference's top-2 margin is >= 1e-4 (0 flips
    measured at all), token ids identical, encoder rows < 1e-4 abs and per-utterance sums of squares < 1e-5 rel."""
    e = sv["large"]
    g = np.load(f"{GOLD}/{name}.npz")
    r = _run(e, g, "exact")
    torch.cuda.synchronize()
    enc = r["enc"].cpu().numpy()
    ol = g["enc_lens"]
    rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(len(ol))])
    assert np.abs(rows - g["enc_rows"]).max() < 1e-4
    for b in range(len(ol)):
        s = enc[b, : int(ol[b])].astype(np.float64)
        assert abs((s ** 2).sum() - g["enc_sumsq"][b]) < 1e-5 * g["enc_sumsq"][b]
    flips = _frames_close(r["frame_ids"].cpu().numpy(), g["frame_ids"], g["lens"], g["margin"])
    got, want = _tokens(r), _tok(g)
    bad = [b for b in range(len(want)) if got[b] != want[b]]
    print(f"{name} exact: {flips} close-call frame flips, {len(bad)} utterances with different tokens")
    assert flips > 0 or not bad, bad[:5]
    assert len(bad) <= flips


@pytest.mark.parametrize("name", SV_HEADLINE)
def test_headline_fast_default_dispatch(sv, name):
    """FAST mode, default dispatch, at C4: encoder rows within bf16 tolerance (rel-L2 < 2e-2) and the CTC frame
    decisions within SV_FAST_BOUNDS of the reference's own log-probs."""
    from tests.fast_parity import frame_stats
    e = sv["large"]
    g = np.load(f"{GOLD}/{name}.npz")
    r = _run(e, g, "fast")
    torch.cuda.synchronize()
    enc = r["enc"].cpu().numpy()
    ol = g["enc_lens"]
    rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(len(ol))])
    rel = np.linalg.norm(rows - g["enc_rows"]) / np.linalg.norm(g["enc_rows"])
    st = frame_stats(r["frame_ids"].cpu().numpy(), ol, g)
    print(f"{name} fast: enc rows rel-L2 {rel:.2e}; {st}")
    assert rel < 2e-2, rel
    assert not sv_fast_violations(st), sv_fast_violations(st)


def test_headline_fast_bounds_catch_a_ctc_shift():
    """The SenseVoice fast bounds can fail: the CTC head bias moved by N(0, 0.1) nat per id breaks them at C4."""
    from tests.fast_parity import frame_stats
    cfg = sense_voice_small()
    w = make_weights(cfg, seed=0)
    rng = np.random.default_rng(123)
    w["ctc.ctc_lo.bias"] = (w["ctc.ctc_lo.bias"] + 0.1 * rng.standard_normal(w["ctc.ctc_lo.bias"].shape)).astype(np.float32)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(w)
    g = np.load(f"{GOLD}/sv_large_b64.npz")
    r = _run(e, g, "fast")
    torch.cuda.synchronize()
    st = frame_stats(r["frame_ids"].cpu().numpy(), g["enc_lens"], g)
    print(f"perturbed CTC head, fast: {st}")
    assert sv_fast_violations(st), st


@pytest.mark.parametrize("name", ["sv_large_ragged"])
def test_large_fast_agreement(sv, name):
    e = sv["large"]
    g = np.load(f"{GOLD}/{name}.npz")
    r = _run(e, g, "fast")
    torch.cuda.synchronize()
    enc = r["enc"].cpu().numpy()
    ol = g["enc_lens"]
    rows = np.stack([enc[b, [0, 3, 4, int(ol[b]) // 2, int(ol[b]) - 1]] for b in range(len(ol))])
    rel = np.linalg.norm(rows - g["enc_rows"]) / np.linalg.norm(g["enc_rows"])
    assert rel < 2e-2, rel
    fr = r["frame_ids"].cpu().numpy()
    agree = np.mean(np.concatenate([fr[b, : ol[b]] == g["frame_ids"][b, : ol[b]] for b in range(len(ol))]))
    print(f"SenseVoice fast-mode frame agreement {agree:.4f}, enc rows rel {rel:.2e}")
    assert agree > 0.6


def test_ctc_collapse_op_matches_unique_consecutive():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    """unique_consecutive + drop blank on frames with long repeats, blanks, ragged lengths, an empty
    utterance and L_cap truncation (sense_voice/model.py:894-906)."""
    rng = np.random.default_rng(3)
    B, T = 6, 700
    ids = rng.integers(0, 5, size=(B, T)).astype(np.int32)
    ids[1] = np.repeat(rng.integers(0, 3, size=T // 7), 7)   # runs of 7 equal ids
    ids[2] = 0
    ids[3, ::2] = 0
    olen = np.array([700, 699, 650, 64, 0, 65], dtype=np.int32)
    want = []
    for b in range(B):
        y = torch.unique_consecutive(torch.from_numpy(ids[b, : olen[b]]))
        want.append(y[y != 0].tolist())
    tok, nt = op_ctc_collapse(torch.from_numpy(ids).cuda(), torch.from_numpy(olen).cuda(), blank=0, L_cap=T)
    tok, nt = tok.cpu().numpy(), nt.cpu().numpy()
    for b in range(B):
        assert nt[b] == len(want[b])
        assert tok[b, : nt[b]].tolist() == want[b]
        assert np.all(tok[b, nt[b]:] == -1)
    tok, nt = op_ctc_collapse(torch.from_numpy(ids).cuda(), torch.from_numpy(olen).cuda(), blank=0, L_cap=10)
    tok, nt = tok.cpu().numpy(), nt.cpu().numpy()
    for b in range(B):
        assert nt[b] == len(want[b])
        assert tok[b].tolist() == (want[b] + [-1] * 10)[:10]


def test_sensevoice_deterministic(sv):
    e = sv["large"]
    g = np.load(f"{GOLD}/sv_large_c1.npz")
    r1, r2 = _run(e, g, "fast"), _run(e, g, "fast")
    torch.cuda.synchronize()
    assert torch.equal(r1["tokens"], r2["tokens"]) and torch.equal(r1["enc"], r2["enc"])


def _sv_automodel():
    from funasr_amd.auto_model import AutoModel
    cfg = sense_voice_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    return AutoModel(model="SenseVoiceSmall", model_conf={}, synthetic_seed=0, tokenizer="SentencepiecesTokenizer",
                     tokenizer_conf=dict(bpemodel=os.path.join(GOLD, "sv_bpe.model")), device="cuda", mode="exact",
                     encoder=kw["encoder"], encoder_conf=kw["encoder_conf"])


def test_automodel_sensevoice_matches_reference_generate():
    """AutoModel(model="SenseVoiceSmall").generate(fbank, language/use_itn) returns the reference's
    result dicts (text = sentencepiece decode of the collapsed CTC ids)."""
    import json
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    am = _sv_automodel()
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    want = json.load(open(f"{GOLD}/automodel_sv_tiny.json", encoding="utf-8"))
    for tag, opts in (("auto", {}), ("en_itn", dict(language="en", use_itn=True))):
        res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens), data_type="fbank",
                          key=["uttA", "uttB"], batch_size=2, **opts)
        assert res == want[tag], tag


def test_automodel_sensevoice_waveform_path():
    """Waveform input: pfm_fbank -> LFR/CMVN -> pfm_run_ctc; tokens equal the oracle's on the same
    features except near-tie frames (the fbank agrees with knf to ~1e-4, not bit-exactly)."""
    from oracle import fbank_ref
    from oracle.sensevoice_ref import sensevoice_infer
    from tests.golden.inputs import waveform
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    am = _sv_automodel()
    wavs = [waveform(41, 16000 * 2), waveform(42, 16000 * 4 + 77)]
    res = am.generate(input=wavs, batch_size=2, key=["a", "b"])
    assert [r["key"] for r in res] == ["a", "b"]
    cfg = sense_voice_tiny(vocab_size=300)
    feats = [fbank_ref.frontend(w) for w in wavs]
    T = max(f.shape[0] for f in feats)
    x = np.zeros((2, T, 560), np.float32)
    for i, f in enumerate(feats):
        x[i, : f.shape[0]] = f
    r = sensevoice_infer(x, np.array([f.shape[0] for f in feats]), make_weights(cfg), cfg)
    tok = am.kwargs["tokenizer"]
    for got, want_ids in zip([x["text"] for x in res], r["tokens"]):
        want = tok.decode(want_ids)
        n = min(len(got), len(want))
        assert sum(a == b for a, b in zip(got[:n], want[:n])) >= 0.8 * max(len(got), len(want))


def test_oversized_lengths_are_clamped(sv):
    """fbank lengths > T (and < 0) behave as min(max(len, 0), T), as every other length consumer clamps:
    the collapse never reads past an utterance's [T + 4] id row (pfm_run_ctc does not validate lens)."""
    e = sv["tiny"]
    g = np.load(f"{GOLD}/sv_tiny.npz")
    x, l = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
    T = x.shape[1]
    xs = torch.from_numpy(x).cuda()
    q = _query(e.cfg)
    big = torch.tensor([T + 1000, T + 7][: x.shape[0]], dtype=torch.int32).cuda()
    ok = torch.full((x.shape[0],), T, dtype=torch.int32).cuda()
    r1 = e.run_ctc(xs, big, q, mode="exact", want_frames=True)
    r0 = e.run_ctc(xs, ok, q, mode="exact", want_frames=True)
    torch.cuda.synchronize()
    assert torch.equal(r1["ntok"], r0["ntok"]) and torch.equal(r1["tokens"], r0["tokens"])
    assert torch.equal(r1["frame_ids"], r0["frame_ids"])


def _ts_model(bias):
    from funasr_amd.sense_voice import SenseVoiceSmall
    cfg = sense_voice_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    m = SenseVoiceSmall(encoder=kw["encoder"], encoder_conf=kw["encoder_conf"], input_size=cfg.input_size,
                        vocab_size=cfg.vocab_size, mode="exact").cuda()
    m.load_state_dict(_weights(cfg, {int(k): v for k, v in (bias or {}).items()}))
    return m


def test_ctc_align_kernel_vs_reference():
    """pfm_ctc_align (the forced alignment of output_timestamp) on the GPU encoder output reproduces the
    alignments the reference's ctc_forced_align returned in inference(output_timestamp=True)
    (tests/golden/sv_timestamps.npz, tiny config, vocab 300, one utterance per call)."""
    import json
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = np.load(f"{GOLD}/sv_timestamps.npz")
    want = json.load(open(f"{GOLD}/sv_timestamps.json", encoding="utf-8"))
    for k, w in enumerate(want):
        m = _ts_model(w["bias"])
        eng = m.engine()
        x, l = fbank_input(w["seed"], 1, w["T"], [w["T"]])
        r = eng.run_ctc(torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda(), _query(eng.cfg), mode="exact",
                        want_enc=True)
        ids = _tokens(r)[0]
        assert ids[4:] == g[f"sv{k}_targets"].tolist(), k
        align = eng.ctc_align(r["enc"], torch.from_numpy(l).cuda() + 4, [ids[4:]]).cpu().numpy()
        assert np.array_equal(align[0, : w["T"]], g[f"sv{k}_align"]), (k, align[0, : w["T"]], g[f"sv{k}_align"])


def test_sensevoice_output_timestamp_matches_reference():
    """SenseVoiceSmall.inference(output_timestamp=True) returns the reference's result dicts: text and the
    word-level [start ms, end ms] list (model.py:917-965), including a blank-heavy utterance with one word."""
    import json
    from funasr_amd.text import SentencepiecesTokenizer
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    tok = SentencepiecesTokenizer(bpemodel=os.path.join(GOLD, "sv_bpe.model"))
    want = json.load(open(f"{GOLD}/sv_timestamps.json", encoding="utf-8"))
    for w in want:
        m = _ts_model(w["bias"])
        x, l = fbank_input(w["seed"], 1, w["T"], [w["T"]])
        res, _ = m.inference(torch.from_numpy(x), data_lengths=torch.from_numpy(l), key=[w["key"]], tokenizer=tok,
                             data_type="fbank", output_timestamp=True)
        assert res == [{"key": w["key"], "text": w["text"], "timestamp": w["timestamp"]}], w["seed"]


def test_ctc_align_ragged_batch_equals_single_calls():
    """A ragged batch aligns each utterance on its own frames: the same alignments as one call per utterance."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = _ts_model(None)
    eng = m.engine()
    x, l = fbank_input(51, 3, 50, [50, 33, 18])
    r = eng.run_ctc(torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda(), _query(eng.cfg), mode="exact",
                    want_enc=True)
    ids = _tokens(r)
    a = eng.ctc_align(r["enc"], torch.from_numpy(l).cuda() + 4, [t[4:] for t in ids]).cpu().numpy()
    for i in range(3):
        n = int(l[i])
        ri = eng.run_ctc(torch.from_numpy(x[i:i + 1, :n].copy()).cuda(), torch.from_numpy(l[i:i + 1]).cuda(),
                         _query(eng.cfg), mode="exact", want_enc=True)
        assert _tokens(ri)[0] == ids[i]
        ai = eng.ctc_align(ri["enc"], torch.from_numpy(l[i:i + 1]).cuda() + 4, [ids[i][4:]]).cpu().numpy()
        assert np.array_equal(a[i, :n], ai[0, :n]), i
        assert np.all(a[i, n:] == -1)
