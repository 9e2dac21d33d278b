"""pfm_fbank (fbank -> LFR -> CMVN on the MI355X) against the reference's C++ kaldi-native-fbank
(tests/golden/fbank_knf.npz) and the reference apply_lfr / apply_cmvn semantics; plus the
AutoModel.generate() contract end to end (fbank and waveform inputs)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_tiny  # noqa: E402
from oracle import fbank_ref  # noqa: E402
from tests.golden.inputs import fbank_input, token_list, waveform  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# pfm_fbank follows knf's float / double boundaries (sequential f32 DC mean, f64 FFT, f32 power and mel
# sums in knf's order, run-time logf mel table); only the final log differs: the GPU rounds the f64 log
# once (correctly rounded) where glibc's logf is off by an ulp on ~0.03 % of energies. So: bit-identical
# on >= 99.9 % of entries, and no entry further than 1e-6 relative (one f32 ulp of a log-mel value).
MIN_BITEXACT = 0.999
TOL_REL = 1e-6


def _check_close(got, want, what, scale=None):
    """scale: the CMVN scale row when the features went through (x + shift) * scale -- an ulp of the log-mel x
    is then judged against |x| * scale, not against the (possibly cancelled) output."""
    got, want = np.asarray(got, np.float32), np.asarray(want, np.float32)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    if got.size == 0:
        return
    frac = float((got == want).mean())
    assert frac >= MIN_BITEXACT, (what, frac)
    if scale is None:
        rel = float((np.abs(got - want) / np.maximum(np.abs(want), 1e-3)).max())
        assert rel <= TOL_REL, (what, rel)
    else:
        err = float(np.abs(got - want).max())
        assert err <= 2 * TOL_REL * 30.0 * float(np.abs(scale).max()), (what, err)


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from funasr_amd.runtime import PfmEngine
    return PfmEngine(paraformer_tiny(), 0)


def _wavs():
    g = np.load(f"{GOLD}/fbank_knf.npz")
    wavs, refs = [], []
    for i in range(7):
        wavs.append(waveform(int(g[f"syn{i}_seed"]), int(g[f"syn{i}_n"])))
        refs.append(g[f"syn{i}_fbank"])
    wavs.append(g["mid_pcm"].astype(np.float32) / 32768.0)
    refs.append(g["mid_fbank"])
    return wavs, refs


@pytest.mark.parametrize("with_cmvn", [False, True])
def test_fbank_lfr_cmvn_batch(engine, with_cmvn):
    wavs, refs = _wavs()
    cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"] if with_cmvn else None
    S = max(len(w) for w in wavs)
    buf = np.zeros((len(wavs), S), np.float32)
    for i, w in enumerate(wavs):
        buf[i, : len(w)] = w
    ns = np.array([len(w) for w in wavs], np.int32)
    feats, tout = engine.fbank(torch.from_numpy(buf).cuda(), torch.from_numpy(ns).cuda(), cmvn)
    torch.cuda.synchronize()
    feats, tout = feats.cpu().numpy(), tout.cpu().numpy()
    for i, ref in enumerate(refs):
        want = fbank_ref.apply_lfr(ref)
        if cmvn is not None:
            want = fbank_ref.apply_cmvn(want, cmvn)
        T = want.shape[0]
        assert tout[i] == T, (i, tout[i], T)
        _check_close(feats[i, :T], want, i, None if cmvn is None else cmvn[1])
        assert np.all(feats[i, T:] == 0)


def test_fbank_single_long(engine):
    w = waveform(7, 480000)   # 30 s -> 2998 frames -> 500 LFR frames (C2 shape)
    feats, tout = engine.fbank(torch.from_numpy(w[None]).cuda(), torch.tensor([480000], dtype=torch.int32).cuda())
    torch.cuda.synchronize()
    want = fbank_ref.frontend(w)
    assert int(tout[0]) == 500 == want.shape[0]
    got = feats[0].cpu().numpy()
    _check_close(got, want, "30 s")
    assert float((got == want).mean()) >= 0.9999   # the oracle rounds the log the same way


def _automodel(**extra):
    from funasr_amd.auto_model import AutoModel
    cfg = paraformer_tiny()
    kw = cfg.reference_kwargs()
    return AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                     tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), device="cuda", mode="exact",
                     **kw, **extra)


def test_automodel_fbank_matches_reference_generate():
    am = _automodel()
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens)[:, None],
                      data_type="fbank", key=["uttA", "uttB"])
    want = json.load(open(f"{GOLD}/automodel_tiny.json", encoding="utf-8"))
    assert res == want


def test_automodel_pred_timestamp_matches_reference_generate():
    """generate(..., pred_timestamp=True): text + word timestamps equal the reference's result dicts
    (CIF peaks / alphas from pfm_run, exact mode)."""
    am = _automodel()
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens)[:, None],
                      data_type="fbank", key=["uttA", "uttB"], pred_timestamp=True)
    want = json.load(open(f"{GOLD}/automodel_tiny_ts.json", encoding="utf-8"))
    assert res == want


def test_automodel_bpe_tokenizer_matches_reference_generate():
    """Paraformer with a SentencepiecesTokenizer (bpemodel): the reference keeps text =
    tokens2text(ids2tokens(ids)) and skips sentence_postprocess (paraformer/model.py:567-586)."""
    from funasr_amd.auto_model import AutoModel
    cfg = paraformer_tiny(vocab_size=300)
    kw = cfg.reference_kwargs()
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                   tokenizer="SentencepiecesTokenizer", tokenizer_conf=dict(bpemodel=f"{GOLD}/sv_bpe.model"),
                   device="cuda", mode="exact", **kw)
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    res = am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens)[:, None],
                      data_type="fbank", key=["uttA", "uttB"])
    want = json.load(open(f"{GOLD}/automodel_tiny_bpe.json", encoding="utf-8"))
    assert res == want
    with pytest.raises(UnboundLocalError):   # the reference's bpemodel + pred_timestamp branch
        am.generate(input=torch.from_numpy(feats), input_len=torch.from_numpy(lens)[:, None],
                    data_type="fbank", key=["uttA", "uttB"], pred_timestamp=True)
