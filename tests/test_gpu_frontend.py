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
# log-mel abs tolerance vs knf (f64 FFT, f32 mel sums in knf order); see DESIGN.md
TOL_LOGMEL = 2e-4


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
        scale = 1.0 if cmvn is None else float(np.abs(cmvn[1]).max())
        assert np.abs(feats[i, :T] - want).max() < TOL_LOGMEL * scale, i
        assert np.all(feats[i, T:] == 0)


def test_fbank_single_long(engine):
    w = waveform(7, 480000)   # 30 s -> 2998 frames -> 500 LFR frames (C2 shape)
    feats, tout = engine.fbank(torch.from_numpy(w[None]).cuda(), torch.tensor([480000], dtype=torch.int32).cuda())
    torch.cuda.synchronize()
    want = fbank_ref.frontend(w)
    assert int(tout[0]) == 500 == want.shape[0]
    assert np.abs(feats[0].cpu().numpy() - want).max() < TOL_LOGMEL


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
