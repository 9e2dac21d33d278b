"""FSMN-VAD on the GPU: pfm_vad_run (the FSMN encoder with HBM memory caches) vs the
oracle (oracle/vad_ref.py, pinned to the reference posteriors), the online frontend at LFR (5, 1) vs the
oracle frontend, and FsmnVADStreaming.inference / AutoModel segments vs the reference inference() goldens.

Tolerances: posteriors on identical features within 1e-4 (the test weights amplify the silence logit
x2000, see funasr_amd.weights.vad_test_weights); frontend rows within 2e-4 (log-mel, as
tests/test_gpu_frontend.py); segments exact.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import fsmn_vad  # noqa: E402
from funasr_amd.weights import vad_test_weights  # noqa: E402
from tests.golden.inputs import vad_waveform  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def vad():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from funasr_amd.runtime import PfmEngine, PfmVad
    from funasr_amd.config import paraformer_tiny
    cfg = fsmn_vad()
    w = vad_test_weights(cfg, 0)
    v = PfmVad(cfg, 0)
    v.load_state_dict(w)
    eng = PfmEngine(paraformer_tiny(), 0)   # any handle serves the frontend ops
    return cfg, v, w, eng


def test_vad_encoder_chunks_vs_oracle(vad):
    """Three chunks through one stream (caches carried across chunks, including a 7-row chunk shorter
    than the memory order 20)."""
    from oracle.vad_ref import vad_forward
    cfg, v, w, _ = vad
    rng = np.random.default_rng(2)
    v.reset()
    cache = None
    for T in (300, 7, 129):
        x = (rng.standard_normal((T, cfg.input_dim)) * 3).astype(np.float32)
        p, probs = v.run(torch.from_numpy(x).cuda(), want_probs=True)
        torch.cuda.synchronize()
        ref, cache = vad_forward(x, w, cfg, cache)
        np.testing.assert_allclose(probs.cpu().numpy(), ref.numpy(), atol=1e-4, rtol=0)
        np.testing.assert_allclose(p.cpu().numpy(), ref[:, 0].numpy(), atol=1e-4, rtol=0)


@pytest.mark.parametrize("name", ["v1", "v2"])
def test_vad_frontend_and_posteriors(vad, name):
    """Online frontend (LFR 5/1) rows vs the oracle frontend; posteriors of those rows vs the oracle."""
    from funasr_amd.frontend import WavFrontendOnline
    from oracle.streaming_ref import FrontendOnline
    from oracle.vad_ref import vad_forward
    cfg, v, w, eng = vad
    gj = json.load(open(f"{GOLD}/vad.json"))[name]
    wav = vad_waveform(gj["seed"], gj["seconds"], gj["gaps"])
    fe, fo = WavFrontendOnline(cmvn_file=None, lfr_m=5, lfr_n=1), FrontendOnline(None, lfr_m=5, lfr_n=1)
    stride = 60000 * 16
    n = len(wav) // stride + 1
    cache, fc = None, {}
    v.reset()
    for i in range(n):
        seg, fin = wav[i * stride:(i + 1) * stride], i == n - 1
        got = fe.step(eng, [(seg, fin, fc)])[0]
        ref = fo(seg, fin)
        assert got.shape[0] == ref.shape[0]
        assert np.abs(got.cpu().numpy() - ref).max() < 2e-4
        p = v.run(got)
        torch.cuda.synchronize()
        pr, cache = vad_forward(got.cpu().numpy(), w, cfg, cache)
        np.testing.assert_allclose(p.cpu().numpy(), pr[:, 0].numpy(), atol=1e-4, rtol=0)


@pytest.mark.parametrize("name", ["v1", "v2"])
def test_automodel_vad_segments_vs_reference(name):
    from funasr_amd.auto_model import AutoModel
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = fsmn_vad()
    am = AutoModel(model="FsmnVADStreaming", model_conf={}, device="cuda", mode="exact",
                   frontend_conf=dict(lfr_m=5, lfr_n=1), **cfg.reference_kwargs())
    am.model.load_state_dict(vad_test_weights(cfg, 0))
    gj = json.load(open(f"{GOLD}/vad.json"))[name]
    wav = vad_waveform(gj["seed"], gj["seconds"], gj["gaps"])
    res = am.generate(input=wav, key=name)
    assert res[0]["key"] == name
    assert res[0]["value"] == gj["segments"]


@pytest.mark.parametrize("name", ["v1_batched", "v1_b4"])
def test_automodel_vad_asr_punc_pipeline_vs_reference(name):
    """AutoModel(model=Paraformer, vad_model=FsmnVADStreaming, punc_model=CTTransformer).generate(wav):
    the reference inference_with_vad result text (VAD segments -> duration-sorted batches of
    batch_size_s -> ASR -> restored order -> joined text -> punctuation)."""
    from funasr_amd.auto_model import AutoModel
    from funasr_amd.config import ct_transformer_tiny, paraformer_tiny
    from funasr_amd.weights import make_weights
    from tests.golden.inputs import token_list
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg, pcfg, vcfg = paraformer_tiny(), ct_transformer_tiny(), fsmn_vad()
    cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
    vad_kwargs = dict(model_conf={}, frontend="WavFrontendOnline", frontend_conf=dict(lfr_m=5, lfr_n=1),
                      **vcfg.reference_kwargs())
    punc_kwargs = dict(model_conf={}, tokenizer="CharTokenizer", synthetic_seed=0,
                       tokenizer_conf=dict(token_list=token_list(pcfg.vocab_size), unk_symbol="<unk>"),
                       **pcfg.reference_kwargs())
    am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                   tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), device="cuda", mode="exact",
                   vad_model="FsmnVADStreaming", vad_kwargs=vad_kwargs, punc_model="CTTransformer",
                   punc_kwargs=punc_kwargs, **cfg.reference_kwargs())
    am.kwargs["frontend"].cmvn = cmvn
    am.vad_model.load_state_dict(vad_test_weights(vcfg, 0))
    gj = json.load(open(f"{GOLD}/vad_pipeline.json", encoding="utf-8"))[name]
    wav = vad_waveform(51, 12.0, [(2.0, 4.0), (6.5, 7.7), (10.0, 12.0)])
    res = am.generate(input=wav, batch_size_s=gj["batch_size_s"])
    assert len(res) == 1
    assert set(res[0]) == set(gj["result"][0])
    want = gj["result"][0]["text"]
    # v1_batched: batch_size_s=300 packs the three segments into one ragged batch, as the reference does on a GPU
    # device (its CPU run decodes one segment per call, auto_model.py:434-435: golden "v1", whose text differs from
    # the batched reference's by one near-tie token); v1_b4: batch_size_s=4, one segment per batch. The goldens'
    # frontends are the reference's compiled kaldi-native-fbank (make_golden.py _patch_kaldi_fbank_knf), which
    # pfm_fbank reproduces to float rounding (test_gpu_frontend.py), so wav -> text is asserted end to end.
    assert res[0]["text"] == want, (res[0]["text"], want)


def test_frame_energy_bit_identical_to_numpy(vad):
    """pfm_vad_frame_energy (ComputeDecibel's frame energies on the device, fsmn_vad_streaming/model.py:326-348)
    equals numpy's float32 np.sum(np.square(frames), axis=1) bit for bit -- numpy's pairwise summation order --
    on speech-like, silent, loud, tiny and odd-length chunks, and the decibels the VAD derives from them equal the
    host statement's (VadDetector.frame_decibels, the reference's numpy code)."""
    from funasr_amd.vad import VadDetector
    _, v, _, _ = vad
    rng = np.random.default_rng(11)
    waves = [vad_waveform(61, 7.3, [(1.0, 2.5), (4.0, 4.4)]),
             np.zeros(16000, np.float32),
             (rng.standard_normal(48000) * 0.9).astype(np.float32),
             (rng.standard_normal(20011) * 1e-4).astype(np.float32),
             rng.uniform(-1, 1, 399).astype(np.float32),
             rng.uniform(-1, 1, 400).astype(np.float32),
             rng.uniform(-1, 1, 963).astype(np.float32)]
    det = VadDetector(dict(fsmn_vad().vad_opts))
    for w in waves:
        fr = np.lib.stride_tricks.sliding_window_view(w, 400)[::160] if len(w) >= 400 else np.zeros((0, 400), np.float32)
        want = np.sum(np.square(fr), axis=1).astype(np.float32)
        got = v.frame_energy(w)
        assert got.dtype == np.float32 and got.shape == want.shape
        assert np.array_equal(got.view(np.int32), want.view(np.int32)), len(w)
        db = 10 * np.log10(got + 0.000001)
        assert np.array_equal(db, det.frame_decibels(w))
