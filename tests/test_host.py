"""Host-side logic on CPU: weight layout, config plumbing, tokenizer / post-processing vs the reference's
outputs, CMVN parsing, input normalisation, and fail-loud behaviour without a GPU."""
import json
import os

import numpy as np
import pytest
import torch

from funasr_amd.config import ParaformerConfig, paraformer_large, paraformer_tiny
from funasr_amd.text import CharTokenizer, sentence_postprocess
from funasr_amd.weights import gen_tensor, make_weights, num_params, param_layout
from tests.golden.inputs import token_list

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_param_count_and_keys():
    cfg = paraformer_large()
    assert num_params(cfg) == 220_084_533
    keys = [k for k, _, _ in param_layout(cfg)]
    assert len(keys) == 956 and len(set(keys)) == 956
    assert "encoder.encoders0.0.self_attn.linear_q_k_v.weight" in keys
    assert "decoder.decoders3.0.feed_forward.w_2.weight" in keys
    shapes = {k: s for k, s, _ in param_layout(cfg)}
    assert shapes["encoder.encoders0.0.self_attn.linear_q_k_v.weight"] == (1536, 560)
    assert shapes["predictor.cif_conv1d.weight"] == (512, 512, 3)
    assert shapes["decoder.output_layer.weight"] == (8404, 512)


def test_weight_generator_is_deterministic_and_independent():
    a = gen_tensor(0, "x.weight", (4, 8), 8)
    b = gen_tensor(0, "x.weight", (4, 8), 8)
    c = gen_tensor(1, "x.weight", (4, 8), 8)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert np.abs(a).max() <= 1 / np.sqrt(8)
    w = make_weights(paraformer_tiny())
    assert np.allclose(w["encoder.after_norm.weight"].mean(), 1.0, atol=0.02)


def test_config_from_reference_kwargs_roundtrip():
    cfg = paraformer_tiny()
    kw = cfg.reference_kwargs()
    back = ParaformerConfig.from_kwargs(**kw)
    assert back == cfg
    with pytest.raises(ValueError):
        ParaformerConfig.from_kwargs(encoder_conf={"input_layer": "conv2d"})
    with pytest.raises(ValueError):
        ParaformerConfig.from_kwargs(decoder_conf={"num_blocks": 16, "att_layer_num": 12})


def test_postprocess_matches_reference():
    for case in json.load(open(f"{GOLD}/postprocess.json", encoding="utf-8")):
        sent, words = sentence_postprocess(case["tokens"])
        assert sent == case["sentence"], case
        assert words == case["words"], case


def test_char_tokenizer():
    tl = token_list(8404)
    tok = CharTokenizer(token_list=tl)
    assert tok.get_num_vocabulary_size() == 8404
    ids = [3, 4, 10]
    toks = tok.ids2tokens(ids)
    assert toks == [tl[3], tl[4], tl[10]]
    assert tok.tokens2ids(toks) == ids
    assert tok.tokens2text(["a", "<space>", "b"]) == "a b"


def test_char_tokenizer_from_files(tmp_path):
    p = tmp_path / "tokens.json"
    p.write_text(json.dumps(["<blank>", "<s>", "</s>", "你", "<unk>"]), encoding="utf-8")
    assert CharTokenizer(token_list=str(p)).ids2tokens([3]) == ["你"]
    q = tmp_path / "tokens.txt"
    q.write_text("<blank>\n<s>\n</s>\n好\n<unk>\n", encoding="utf-8")
    assert CharTokenizer(token_list=str(q)).ids2tokens([3]) == ["好"]


def test_load_cmvn_vs_reference():
    from funasr_amd.frontend import load_cmvn
    g = np.load(f"{GOLD}/lfr_cmvn.npz")
    ref = "/root/reference/runtime/triton_gpu/model_repo_paraformer_large_online/lfr_cmvn_pe/am.mvn"
    if not os.path.exists(ref):
        pytest.skip("reference am.mvn not present (GPU box)")
    assert np.array_equal(load_cmvn(ref), g["cmvn"])


def test_load_cmvn_synthetic(tmp_path):
    from funasr_amd.frontend import load_cmvn
    p = tmp_path / "am.mvn"
    p.write_text("<Nnet>\n<Splice> 4 4\n[ 0 ]\n<AddShift> 4 4\n<LearnRateCoef> 0 [ 1 2 3 4 ]\n"
                 "<Rescale> 4 4\n<LearnRateCoef> 0 [ 0.5 0.25 2 1 ]\n</Nnet>\n")
    c = load_cmvn(str(p))
    assert c.shape == (2, 4) and c[0, 2] == 3 and c[1, 1] == 0.25


def test_read_wav_roundtrip(tmp_path):
    import wave
    from funasr_amd.frontend import read_wav
    x = (np.sin(np.arange(1600) / 10) * 20000).astype("<i2")
    p = tmp_path / "a.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(x.tobytes())
    y = read_wav(str(p))
    assert np.array_equal(y, x.astype(np.float32) / 32768.0)


def test_prepare_data_iterator(tmp_path):
    from funasr_amd.auto_model import prepare_data_iterator
    scp = tmp_path / "wav.scp"
    scp.write_text("u1 /a/b.wav\nu2 /c/d.wav\n")
    keys, items = prepare_data_iterator(str(scp))
    assert keys == ["u1", "u2"] and items == ["/a/b.wav", "/c/d.wav"]
    t = torch.zeros(2, 10, 560)
    keys, items = prepare_data_iterator(t, key="k")
    assert keys == ["k"] and items[0] is t
    keys, items = prepare_data_iterator([np.zeros(5), np.zeros(6)])
    assert len(keys) == 2 and all(k.startswith("rand_key_") for k in keys)


def test_model_state_dict_contract():
    from funasr_amd.model import Paraformer
    cfg = paraformer_tiny()
    m = Paraformer(**cfg.reference_kwargs())
    sd = m.state_dict()
    assert set(sd) == {k for k, _, _ in param_layout(cfg)}
    assert len(list(m.parameters())) >= 1
    m.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg).items()})
    with pytest.raises(RuntimeError):
        m.load_state_dict({"encoder.after_norm.weight": torch.zeros(3)}, strict=True)


def test_ctc_head_checkpoint_needs_ctc_weight():
    """A checkpoint with ctc.ctc_lo into a model built with ctc_weight 0.0 (a config.yaml that leaves it out;
    the reference's constructor default is 0.5 and keeps the head): strict load names the fix, a non-strict load
    warns; built with ctc_weight > 0 the same checkpoint loads strictly."""
    import dataclasses
    from funasr_amd.model import Paraformer
    cfg = dataclasses.replace(paraformer_tiny(), ctc_weight=0.3)
    sd = {k: torch.from_numpy(v) for k, v in make_weights(cfg).items()}
    assert "ctc.ctc_lo.weight" in sd
    m0 = Paraformer(**paraformer_tiny().reference_kwargs(), ctc_weight=0.0)
    with pytest.raises(RuntimeError, match="ctc_weight"):
        m0.load_state_dict(sd, strict=True)
    with pytest.warns(UserWarning, match="ctc_weight"):
        m0.load_state_dict(sd, strict=False)
    m1 = Paraformer(**paraformer_tiny().reference_kwargs(), ctc_weight=0.3)
    m1.load_state_dict(sd, strict=True)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly():
    from funasr_amd.auto_model import AutoModel
    from funasr_amd.model import Paraformer
    from funasr_amd.runtime import PfmEngine, PfmError
    with pytest.raises(PfmError):
        PfmEngine(paraformer_tiny(), 0)
    with pytest.raises(RuntimeError):
        AutoModel(model="Paraformer", synthetic_seed=0)
    m = Paraformer(**paraformer_tiny().reference_kwargs())
    with pytest.raises(PfmError):
        m.inference(torch.zeros(1, 10, 560), data_type="fbank")


def test_registry():
    from funasr_amd import tables
    import funasr_amd.model  # noqa: F401
    assert "Paraformer" in tables.model_classes


def test_timestamps_match_reference():
    """ts_prediction_lfr6_standard restatement vs the reference on seeded CIF weights (both fire-search
    branches, '</s>', VAD offset, upsample 1/3): identical text and [start_ms, end_ms] lists."""
    from funasr_amd.timestamp import ts_prediction_lfr6_standard
    g = json.load(open(os.path.join(GOLD, "timestamps.json"), encoding="utf-8"))
    for c in g["ts_prediction"]:
        txt, ts = ts_prediction_lfr6_standard(torch.tensor(c["peaks"], dtype=torch.float32),
                                              torch.tensor(c["alphas"], dtype=torch.float32), list(c["chars"]),
                                              vad_offset=c["vad_offset"], upsample_rate=c["upsample_rate"])
        assert txt == c["text"]
        assert ts == c["timestamp"]


def test_postprocess_with_timestamps_matches_reference():
    g = json.load(open(os.path.join(GOLD, "timestamps.json"), encoding="utf-8"))
    for c in g["postprocess_ts"]:
        if "error" in c:   # the reference raises on these inputs; so must the restatement
            with pytest.raises(Exception):
                sentence_postprocess(list(c["tokens"]), [[100 * i, 100 * i + 80] for i in range(len(c["tokens"]))])
            continue
        sent, ts, words = sentence_postprocess(list(c["tokens"]), c["spans"])
        assert (sent, ts, words) == (c["sentence"], c["timestamp"], c["words"]), c["tokens"]


def test_sensevoice_state_dict_contract_and_registry():
    from funasr_amd import tables
    from funasr_amd.config import sense_voice_small, sense_voice_tiny
    from funasr_amd.sense_voice import SenseVoiceSmall
    assert tables.model_classes["SenseVoiceSmall"] is SenseVoiceSmall
    cfg = sense_voice_tiny(vocab_size=300)
    m = SenseVoiceSmall(**cfg.reference_kwargs())
    assert m.cfg == cfg
    assert set(m.state_dict()) == {k for k, _, _ in param_layout(cfg)}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in make_weights(cfg).items()})
    assert m.query_ids() == [0, 1, 2, 15]
    assert m.query_ids("zh", use_itn=True) == [3, 1, 2, 14]
    assert m.query_ids("xx", text_norm="withitn") == [0, 1, 2, 14]
    from funasr_amd.weights import num_params
    assert num_params(sense_voice_small()) == 233_999_167


def test_sentencepiece_tokenizer_and_build_tokenizer():
    from funasr_amd.auto_model import build_tokenizer
    from funasr_amd.text import CharTokenizer, SentencepiecesTokenizer
    bpe = os.path.join(GOLD, "sv_bpe.model")
    tok, vocab = build_tokenizer(None, dict(bpemodel=bpe))
    assert isinstance(tok, SentencepiecesTokenizer) and vocab == 300
    ids = tok.encode("loto rito hona")
    assert tok.decode(ids) == "loto rito hona"
    tok2, v2 = build_tokenizer("CharTokenizer", dict(token_list=["<blank>", "<s>", "</s>", "a", "<unk>"]))
    assert isinstance(tok2, CharTokenizer) and v2 == 5
    assert build_tokenizer(None, {}) == (None, -1)


def test_datadir_writer_semantics(tmp_path):
    """funasr_amd.writer.DatadirWriter behaves as funasr/utils/datadir_writer.py: nested dirs created on first write,
    "key value" lines flushed at once, a duplicated key warns, a file writer refuses children."""
    import warnings
    from funasr_amd.writer import DatadirWriter
    w = DatadirWriter(tmp_path / "out")
    w["1best_recog"]["text"]["a"] = "x y"
    assert (tmp_path / "out" / "1best_recog" / "text").read_text(encoding="utf-8") == "a x y\n"
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        w["1best_recog"]["text"]["a"] = "z"
    assert any("Duplicated" in str(r.message) for r in rec)
    with pytest.raises(RuntimeError):
        w["1best_recog"]["text"]["sub"]
    with pytest.raises(RuntimeError):
        w["1best_recog"]["k"] = "v"
    w.close()
    assert (tmp_path / "out" / "1best_recog" / "text").read_text(encoding="utf-8") == "a x y\na z\n"


def test_postprocessed_texts_equal_sentence_postprocess():
    """CharTokenizer.postprocessed_texts (the vectorised greedy-result path of Paraformer.inference) and its matrix
    form postprocessed_texts_matrix equal sentence_postprocess(ids2tokens(ids))[0] row for row: all-Chinese rows (the
    fast path), rows with ASCII words, BPE pieces, single-letter runs, specials, spaces and empty rows (the general
    path)."""
    import numpy as np
    from funasr_amd.text import CharTokenizer, sentence_postprocess
    vocab = ["<blank>", "<s>", "</s>", "一", "丁", "中", "国", "1", "23", "@", "a", "b", "C", "hello", "wor@@", "ld",
             "<unk>", "<OOV>", "'", "x y", "é", "<s>中", "，", "9a"]
    tok = CharTokenizer(token_list=vocab)
    rng = np.random.default_rng(3)
    rows = [[], [1], [16, 17], [3, 4, 5], [3, 16, 4], [7, 8, 9, 3]]
    for _ in range(4000):
        n = int(rng.integers(0, 12))
        hi = 10 if rng.random() < 0.5 else len(vocab)
        rows.append([int(v) for v in rng.integers(1, hi, n)])
    want = [sentence_postprocess(tok.ids2tokens(r))[0] for r in rows]
    assert tok.postprocessed_texts(rows) == want
    # the matrix form: rows toks[i, :ntok[i]] minus blank / sos / eos (a count past the width: an empty row)
    B, L = 600, 14
    toks = rng.integers(0, len(vocab), (B, L)).astype(np.int32)
    toks[:200] = rng.integers(0, 10, (200, L))    # mostly the one-character / simple fast path
    ntok = rng.integers(0, L + 3, B).astype(np.int32)
    rows_m = [[int(t) for t in toks[i, :ntok[i]] if t not in (0, 1, 2)] if ntok[i] <= L else [] for i in range(B)]
    assert tok.postprocessed_texts_matrix(toks, ntok, (2, 1, 0)) == [sentence_postprocess(tok.ids2tokens(r))[0]
                                                                     for r in rows_m]
