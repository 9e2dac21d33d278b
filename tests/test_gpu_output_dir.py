"""generate(..., output_dir=d): the result files the reference writes through DatadirWriter
(funasr/utils/datadir_writer.py; paraformer/model.py:548-591 {n}best_recog/{token,text}; sense_voice/model.py:899-915
1best_recog/text), compared byte for byte with a reference run (tests/golden/output_dir.json, make_golden.py
save_output_dir): greedy over two calls (one writer per model: the second call appends), the joint CTC beam search
with nbest 2, SenseVoice."""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_tiny, sense_voice_tiny  # noqa: E402
from tests.golden.inputs import fbank_input, token_list  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _tree(root):
    out = {}
    for dp, _, fns in os.walk(root):
        for fn in fns:
            full = os.path.join(dp, fn)
            with open(full, encoding="utf-8") as f:
                out[os.path.relpath(full, root)] = f.read()
    return out


@pytest.fixture(scope="module")
def want():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return json.load(open(f"{GOLD}/output_dir.json", encoding="utf-8"))


def _inputs():
    feats, lens = fbank_input(seed=11, B=2, T=40, lens=[40, 27])
    return torch.from_numpy(feats), torch.from_numpy(lens.astype(np.int32))


def _paraformer(cfg, seed, ctc_weight):
    from funasr_amd.auto_model import AutoModel
    return AutoModel(model="Paraformer", model_conf=dict(ctc_weight=ctc_weight, predictor_bias=1), synthetic_seed=seed,
                     tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), device="cuda", mode="exact",
                     **cfg.reference_kwargs())


def test_output_dir_greedy_two_calls(want, tmp_path):
    x, ln = _inputs()
    am = _paraformer(paraformer_tiny(), 0, 0.0)
    am.generate(input=x, input_len=ln[:, None], data_type="fbank", key=["uttA", "uttB"], output_dir=str(tmp_path))
    am.generate(input=x[1:, :27], input_len=ln[1:, None], data_type="fbank", key=["uttC"], output_dir=str(tmp_path))
    am.model.writer.close()
    assert _tree(tmp_path) == want["greedy"]


def test_output_dir_beam_nbest(want, tmp_path):
    x, ln = _inputs()
    cfg = dataclasses.replace(paraformer_tiny(), ctc_weight=0.3)
    am = _paraformer(cfg, 4, 0.3)
    res = am.generate(input=x, input_len=ln[:, None], data_type="fbank", key=["uttA", "uttB"],
                      output_dir=str(tmp_path), decoding_ctc_weight=0.3, beam_size=3, nbest=2)
    am.model.writer.close()
    assert res == want["beam_results"]
    assert _tree(tmp_path) == want["beam"]


def test_output_dir_sensevoice(want, tmp_path):
    from funasr_amd.auto_model import AutoModel
    x, ln = _inputs()
    kw = sense_voice_tiny(vocab_size=300).reference_kwargs()
    am = AutoModel(model="SenseVoiceSmall", model_conf={}, synthetic_seed=0, tokenizer="SentencepiecesTokenizer",
                   tokenizer_conf=dict(bpemodel=os.path.join(GOLD, "sv_bpe.model")), device="cuda", mode="exact",
                   encoder=kw["encoder"], encoder_conf=kw["encoder_conf"])
    am.generate(input=x, input_len=ln, data_type="fbank", key=["uttA", "uttB"], batch_size=2, output_dir=str(tmp_path))
    am.model.writer.close()
    assert _tree(tmp_path) == want["sensevoice"]
