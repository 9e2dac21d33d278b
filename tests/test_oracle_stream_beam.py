"""CPU pin of the oracle for streaming + CTC prefix beam (config C5 as named): oracle/streaming_ref.chunk_step (the
chunk encoder / CIF / decoder restatement) feeding oracle/beam_ref.beam_search with the chunk's decoder log-probs and
its encoder window's CTC log-probs reproduces, chunk by chunk, the n-best yseqs and scores the reference's own
BeamSearchPara returned inside generate_chunk (tests/golden/stream_beam_tiny.npz, make_golden.py save_stream_beam).
Scores within 1e-4 (f32 sums over the chunk's positions, computed in a different operation order upstream of the
search); yseqs identical. The GPU path (pfm_stream_step_beam) is held to the same goldens in test_gpu_stream_beam.py.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from funasr_amd.config import paraformer_streaming_tiny
from funasr_amd.weights import make_weights

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["sb_lb00", "sb_lb41_nb"])
def test_oracle_stream_beam_vs_reference(name):
    from oracle.beam_ref import beam_search, ctc_log_probs
    from oracle.streaming_ref import StreamState, chunk_step
    cfg = dataclasses.replace(paraformer_streaming_tiny(), ctc_weight=0.3)
    w = {k: torch.from_numpy(v) for k, v in make_weights(cfg, seed=0).items()}
    g = np.load(f"{GOLD}/stream_beam_tiny.npz")
    elb, dlb, beam, nbest, tail = g[f"{name}_opts"].tolist()
    wctc, pen = g[f"{name}_fopts"].tolist()
    yoff, nh = g[f"{name}_yseq_off"], g[f"{name}_nhyp"]
    hoff = np.concatenate([[0], np.cumsum(nh)])
    st = StreamState(cfg, (0, 10, 5), elb, dlb)
    seq = list(g["chunks"]) + ([None] if tail else [g["last"]])
    decoded = 0
    for i, x in enumerate(seq):
        fin = i == len(seq) - 1
        if x is None:
            st.tail_chunk = True
        r = chunk_step(x, st, w, cfg, fin, keep=True)
        want = [g[f"{name}_yseq"][yoff[q]:yoff[q + 1]].tolist() for q in range(hoff[i], hoff[i + 1])]
        if r["ntok"] < 1:
            assert want == [], i
            continue
        am = torch.log_softmax(r["logits"], -1).numpy()
        xc = ctc_log_probs(r["enc"], w).numpy()
        hyps = beam_search(am, xc, beam, wctc, pen, cfg.sos, cfg.eos, cfg.blank_id)[:nbest]
        assert [h.yseq for h in hyps] == want, (name, i)
        np.testing.assert_allclose([float(h.score) for h in hyps], g[f"{name}_scores"][hoff[i]:hoff[i + 1]],
                                   atol=1e-4, rtol=1e-5)
        decoded += 1
    assert decoded >= len(seq) - 1
