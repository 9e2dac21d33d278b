"""Joint decoder + CTC prefix beam search on the device (pfm_run_beam, k_beam.hip) against the reference's own
BeamSearchPara runs (tests/golden/beam_*.npz: Paraformer with a CTC head, ctc_weight 0.3, decoded with
decoding_ctc_weight > 0; make_golden.py save_beam).

EXACT mode: the n-best token sequences equal the reference's and their scores agree within 1e-5 relative
(tiny config); at Paraformer-large scale, where the reference's two best hypotheses differ by 2 f32 ulps
(-2223.5 vs -2223.50049), the GPU's best hypothesis must be one of the reference hypotheses within 1e-3 of the
reference's best score and every score within 1e-3 of the reference's. AutoModel / Paraformer.inference with
decoding_ctc_weight reproduces the reference inference() token_int dicts.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_large, paraformer_tiny  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.golden.inputs import fbank_input  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cfg(g):
    base = paraformer_large() if bool(g["large"]) else paraformer_tiny()
    return dataclasses.replace(base, ctc_weight=0.3)


def _golden(g):
    off = g["yseq_off"]
    hyps = [g["yseq"][off[k]:off[k + 1]].tolist() for k in range(len(off) - 1)]
    return hyps, g["scores"], g["owner"]


def _strip(y, cfg):
    return [t for t in y[1:-1] if t not in (cfg.eos, cfg.sos, cfg.blank_id)]


def _weights(g, cfg):
    """The golden's weights: seeded, plus the eos boost on the decoder output bias of beam_tiny_nb."""
    w = make_weights(cfg, int(g["wseed"]))
    boost = float(g["eos_boost"]) if "eos_boost" in g else 0.0
    if boost:
        w["decoder.output_layer.bias"] = w["decoder.output_layer.bias"].copy()
        w["decoder.output_layer.bias"][cfg.eos] += boost
    return w


def _engine(g):
    from funasr_amd.runtime import PfmEngine
    cfg = _cfg(g)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(_weights(g, cfg))
    return e, cfg


def _run(e, g, mode="exact"):
    feats, lens = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
    r = e.run_beam(torch.from_numpy(feats).cuda(), torch.from_numpy(lens).cuda(), mode=mode,
                   beam=int(g["beam_size"]), ctc_weight=float(g["decoding_ctc_weight"]), penalty=float(g["penalty"]),
                   nbest=int(g["nbest"]))
    torch.cuda.synchronize()
    return r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy(), r["scores"].cpu().numpy()


# beam_tiny_nb: beam 2, nbest 5, decoding_ctc_weight 0.01 and an eos-biased decoder, so hypotheses end at many
# positions and the reference's sorted(ended_hyps)[:nbest] holds five per utterance (more than the beam)
@pytest.mark.parametrize("name", ["beam_tiny", "beam_tiny_pen", "beam_tiny_nb"])
def test_beam_exact_vs_reference(name):
    g = np.load(f"{GOLD}/{name}.npz")
    e, cfg = _engine(g)
    toks, nt, sc = _run(e, g)
    hyps, scores, owner = _golden(g)
    nbest = int(g["nbest"])
    k = 0
    for i in range(int(g["B"])):
        for n in range(nbest):
            if k < len(owner) and owner[k] == i:
                assert nt[i, n] >= 0
                assert toks[i, n, : nt[i, n]].tolist() == _strip(hyps[k], cfg), (i, n)
                assert abs(sc[i, n] - scores[k]) <= 1e-5 * abs(scores[k]), (i, n, sc[i, n], scores[k])
                k += 1
            else:
                assert nt[i, n] == -1
    assert k == len(owner)


def _oracle_logprobs(g, cfg):
    """The oracle model's decoder log-probs [B, L, V] and CTC log-probs [B, T, V] (zero past each utterance's
    frames) on the golden's inputs: the arrays the reference's beam search consumed (test_oracle_golden.py pins
    the oracle search on them to the reference's n-best)."""
    from oracle.beam_ref import ctc_log_probs
    from oracle.paraformer_ref import paraformer_infer
    w = _weights(g, cfg)
    feats, lens = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
    r = paraformer_infer(feats, lens, w, cfg, keep_logits=True)
    logp = torch.log_softmax(r["logits"], dim=-1)
    B, T = int(g["B"]), int(g["T"])
    x = torch.zeros(B, T, cfg.vocab_size)
    for i in range(B):
        n = int(r["enc_lens"][i])
        x[i, :n] = ctc_log_probs(r["enc"][i, :n], w)
    return logp, x, torch.as_tensor(r["enc_lens"]).int(), torch.as_tensor(r["ntok"]).int()


@pytest.mark.parametrize("name", ["beam_tiny", "beam_tiny_pen", "beam_tiny_nb"])
def test_beam_kernel_on_reference_logprobs(name):
    """The search kernel alone (pfm_op_ctc_beam) on the oracle model's log-probs: the reference's n-best token
    sequences and scores (1e-5 relative) — separates the search from the model's arithmetic."""
    from funasr_amd.runtime import op_ctc_beam
    g = np.load(f"{GOLD}/{name}.npz")
    cfg = _cfg(g)
    logp, x, elens, ntok = _oracle_logprobs(g, cfg)
    nbest = int(g["nbest"])
    toks, nt, sc = op_ctc_beam(logp.cuda(), x.cuda(), elens.cuda(), ntok.cuda(), int(g["beam_size"]),
                               float(g["decoding_ctc_weight"]), float(g["penalty"]), nbest, cfg.sos, cfg.eos,
                               cfg.blank_id)
    toks, nt, sc = toks.cpu().numpy(), nt.cpu().numpy(), sc.cpu().numpy()
    hyps, scores, owner = _golden(g)
    k = 0
    for i in range(int(g["B"])):
        for n in range(nbest):
            if k < len(owner) and owner[k] == i:
                assert toks[i, n, : nt[i, n]].tolist() == _strip(hyps[k], cfg), (i, n, sc[i, n], scores[k])
                assert abs(sc[i, n] - scores[k]) <= 1e-5 * abs(scores[k]), (i, n, sc[i, n], scores[k])
                k += 1
    assert k == len(owner)


def test_beam_exact_large_vs_reference():
    g = np.load(f"{GOLD}/beam_large.npz")
    e, cfg = _engine(g)
    toks, nt, sc = _run(e, g)
    hyps, scores, owner = _golden(g)
    for i in range(int(g["B"])):
        ref = [(hyps[k], scores[k]) for k in range(len(owner)) if owner[k] == i]
        best = max(s for _, s in ref)
        near = [_strip(y, cfg) for y, s in ref if s >= best - 1e-3]
        assert toks[i, 0, : nt[i, 0]].tolist() in near, i
        for n in range(len(ref)):
            got = toks[i, n, : nt[i, n]].tolist()
            match = [s for y, s in ref if _strip(y, cfg) == got]
            assert match and abs(sc[i, n] - match[0]) <= 1e-3, (i, n, sc[i, n], match)


def test_beam_fast_mode_runs_and_is_close():
    """fast (bf16) mode: same API; the best hypothesis shares >= 90 % of its positions with the exact one."""
    g = np.load(f"{GOLD}/beam_tiny.npz")
    e, _ = _engine(g)
    te, ne, _ = _run(e, g, "exact")
    tf, nf, sf = _run(e, g, "fast")
    assert np.all(np.isfinite(sf[nf >= 0]))
    for i in range(int(g["B"])):
        a, b = te[i, 0, : ne[i, 0]], tf[i, 0, : nf[i, 0]]
        n = min(len(a), len(b))
        assert abs(len(a) - len(b)) <= 1 and (n == 0 or np.mean(a[:n] == b[:n]) >= 0.9)


def test_automodel_beam_matches_reference_inference():
    """Paraformer.inference(decoding_ctc_weight=..., beam_size, penalty, nbest) -> the reference inference()
    result dicts (one {"key", "token_int"} per n-best hypothesis, utterance order)."""
    from funasr_amd.model import Paraformer
    for name in ("beam_tiny", "beam_tiny_pen", "beam_tiny_nb"):
        g = np.load(f"{GOLD}/{name}.npz")
        cfg = _cfg(g)
        kw = cfg.reference_kwargs()
        m = Paraformer(**kw, ctc_weight=0.3, predictor_bias=1, mode="exact").cuda()
        m.load_state_dict(_weights(g, cfg))
        feats, lens = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
        res, _ = m.inference(torch.from_numpy(feats), data_lengths=torch.from_numpy(lens)[:, None],
                             key=[f"utt{i}" for i in range(int(g["B"]))], data_type="fbank",
                             decoding_ctc_weight=float(g["decoding_ctc_weight"]), beam_size=int(g["beam_size"]),
                             penalty=float(g["penalty"]), nbest=int(g["nbest"]))
        roff = g["result_off"]
        want = [g["result_tokens"][roff[k]:roff[k + 1]].tolist() for k in range(len(roff) - 1)]
        assert [r["token_int"] for r in res] == want, name
        assert [r["key"] for r in res] == [f"utt{int(o)}" for o in g["owner"]]


def test_beam_barrier_timeout_is_an_error(monkeypatch):
    """A search whose cross-workgroup arrival barrier times out (forced: PFM_BEAM_SPIN_CAP=0) fails the call with
    PFM_E_DEVICE instead of returning 'no hypothesis' rows; the same engine decodes normally afterwards."""
    from funasr_amd.runtime import PfmError
    g = np.load(f"{GOLD}/beam_tiny.npz")
    e, cfg = _engine(g)
    feats, lens = fbank_input(seed=int(g["seed"]), B=int(g["B"]), T=int(g["T"]), lens=g["lens"])
    x, l = torch.from_numpy(feats).cuda(), torch.from_numpy(lens).cuda()
    kw = dict(mode="exact", beam=int(g["beam_size"]), ctc_weight=float(g["decoding_ctc_weight"]),
              penalty=float(g["penalty"]), nbest=int(g["nbest"]))
    monkeypatch.setenv("PFM_BEAM_SPIN_CAP", "0")
    with pytest.raises(PfmError, match="barrier"):
        e.run_beam(x, l, **kw)
    monkeypatch.delenv("PFM_BEAM_SPIN_CAP")
    r = e.run_beam(x, l, **kw)
    assert int((r["ntok"][:, 0] >= 0).sum()) == int(g["B"])


def test_beam_rejects_bad_arguments():
    from funasr_amd.runtime import PfmEngine, PfmError
    g = np.load(f"{GOLD}/beam_tiny.npz")
    e, _ = _engine(g)
    x, l = torch.zeros(1, 10, 560).cuda(), torch.tensor([10], dtype=torch.int32).cuda()
    with pytest.raises(PfmError):
        e.run_beam(x, l, beam=3, nbest=17)   # the kernel keeps at most 16 ended hypotheses (nbest > beam is legal)
    with pytest.raises(PfmError):
        e.run_beam(x, l, beam=17)
    with pytest.raises(PfmError):
        e.run_beam(x, l, beam=3, ctc_weight=0.0)
    plain = PfmEngine(paraformer_tiny(), 0)   # no CTC head
    plain.load_state_dict(make_weights(paraformer_tiny(), 0))
    with pytest.raises(PfmError):
        plain.run_beam(x, l, beam=2)


@pytest.mark.parametrize("seed,B,T,L,V,beam,pen", [(3, 4, 100, 40, 500, 5, 0.0), (4, 3, 64, 30, 300, 8, 0.5),
                                                    (5, 2, 120, 50, 2000, 10, 0.0)])
def test_beam_kernel_random_logprobs_vs_oracle(seed, B, T, L, V, beam, pen):
    """The search kernel alone (pfm_op_ctc_beam) against the oracle restatement (oracle/beam_ref.py, pinned to the
    reference's beam_search goldens) on identical seeded log-probs over a grid of sizes, beams and length bonuses:
    the same n-best token sequences, scores within 1e-5 relative. Ragged frame / token counts per utterance."""
    from funasr_amd.runtime import op_ctc_beam
    from oracle.beam_ref import beam_search
    g = torch.Generator().manual_seed(seed)
    am = torch.log_softmax(torch.randn(B, L, V, generator=g) * 2.5, -1)
    x = torch.log_softmax(torch.randn(B, T, V, generator=g) * 2.5, -1)
    lens = torch.tensor([T - 13 * i for i in range(B)], dtype=torch.int32)
    ntok = torch.tensor([L - 7 * i for i in range(B)], dtype=torch.int32)
    sos, eos = V - 1, V - 2
    nbest = min(3, beam)
    toks, nt, sc = op_ctc_beam(am.cuda(), x.cuda(), lens.cuda(), ntok.cuda(), beam, 0.3, pen, nbest, sos, eos, 0)
    toks, nt, sc = toks.cpu().numpy(), nt.cpu().numpy(), sc.cpu().numpy()
    for i in range(B):
        hyps = beam_search(am[i, : int(ntok[i])].numpy(), x[i, : int(lens[i])].numpy(), beam, 0.3, pen, sos, eos)
        for n in range(nbest):
            if n >= len(hyps):
                assert nt[i, n] == -1
                continue
            want = [t for t in hyps[n].yseq[1:-1] if t not in (eos, sos, 0)]
            assert toks[i, n, : nt[i, n]].tolist() == want, (i, n)
            assert abs(sc[i, n] - float(hyps[n].score)) <= 1e-5 * abs(float(hyps[n].score)), (i, n)
