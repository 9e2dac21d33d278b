"""Streaming Paraformer with the CTC prefix beam (config C5 as named: "streaming ... with CTC prefix-beam"):
pfm_stream_step_beam vs the reference generate_chunk with its BeamSearchPara (tests/golden/stream_beam_tiny.npz,
paraformer_streaming/model.py:510-552 and init_beam_search, paraformer/model.py:396-441), and the model's
inference() over waveform calls vs the reference inference() with decoding_ctc_weight (stream_beam_wave.json).

EXACT mode: every chunk's n-best token sequences identical to the reference's, scores within 1e-4 (f32 sums over
the chunk's positions), the chunk's concatenated ids (what generate_chunk returns) identical.
"""
import dataclasses
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_streaming_tiny  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DROP = (0, 1, 2)   # blank, sos, eos of the tiny vocabulary


def _cfg():
    return dataclasses.replace(paraformer_streaming_tiny(), ctc_weight=0.3)


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from funasr_amd.runtime import PfmEngine
    cfg = _cfg()
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    return cfg, e


def _hyps(r, i):
    """n-best token lists of stream i (hypotheses with ntok -1 absent)."""
    nt = r["ntok"][i].tolist()
    return [r["tokens"][i, q, :n].tolist() for q, n in enumerate(nt) if n >= 0]


@pytest.mark.parametrize("name", ["sb_lb00", "sb_lb41_nb"])
def test_stream_beam_golden(eng, name):
    from funasr_amd.runtime import PfmStreams
    cfg, e = eng
    g = np.load(f"{GOLD}/stream_beam_tiny.npz")
    elb, dlb, beam, nbest, tail = g[f"{name}_opts"].tolist()
    wctc, pen = g[f"{name}_fopts"].tolist()
    s = PfmStreams(e, 1, (0, 10, 5), elb, dlb, "exact")
    seq = list(g["chunks"]) + ([None] if tail else [g["last"]])
    ioff, yoff, nh = g[f"{name}_ids_off"], g[f"{name}_yseq_off"], g[f"{name}_nhyp"]
    hoff = np.concatenate([[0], np.cumsum(nh)])
    decoded = 0
    for i, x in enumerate(seq):
        fin = i == len(seq) - 1
        feats = None if x is None else torch.from_numpy(np.ascontiguousarray(x[None])).cuda()
        r = s.step_beam([0], feats, [0 if x is None else x.shape[0]], [fin], beam=beam, ctc_weight=wctc,
                        penalty=pen, nbest=nbest)
        torch.cuda.synchronize()
        r = {k: v.cpu() for k, v in r.items()}
        got = _hyps(r, 0)
        want = [[t for t in g[f"{name}_yseq"][yoff[q]:yoff[q + 1]][1:-1].tolist() if t not in DROP]
                for q in range(hoff[i], hoff[i + 1])]
        assert got == want, (name, i)
        if want:
            np.testing.assert_allclose(r["scores"][0, : len(want)].numpy(), g[f"{name}_scores"][hoff[i]:hoff[i + 1]],
                                       atol=1e-4, rtol=1e-5)
            decoded += 1
        assert sum(got, []) == g[f"{name}_ids"][ioff[i]:ioff[i + 1]].tolist(), (name, i)
    assert decoded >= len(seq) - 1


def test_stream_beam_small_lcap_refused_before_state_moves(eng):
    """A step whose L_cap cannot hold the window's worst-case token count is refused before the stream's caches
    advance: retrying it with a valid L_cap gives exactly the n-best lists of a stream that never saw the refusal."""
    from funasr_amd.runtime import PfmError, PfmStreams
    cfg, e = eng
    g = np.load(f"{GOLD}/stream_beam_tiny.npz")
    a = PfmStreams(e, 1, (0, 10, 5), 4, 1, "exact")
    b = PfmStreams(e, 1, (0, 10, 5), 4, 1, "exact")
    for i, x in enumerate(list(g["chunks"])[:4]):
        feats = torch.from_numpy(np.ascontiguousarray(x[None])).cuda()
        kw = dict(beam=3, ctc_weight=0.3, nbest=2)
        if i == 2:
            with pytest.raises(PfmError, match="L_cap"):
                a.step_beam([0], feats, [x.shape[0]], [False], L_cap=3, **kw)
        ra = a.step_beam([0], feats, [x.shape[0]], [False], **kw)
        rb = b.step_beam([0], feats, [x.shape[0]], [False], **kw)
        torch.cuda.synchronize()
        ra, rb = {k: v.cpu() for k, v in ra.items()}, {k: v.cpu() for k, v in rb.items()}
        assert _hyps(ra, 0) == _hyps(rb, 0), i
        assert torch.equal(ra["scores"], rb["scores"]), i


def test_stream_beam_batched_equals_single(eng):
    """Three streams with ragged chunks (one joins late, one ends on a tail chunk) in one step_beam per chunk give
    every stream the n-best lists it gets alone (the window lengths and token counts differ per stream)."""
    from funasr_amd.runtime import PfmStreams
    cfg, e = eng
    rng = np.random.default_rng(8)
    ns = {0: (0, [10, 10, 10, 10, 6]), 1: (1, [10, 7, 10, 3]), 2: (0, [10, 10, 0])}
    xs = {k: [rng.standard_normal((n, cfg.input_size)).astype(np.float32) if n else None for n in cs]
          for k, (_, cs) in ns.items()}
    opts = dict(beam=3, ctc_weight=0.4, penalty=0.2, nbest=2)

    def alone(k):
        s = PfmStreams(e, 1, (0, 10, 5), 4, 1, "exact")
        out = []
        for j, x in enumerate(xs[k]):
            r = s.step_beam([0], None if x is None else torch.from_numpy(x[None]).cuda(),
                            [0 if x is None else x.shape[0]], [j == len(xs[k]) - 1], **opts)
            out.append(_hyps({a: v.cpu() for a, v in r.items()}, 0))
        return out

    single = {k: alone(k) for k in ns}
    s = PfmStreams(e, 4, (0, 10, 5), 4, 1, "exact")
    batched = {k: [] for k in ns}
    for step in range(max(j0 + len(cs) for j0, cs in ns.values())):
        act = [k for k, (j0, cs) in ns.items() if j0 <= step < j0 + len(cs)]
        cur = [xs[k][step - ns[k][0]] for k in act]
        nf = [0 if x is None else x.shape[0] for x in cur]
        feats = None
        if max(nf):
            f = np.zeros((len(act), max(nf), cfg.input_size), np.float32)
            for i, x in enumerate(cur):
                if x is not None:
                    f[i, : x.shape[0]] = x
            feats = torch.from_numpy(f).cuda()
        fins = [step - ns[k][0] == len(ns[k][1]) - 1 for k in act]
        r = s.step_beam([3 - k for k in act], feats, nf, fins, **opts)
        rc = {a: v.cpu() for a, v in r.items()}
        for i, k in enumerate(act):
            batched[k].append(_hyps(rc, i))
    assert batched == single
    assert sum(len(h) for hs in single.values() for h in hs) > 0


def test_automodel_streaming_beam_vs_reference():
    """AutoModel(model="ParaformerStreaming", model_conf ctc_weight 0.3).generate(..., decoding_ctc_weight=0.4,
    beam_size=3, nbest=2) per waveform call: the text of every call equals the reference inference() golden (the
    tokens of both n-best hypotheses of every chunk, concatenated, as generate_chunk returns them)."""
    from funasr_amd.auto_model import AutoModel
    from tests.golden.inputs import token_list, waveform
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = _cfg()
    am = AutoModel(model="ParaformerStreaming", model_conf=dict(ctc_weight=0.3, predictor_bias=1), synthetic_seed=0,
                   tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), device="cuda", mode="exact",
                   frontend_conf=dict(cmvn_file=None), **cfg.reference_kwargs())
    am.model.load_state_dict(make_weights(cfg, seed=0))
    am.kwargs["frontend"].cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
    gw = json.load(open(f"{GOLD}/stream_beam_wave.json"))
    wav = waveform(seed=gw["seed"], n=gw["n"])
    cache, pos = {}, 0
    for j, n in enumerate(gw["calls"]):
        res = am.generate(input=wav[pos:pos + n], cache=cache, is_final=j == len(gw["calls"]) - 1,
                          chunk_size=[0, 10, 5], encoder_chunk_look_back=4, decoder_chunk_look_back=1,
                          decoding_ctc_weight=gw["decoding_ctc_weight"], beam_size=gw["beam_size"],
                          nbest=gw["nbest"])
        pos += n
        assert res[0]["text"] == gw["texts"][j], j


def test_stream_beam_bad_args(eng):
    from funasr_amd.runtime import PfmEngine, PfmError, PfmStreams
    cfg, e = eng
    s = PfmStreams(e, 1, (0, 10, 5), 0, 0, "exact")
    x = torch.zeros((1, 10, cfg.input_size), device="cuda")
    with pytest.raises(PfmError):
        s.step_beam([0], x, [10], [False], beam=17)
    with pytest.raises(PfmError):
        s.step_beam([0], x, [10], [False], ctc_weight=0.0)
    with pytest.raises(PfmError):
        s.step_beam([0], x, [10], [False], nbest=17)
    plain = paraformer_streaming_tiny()   # no CTC head
    e2 = PfmEngine(plain, 0)
    e2.load_state_dict(make_weights(plain, seed=0))
    with pytest.raises(PfmError):
        PfmStreams(e2, 1, (0, 10, 5), 0, 0, "exact").step_beam([0], x, [10], [False])


@pytest.fixture(scope="module")
def eng_large():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from funasr_amd.config import paraformer_streaming
    from funasr_amd.runtime import PfmEngine
    cfg = dataclasses.replace(paraformer_streaming(), ctc_weight=0.3)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    return cfg, e


def _large_chunks(e, mode, g):
    from funasr_amd.runtime import PfmStreams
    elb, dlb, beam, nbest, tail = g["opts"].tolist()
    wctc, pen = g["fopts"].tolist()
    s = PfmStreams(e, 1, (0, 10, 5), elb, dlb, mode)
    seq = list(g["chunks"]) + ([None] if tail else [])
    out = []
    for i, x in enumerate(seq):
        fin = i == len(seq) - 1
        feats = None if x is None else torch.from_numpy(np.ascontiguousarray(x[None])).cuda()
        r = s.step_beam([0], feats, [0 if x is None else x.shape[0]], [fin], beam=beam, ctc_weight=wctc, penalty=pen,
                        nbest=nbest)
        torch.cuda.synchronize()
        r = {k: v.cpu() for k, v in r.items()}
        out.append((_hyps(r, 0), r["scores"][0].numpy()))
    return out


def _large_want(g, i):
    yoff, nh = g["yseq_off"], g["nhyp"]
    hoff = np.concatenate([[0], np.cumsum(nh)])
    large_drop = (0, 1, 2)
    hyps = [[t for t in g["yseq"][yoff[q]:yoff[q + 1]][1:-1].tolist() if t not in large_drop]
            for q in range(hoff[i], hoff[i + 1])]
    return hyps, g["scores"][hoff[i]:hoff[i + 1]]


def test_stream_beam_large_exact_vs_reference(eng_large):
    """Config C5 as benched, EXACT mode: Paraformer-large streaming with a CTC head, beam 10, decoding_ctc_weight 0.3,
    look-back 4 / 1: every chunk's n-best (nbest 2) token sequences identical to the reference generate_chunk's
    BeamSearchPara and the scores within 1e-4 relative (tests/golden/stream_beam_large.npz, make_golden.py
    save_stream_beam_large)."""
    cfg, e = eng_large
    g = np.load(f"{GOLD}/stream_beam_large.npz")
    got = _large_chunks(e, "exact", g)
    ioff = g["ids_off"]
    for i, (hyps, scores) in enumerate(got):
        want, wsc = _large_want(g, i)
        assert hyps == want, i
        np.testing.assert_allclose(scores[: len(want)], wsc, rtol=1e-4, atol=1e-4)
        assert sum(hyps, []) == g["ids"][ioff[i]:ioff[i + 1]].tolist(), i


def test_stream_beam_large_fast_close(eng_large):
    """The same chunks in fast mode (bf16 operands; the chunk path keeps plain bf16 weights), held to bounds derived
    from the CPU emulation of plain bf16 rounding (tests/golden/fast_emul.json "G", tests/fast_parity.py
    bounds_from_emulation), not from the kernel's own output: the 1-best's positions disagree with the reference's
    1-best no more often than the emulation's flip bound; the best joint score (log-prob units: a sum over the
    hypothesis' tokens) moves per token no more than the emulation's mean-regret bound, and in any chunk by less than
    0.5 (tighter than the emulation's single-decision bound, max_regret + 0.15). A 0.3-nat decoder bias perturbation,
    checked in tests/test_gpu_parity.py, moves single positions by more than that."""
    import json
    from tests.fast_parity import bounds_from_emulation
    cfg, e = eng_large
    g = np.load(f"{GOLD}/stream_beam_large.npz")
    em = json.load(open(f"{GOLD}/fast_emul.json", encoding="utf-8"))["para_large_b64"]["G"]
    b = bounds_from_emulation(em)
    got = _large_chunks(e, "fast", g)
    agree, tot, worst, gap, ntok = 0, 0, 0.0, 0.0, 0
    for i, (hyps, scores) in enumerate(got):
        want, wsc = _large_want(g, i)
        assert hyps, i
        d = abs(float(scores[0]) - float(wsc[0]))
        worst = max(worst, d)
        a, r = hyps[0], want[0]
        tot += max(len(a), len(r))
        agree += sum(int(x == y) for x, y in zip(a, r))
        gap += d
        ntok += max(1, len(r))
        print(f"chunk {i}: {len(a)} / {len(r)} tokens, best-score gap {d:.4f}")
    print(f"stream beam large fast: 1-best position agreement {agree}/{tot}, best-score gap per token {gap / ntok:.4f} "
          f"(bound {b['mean_regret']:.4f}), largest {worst:.3f}; flip bound {b['flip_frac']:.3f}")
    assert worst < min(0.5, b["max_regret"])
    assert gap / ntok < b["mean_regret"]
    assert agree >= (1.0 - b["flip_frac"]) * tot
