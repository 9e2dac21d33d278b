"""Streaming Paraformer (config C5) through the C-ABI: pfm_streams_create / pfm_stream_step vs the
reference generate_chunk goldens (tests/golden/stream_tiny.npz) and vs oracle/streaming_ref.chunk_step
for batched, ragged streams that join and finish at different steps.

EXACT mode: token ids of every chunk exact; encoder window rows within 1e-4 (as the oracle's own
golden check); CIF chunk-masked alphas within 1e-5. FAST mode: token agreement floor.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_streaming, paraformer_streaming_tiny  # noqa: E402
from funasr_amd.runtime import PfmEngine, PfmStreams  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DROP = (0, 1, 2)


def _eng(cfg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    w = make_weights(cfg, seed=0)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(w)
    return e, w


@pytest.fixture(scope="module")
def tiny():
    cfg = paraformer_streaming_tiny()
    e, w = _eng(cfg)
    return cfg, e, w


def _toks(r, i):
    n = int(r["ntok"][i])
    return [t for t in r["tokens"][i, :n].tolist() if t not in DROP]


@pytest.mark.parametrize("tag,elb,dlb,tail", [("lb00", 0, 0, False), ("lb41", 4, 1, False),
                                              ("lb41_tail", 4, 1, True)])
def test_stream_golden_one_slot(tiny, tag, elb, dlb, tail):
    cfg, e, _ = tiny
    g = np.load(f"{GOLD}/stream_tiny.npz")
    s = PfmStreams(e, 1, (0, 10, 5), elb, dlb, "exact")
    seq = list(g["chunks"]) + ([None] if tail else [g["last"]])
    off, eoff = g[f"{tag}_off"], g[f"{tag}_enc_off"]
    for i, x in enumerate(seq):
        fin = i == len(seq) - 1
        feats = None if x is None else torch.from_numpy(np.ascontiguousarray(x[None])).cuda()
        nf = 0 if x is None else x.shape[0]
        r = s.step([0], feats, [nf], [fin], want_enc=True)
        torch.cuda.synchronize()
        r = {k: (v.cpu() if v is not None else None) for k, v in r.items()}
        assert _toks(r, 0) == g[f"{tag}_tokens"][off[i]:off[i + 1]].tolist(), (tag, i)
        ref = g[f"{tag}_enc"][eoff[i]:eoff[i + 1]]
        np.testing.assert_allclose(r["enc"][0, : ref.shape[0]].numpy(), ref, atol=1e-4, rtol=1e-4)


def _schedules(rng, I):
    """Three streams: A full chunks, B ragged chunks (joins at step 1), C short (ends with a tail)."""
    def chunks(ns):
        return [rng.standard_normal((n, I)).astype(np.float32) if n else None for n in ns]
    return {0: (0, chunks([10, 10, 10, 10, 6])), 1: (1, chunks([10, 7, 10, 3])), 2: (0, chunks([10, 10, 0]))}


@pytest.mark.parametrize("elb,dlb", [(0, 0), (4, 1), (2, 2)])
def test_stream_batched_ragged_vs_oracle(tiny, elb, dlb):
    from oracle.streaming_ref import StreamState, chunk_step
    cfg, e, w = tiny
    rng = np.random.default_rng(5 + elb)
    sched = _schedules(rng, cfg.input_size)
    s = PfmStreams(e, 4, (0, 10, 5), elb, dlb, "exact")
    # slots deliberately not 0..n-1: stream k lives in slot 3-k
    states = {k: StreamState(cfg, (0, 10, 5), elb, dlb) for k in sched}
    nsteps = max(j0 + len(cs) for j0, cs in sched.values())
    for step in range(nsteps):
        act = [k for k, (j0, cs) in sched.items() if j0 <= step < j0 + len(cs)]
        xs = [sched[k][1][step - sched[k][0]] for k in act]
        fins = [step - sched[k][0] == len(sched[k][1]) - 1 for k in act]
        nf = [0 if x is None else x.shape[0] for x in xs]
        Tn = max(nf)
        feats = None
        if Tn:
            f = np.zeros((len(act), Tn, cfg.input_size), np.float32)
            for i, x in enumerate(xs):
                if x is not None:
                    f[i, : x.shape[0]] = x
            feats = torch.from_numpy(f).cuda()
        r = s.step([3 - k for k in act], feats, nf, fins, want_enc=True, want_alphas=True)
        torch.cuda.synchronize()
        r = {k: (v.cpu() if v is not None else None) for k, v in r.items()}
        for i, k in enumerate(act):
            st = states[k]
            if xs[i] is None:
                st.tail_chunk = True
            ref = chunk_step(xs[i], st, w, cfg, fins[i])
            assert int(r["ntok"][i]) == ref["ntok"], (step, k)
            assert _toks(r, i) == ref["tokens"], (step, k)
            tw = ref["enc"].shape[0]
            np.testing.assert_allclose(r["enc"][i, :tw].numpy(), ref["enc"].numpy(), atol=1e-4, rtol=1e-4)
            assert np.abs(r["enc"][i, tw:].numpy()).max(initial=0.0) == 0.0
            np.testing.assert_allclose(r["alphas"][i, :tw].numpy(), ref["alphas"].numpy(), atol=1e-5)


def test_stream_reset_reuses_slot(tiny):
    """A finished slot reset by pfm_streams_reset behaves like a fresh stream."""
    cfg, e, _ = tiny
    g = np.load(f"{GOLD}/stream_tiny.npz")
    s = PfmStreams(e, 2, (0, 10, 5), 4, 1, "exact")
    seq = list(g["chunks"][:3])
    for x in seq:
        s.step([1], torch.from_numpy(np.ascontiguousarray(x[None])).cuda(), [10], [False])
    s.reset([1])
    off = g["lb41_off"]
    for i, x in enumerate(list(g["chunks"]) + [g["last"]]):
        r = s.step([1], torch.from_numpy(np.ascontiguousarray(x[None])).cuda(), [x.shape[0]], [i == 8])
        torch.cuda.synchronize()
        assert _toks({k: v.cpu() for k, v in r.items() if v is not None}, 0) == \
            g["lb41_tokens"][off[i]:off[i + 1]].tolist(), i


def test_stream_fast_mode_agreement(tiny):
    cfg, e, _ = tiny
    g = np.load(f"{GOLD}/stream_tiny.npz")
    s = PfmStreams(e, 1, (0, 10, 5), 4, 1, "fast")
    seq = list(g["chunks"]) + [g["last"]]
    off = g["lb41_off"]
    agree = total = 0
    for i, x in enumerate(seq):
        r = s.step([0], torch.from_numpy(np.ascontiguousarray(x[None])).cuda(), [x.shape[0]], [i == len(seq) - 1])
        torch.cuda.synchronize()
        got = _toks({k: v.cpu() for k, v in r.items() if v is not None}, 0)
        ref = g["lb41_tokens"][off[i]:off[i + 1]].tolist()
        total += max(len(ref), len(got))
        agree += sum(a == b for a, b in zip(got, ref))
    assert total > 0 and agree / total >= 0.6, (agree, total)


def test_stream_large_exact_vs_oracle():
    """Paraformer-streaming large (50 + 16 layers): 6 chunks of one stream, token ids exact."""
    from oracle.streaming_ref import StreamState, chunk_step
    cfg = paraformer_streaming()
    e, w = _eng(cfg)
    rng = np.random.default_rng(3)
    s = PfmStreams(e, 1, (0, 10, 5), 4, 1, "exact")
    st = StreamState(cfg, (0, 10, 5), 4, 1)
    ns = [10, 10, 10, 10, 10, 4]
    for i, n in enumerate(ns):
        x = rng.standard_normal((n, cfg.input_size)).astype(np.float32)
        fin = i == len(ns) - 1
        r = s.step([0], torch.from_numpy(x[None]).cuda(), [n], [fin], want_enc=True)
        torch.cuda.synchronize()
        r = {k: (v.cpu() if v is not None else None) for k, v in r.items()}
        ref = chunk_step(x, st, w, cfg, fin)
        assert _toks(r, 0) == ref["tokens"], i
        tw = ref["enc"].shape[0]
        d = r["enc"][0, :tw].numpy() - ref["enc"].numpy()
        assert np.linalg.norm(d) / np.linalg.norm(ref["enc"].numpy()) < 1e-5, i


def test_stream_large_fast_regret():
    """Paraformer-streaming large, fast mode (bf16 operands; the chunk path keeps plain bf16 weights), 25 chunks of one
    stream against the reference generate_chunk's per-position top-5 log-probs (tests/golden/stream_large.npz): the
    regret bounds the offline path is held to for plain bf16 operands (the CPU emulation of ideal bf16 at B = 64,
    tests/golden/fast_emul.json); per-chunk token counts within one of the reference's."""
    import json
    from tests.fast_parity import bounds_from_emulation, stream_stats
    cfg = paraformer_streaming()
    e, _ = _eng(cfg)
    g = np.load(f"{GOLD}/stream_large.npz")
    s = PfmStreams(e, 1, (0, 10, 5), 4, 1, "fast")
    rng = np.random.default_rng(int(g["seed"]))
    ns = g["ns"].tolist()
    chunks = []
    for i, n in enumerate(ns):
        x = rng.standard_normal((n, cfg.input_size), dtype=np.float32)
        r = s.step([0], torch.from_numpy(x[None]).cuda(), [n], [i == len(ns) - 1])
        torch.cuda.synchronize()
        nt = int(r["ntok"][0])
        chunks.append((r["tokens"][0, :max(nt, 0)].cpu().numpy(), nt))
    st = stream_stats(chunks, g, 0.5)
    em = json.load(open(f"{GOLD}/fast_emul.json", encoding="utf-8"))["para_large_b64"]["G"]
    b = bounds_from_emulation(em)
    print(f"stream large fast: {st}; bounds {b}")
    assert st["positions"] > 100
    assert st["mean_regret"] < b["mean_regret"] and st["flip_frac"] < b["flip_frac"]
    assert st["max_regret"] < b["max_regret"] and st["outside_topk"] <= b["outside_frac"] * st["positions"] + 1
    # a CIF fire near a chunk boundary may move into the next chunk (the carried alpha): per-chunk counts within one,
    # the stream's total within two (measured: 21 of 25 chunks equal)
    got_n = np.array([n for _, n in chunks])
    assert np.abs(got_n - g["ntok"]).max() <= 1 and abs(int(got_n.sum()) - int(g["ntok"].sum())) <= 2
    assert st["equal_counts"] >= 0.75


def test_stream_bad_args(tiny):
    from funasr_amd.runtime import PfmError
    cfg, e, _ = tiny
    s = PfmStreams(e, 2, (0, 10, 5), 0, 0, "exact")
    x = torch.zeros((1, 10, cfg.input_size), device="cuda")
    with pytest.raises(PfmError):
        s.step([2], x, [10], [False])            # slot out of range
    with pytest.raises(PfmError):
        s.step([0], x, [0], [False])             # tail chunk must be final
    with pytest.raises(PfmError):
        s.step([0, 0], torch.zeros((2, 10, cfg.input_size), device="cuda"), [10, 10], [False, False])
    with pytest.raises(PfmError):
        PfmStreams(e, 1, (0, 10, 5), -1, 0, "exact")


# ---------------------------------------------------------------- online frontend + model contract
TOL_LOGMEL = 2e-4   # GPU fbank vs the reference's kaldi-native-fbank (tests/test_gpu_frontend.py)


def _stream_model(tiny_cfg):
    import json  # noqa: F401
    from funasr_amd.auto_model import AutoModel
    from tests.golden.inputs import token_list
    kw = tiny_cfg.reference_kwargs()
    return AutoModel(model="ParaformerStreaming", model_conf=dict(ctc_weight=0.0, predictor_bias=1),
                     synthetic_seed=0, tokenizer_conf=dict(token_list=token_list(tiny_cfg.vocab_size)),
                     device="cuda", mode="exact", frontend_conf=dict(cmvn_file=None), **kw)


@pytest.mark.parametrize("tag", ["w1", "w2"])
def test_online_frontend_vs_reference(tiny, tag):
    """WavFrontendOnline.step (pfm_fbank_raw + pfm_lfr_gather) over the reference's own 600 ms chunking
    of each call: every LFR+CMVN row the reference frontend emitted (tests/golden/stream_<tag>_feats.npy)."""
    import json
    from funasr_amd.frontend import WavFrontendOnline
    from tests.golden.inputs import waveform
    cfg, e, _ = tiny
    gw = json.load(open(f"{GOLD}/stream_wave.json"))[tag]
    cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
    fe = WavFrontendOnline(cmvn_file=None)
    fe.cmvn = cmvn
    wav = waveform(seed=gw["seed"], n=gw["n"])
    cache, prev, pos, got = {}, np.zeros(0, np.float32), 0, []
    for j, n in enumerate(gw["calls"]):
        fin = j == len(gw["calls"]) - 1
        a = np.concatenate([prev, wav[pos:pos + n]])
        pos += n
        nch = int(len(a) // 9600 + int(fin))
        m = int(len(a) % 9600 * (1 - int(fin)))
        for i in range(nch):
            seg = a[i * 9600:(i + 1) * 9600]
            last = fin and i == nch - 1
            if last and len(seg) < 960:
                continue
            got.append(fe.step(e, [(seg, last, cache)])[0].cpu().numpy())
        prev = a[:-m] if m else a[:0]
    assert [f.shape[0] for f in got] == gw["feat_rows"]
    ref = np.load(f"{GOLD}/stream_{tag}_feats.npy")
    assert np.abs(np.concatenate(got) - ref).max() < TOL_LOGMEL * float(np.abs(cmvn[1]).max())


def test_automodel_streaming_generate_vs_reference():
    """AutoModel(model="ParaformerStreaming").generate(chunk, cache=cache, is_final=...) per call: the
    text of every call equals the reference inference() goldens (stream_wave.json, look-back 4 / 1)."""
    import json
    from tests.golden.inputs import waveform
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = paraformer_streaming_tiny()
    am = _stream_model(cfg)
    am.model.load_state_dict(make_weights(cfg, seed=0))
    am.kwargs["frontend"].cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
    gold = json.load(open(f"{GOLD}/stream_wave.json"))
    for tag, gw in gold.items():
        wav = waveform(seed=gw["seed"], n=gw["n"])
        cache, pos = {}, 0
        for j, n in enumerate(gw["calls"]):
            fin = j == len(gw["calls"]) - 1
            res = am.generate(input=wav[pos:pos + n], cache=cache, is_final=fin, chunk_size=[0, 10, 5],
                              encoder_chunk_look_back=4, decoder_chunk_look_back=1)
            pos += n
            assert res[0]["text"] == gw["texts"][j], (tag, j)


def test_inference_streams_batched_equals_single():
    """inference_streams over 3 concurrent streams (different lengths / call sizes) gives each stream the
    tokens it gets alone."""
    from tests.golden.inputs import waveform
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = paraformer_streaming_tiny()
    am = _stream_model(cfg)
    mdl = am.model
    kw = dict(chunk_size=[0, 10, 5], encoder_chunk_look_back=4, decoder_chunk_look_back=1)
    wavs = [waveform(seed=40 + i, n=n) for i, n in enumerate([40000, 23456, 31000])]
    calls = [[9600, 9600, 20800], [5000, 18456], [31000]]
    fe = am.kwargs["frontend"]
    single = []
    for w, cs in zip(wavs, calls):
        cache, pos, toks = {}, 0, []
        for j, n in enumerate(cs):
            toks += mdl.inference_streams([(w[pos:pos + n], cache, j == len(cs) - 1)], frontend=fe, **kw)[0]
            pos += n
        single.append(toks)
    caches = [{} for _ in wavs]
    pos = [0, 0, 0]
    batched = [[], [], []]
    for j in range(3):
        act = [k for k in range(3) if j < len(calls[k])]
        items = []
        for k in act:
            n = calls[k][j]
            items.append((wavs[k][pos[k]:pos[k] + n], caches[k], j == len(calls[k]) - 1))
            pos[k] += n
        for k, t in zip(act, mdl.inference_streams(items, frontend=fe, **kw)):
            batched[k] += t
    assert batched == single
    assert sum(len(t) for t in single) > 0


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_stream_graph_replay_matches_eager(tiny, mode, monkeypatch):
    """HIP-graph replay of the step launch sequences (the default without optional outputs) gives the
    same tokens and counts as eager launches over a ragged batched schedule (graphs are captured at the
    second step of a shape and replayed from the third)."""
    cfg, e, _ = tiny

    def run(graph: str):
        monkeypatch.setenv("PFM_STREAM_GRAPH", graph)
        rng = np.random.default_rng(11)
        s = PfmStreams(e, 3, (0, 10, 5), 4, 1, mode)
        out = []
        ns = [[10] * 6 + [4], [10] * 6 + [7], [10] * 7]
        for j in range(7):
            x = np.zeros((3, 10, cfg.input_size), np.float32)
            for k in range(3):
                x[k, : ns[k][j]] = rng.standard_normal((ns[k][j], cfg.input_size))
            r = s.step([0, 1, 2], torch.from_numpy(x).cuda(), [ns[k][j] for k in range(3)], [j == 6] * 3)
            torch.cuda.synchronize()
            rc = {k: v.cpu() for k, v in r.items() if v is not None}
            out.append((rc["ntok"].tolist(), [_toks(rc, i) for i in range(3)]))
        return out

    eager, graphed = run("0"), run("1")
    assert graphed == eager
    assert sum(sum(n) for n, _ in eager) > 0



def test_stream_graph_replay_after_weight_reload():
    """EXACT-mode streaming graphs hold the addresses of layer 0's padded split planes (K = 560): a weight
    reload after a graph was captured re-splits them in place (same buffers), so later replays see the new
    weights. The same streams object runs one schedule before a reload (graphs captured at step 2, replayed
    after), with layer 0's QKV scaled, and with the original weights back: the first and last runs equal a fresh
    engine's run and the scaled interlude differs."""
    cfg = paraformer_streaming_tiny()
    e, w = _eng(cfg)
    rng = np.random.default_rng(5)
    xs = [torch.from_numpy(rng.standard_normal((2, 10, cfg.input_size), dtype=np.float32)).cuda() for _ in range(6)]

    def run(s):
        s.reset([0, 1])
        out = []
        for j, x in enumerate(xs):
            r = s.step([0, 1], x, [10, 10], [j == len(xs) - 1] * 2)
            torch.cuda.synchronize()
            rc = {k: v.cpu() for k, v in r.items() if v is not None}
            out.append([_toks(rc, i) for i in range(2)])
        return out

    s = PfmStreams(e, 2, (0, 10, 5), 4, 1, "exact")
    base = run(s)
    key = "encoder.encoders0.0.self_attn.linear_q_k_v.weight"
    e.set_weight(key, w[key] * 3.0)
    scaled = run(s)
    e.set_weight(key, w[key])
    again = run(s)
    e2, _ = _eng(cfg)
    fresh = run(PfmStreams(e2, 2, (0, 10, 5), 4, 1, "exact"))
    assert again == base == fresh
    assert scaled != base
    assert sum(len(t) for step in base for t in step) > 0
