"""CT-Transformer punctuation through the C-ABI (pfm_run_punc) vs the reference
CTTransformer goldens (tests/golden/punc_tiny.npz / punc.json) and the oracle (oracle/punc_ref.py).

EXACT mode: logits of every reference punc_forward call within 1e-4, argmax ids identical; AutoModel
text / punc_array identical to the reference inference(). FAST mode: argmax agreement floor.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import ct_transformer, ct_transformer_tiny  # noqa: E402
from funasr_amd.runtime import PfmEngine, PfmError  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def tiny():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = ct_transformer_tiny()
    w = make_weights(cfg, seed=0)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(w)
    return cfg, e, w


def _calls(name):
    g = np.load(f"{GOLD}/punc_tiny.npz")
    ids, off, lg = g[f"{name}_ids"], g[f"{name}_off"], g[f"{name}_logits"]
    return [(ids[off[i]:off[i + 1]], lg[off[i]:off[i + 1]]) for i in range(len(off) - 1)]


@pytest.mark.parametrize("name", ["short", "mixed", "long"])
def test_punc_exact_vs_reference_calls(tiny, name):
    cfg, e, _ = tiny
    for x, ref in _calls(name):
        r = e.run_punc(torch.from_numpy(x[None].astype(np.int32)).cuda(),
                       torch.tensor([len(x)], dtype=torch.int32).cuda(), mode="exact", want_logits=True)
        torch.cuda.synchronize()
        lg = r["logits"][0].cpu().numpy()
        np.testing.assert_allclose(lg, ref, atol=1e-4, rtol=1e-4)
        assert np.array_equal(r["punc"][0].cpu().numpy(), ref.argmax(-1))


def test_punc_batched_ragged_vs_oracle(tiny):
    """Three word sequences of different lengths in one call (padded rows -> -1, keys masked)."""
    from oracle.punc_ref import punc_forward
    cfg, e, w = tiny
    rng = np.random.default_rng(9)
    lens = [37, 5, 120]
    T = max(lens)
    ids = np.zeros((3, T), np.int32)
    for b, n in enumerate(lens):
        ids[b, :n] = rng.integers(3, cfg.vocab_size, n)
    r = e.run_punc(torch.from_numpy(ids).cuda(), torch.tensor(lens, dtype=torch.int32).cuda(), mode="exact",
                   want_logits=True)
    torch.cuda.synchronize()
    punc, lg = r["punc"].cpu().numpy(), r["logits"].cpu().numpy()
    for b, n in enumerate(lens):
        ref = punc_forward(ids[b:b + 1, :n], [n], w, cfg)[0].numpy()
        np.testing.assert_allclose(lg[b, :n], ref, atol=1e-4, rtol=1e-4)
        assert np.array_equal(punc[b, :n], ref.argmax(-1))
        assert np.all(punc[b, n:] == -1)


def test_punc_fast_mode_agreement(tiny):
    cfg, e, _ = tiny
    agree = total = 0
    for name in ("short", "mixed", "long"):
        for x, ref in _calls(name):
            r = e.run_punc(torch.from_numpy(x[None].astype(np.int32)).cuda(),
                           torch.tensor([len(x)], dtype=torch.int32).cuda(), mode="fast")
            torch.cuda.synchronize()
            agree += int((r["punc"][0].cpu().numpy() == ref.argmax(-1)).sum())
            total += len(x)
    assert agree / total >= 0.8, (agree, total)


def test_punc_released_dims_vs_oracle():
    """The released model's dimensions (4 blocks, 272,727-word embedding): argmax ids exact vs the oracle."""
    from oracle.punc_ref import punc_forward
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = ct_transformer()
    w = make_weights(cfg, seed=0)
    e = PfmEngine(cfg, 0)
    e.load_state_dict(w)
    ids = np.random.default_rng(4).integers(3, cfg.vocab_size, (1, 217)).astype(np.int32)
    r = e.run_punc(torch.from_numpy(ids).cuda(), torch.tensor([217], dtype=torch.int32).cuda(), mode="exact",
                   want_logits=True)
    torch.cuda.synchronize()
    ref = punc_forward(ids, [217], w, cfg)[0].numpy()
    np.testing.assert_allclose(r["logits"][0].cpu().numpy(), ref, atol=1e-4, rtol=1e-4)
    assert np.array_equal(r["punc"][0].cpu().numpy(), ref.argmax(-1))


def test_automodel_punc_generate_vs_reference():
    """AutoModel(model="CTTransformer").generate(input=text): text and punc_array of the reference."""
    from funasr_amd.auto_model import AutoModel
    from tests.golden.inputs import token_list
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = ct_transformer_tiny()
    am = AutoModel(model="CTTransformer", model_conf={}, synthetic_seed=0, device="cuda", mode="exact",
                   tokenizer="CharTokenizer", tokenizer_conf=dict(token_list=token_list(cfg.vocab_size),
                                                                  unk_symbol="<unk>"),
                   **cfg.reference_kwargs())
    gold = json.load(open(f"{GOLD}/punc.json", encoding="utf-8"))
    for name, gj in gold.items():
        res = am.generate(input=gj["text_in"], key=name)
        assert res[0]["key"] == name
        assert res[0]["text"] == gj["text"], name
        assert res[0]["punc_array"].tolist() == gj["punc_array"], name


def test_punc_bad_args(tiny):
    cfg, e, _ = tiny
    with pytest.raises(PfmError):
        e.run_punc(torch.zeros((2, 4), dtype=torch.int32).cuda(), torch.tensor([4], dtype=torch.int32).cuda())


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_punc_host_graph_replay_matches_device_path(mode):
    """PFM_PUNC_GRAPH=1 (the default): fast-mode pfm_run_punc_host pads the sentence to a multiple of 16 words and
    replays one HIP graph per padded length from its second call on — 20- and 27-word sentences share one graph, 33 and
    41 another: the first (eager), second (capture) and later (replay) calls, interleaved, equal pfm_run_punc's labels
    on unpadded device operands; after new weights are loaded, the replayed graphs follow them. EXACT mode and
    PFM_PUNC_GRAPH=0 run unpadded and eager, with the same labels."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    os.environ.pop("PFM_PUNC_GRAPH", None)
    cfg = ct_transformer()
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    rng = np.random.default_rng(11)
    seqs = [rng.integers(3, cfg.vocab_size, n).astype(np.int32) for n in (20, 27, 33, 20, 41)]

    def device(x):
        r = e.run_punc(torch.from_numpy(x[None]).cuda(), torch.tensor([len(x)], dtype=torch.int32).cuda(), mode=mode)
        torch.cuda.synchronize()
        return r["punc"][0].cpu().numpy()

    try:
        for weights_seed in (0, 1):
            if weights_seed:
                e.load_state_dict(make_weights(cfg, seed=weights_seed))
            want = [device(x) for x in seqs]
            for rep in range(3):
                for x, wv in zip(seqs, want):
                    got = e.run_punc_host(x, mode=mode)
                    assert np.array_equal(got, wv), (weights_seed, rep, len(x))
    finally:
        os.environ["PFM_PUNC_GRAPH"] = "0"
    try:
        assert all(np.array_equal(e.run_punc_host(x, mode=mode), wv) for x, wv in zip(seqs, want))
    finally:
        del os.environ["PFM_PUNC_GRAPH"]


@pytest.mark.parametrize("n", [30, 100, 200])
def test_punc_fast_logits_close_to_exact(n):
    """Released dims: fast-mode logits (bf16 operands; LayerNorm folded into the skinny QKV / w1 launches, 64-row
    blocks beyond 64 words) within a bf16-sized distance of EXACT's, which the oracle pins; labels mostly equal."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = ct_transformer()
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    ids = torch.from_numpy(np.random.default_rng(n).integers(3, cfg.vocab_size, (1, n)).astype(np.int32)).cuda()
    lens = torch.tensor([n], dtype=torch.int32).cuda()
    rx = e.run_punc(ids, lens, mode="exact", want_logits=True)
    rf = e.run_punc(ids, lens, mode="fast", want_logits=True)
    torch.cuda.synchronize()
    lx, lf = rx["logits"][0].cpu().numpy(), rf["logits"][0].cpu().numpy()
    d = np.abs(lx - lf).max()
    print(f"n={n}: max |fast - exact| = {d:.4f} (logit std {lx.std():.3f})")
    assert d < 0.05 * max(1.0, float(np.abs(lx).max())), d
    assert (rx["punc"] == rf["punc"]).float().mean().item() >= 0.9
