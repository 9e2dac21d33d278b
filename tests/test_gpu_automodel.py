"""AutoModel on the HIP path, end to end:
  * waveform input (config C1): a Paraformer-large 5 s wav (and a 3 s / 7 s one) through AutoModel.generate in
    EXACT mode gives the reference AutoModel.generate's result dicts (reference run on the CPU with kaldi.fbank =
    the compiled kaldi-native-fbank, tests/golden/automodel_wav_large.json); at tiny size the model alone is
    token-exact against the oracle fed the GPU's own pfm_fbank features, and those features equal the oracle
    fbank's, so the tokens equal the oracle's on its own features too;
  * a local model dir (config.yaml + model.pt + tokens.json + am.mvn; download_model_from_hub.py:60-79,
    load_pretrained_model.py:44-47) decodes exactly like the same weights given by seed;
  * data parallel: two gloo ranks sharing cuda:0 (spawned, so no GPU state is inherited) decode a ragged
    list of wav files with length-sorted sharding, and the gathered results equal the one-rank run.
"""
import json
import os
import socket
import wave

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd.config import paraformer_tiny  # noqa: E402
from oracle import fbank_ref  # noqa: E402
from tests.golden.inputs import token_list, waveform  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _automodel(**extra):
    from funasr_amd.auto_model import AutoModel
    kw = paraformer_tiny().reference_kwargs()
    kw.update(extra)
    return AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                     device="cuda", mode="exact", **kw)


def _write_wav(path, x):
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(q.tobytes())


WAV_SPECS = [(41, 16000 * 2 + 311), (42, 16000 * 6), (43, 16000 * 1 + 5), (44, 16000 * 4 + 777),
             (45, 16000 * 3), (46, 16000 * 5 + 4000), (47, 9000)]


def _wav_files(d):
    paths = []
    for i, (seed, n) in enumerate(WAV_SPECS):
        p = os.path.join(str(d), f"utt{i}.wav")
        _write_wav(p, waveform(seed, n))
        paths.append(p)
    return paths


def test_waveform_model_alone_token_exact():
    from funasr_amd.weights import make_weights
    from oracle.paraformer_ref import paraformer_infer
    cfg = paraformer_tiny()
    am = _automodel()                       # no tokenizer -> token_int results
    wavs = [waveform(31, 16000 * 3), waveform(32, 16000 * 5 + 123), waveform(33, 16000 * 2 + 7)]
    res = am.generate(input=wavs, batch_size=3, key=["a", "b", "c"])
    got = [r["token_int"] for r in res]

    eng = am.model.engine()
    S = max(len(w) for w in wavs)
    buf = np.zeros((len(wavs), S), np.float32)
    for i, w in enumerate(wavs):
        buf[i, : len(w)] = w
    feats, tout = eng.fbank(torch.from_numpy(buf).cuda(), torch.tensor([len(w) for w in wavs], dtype=torch.int32))
    torch.cuda.synchronize()
    feats, tout = feats.cpu().numpy(), tout.cpu().numpy()
    w = make_weights(cfg)
    # (1) the model alone: oracle on the GPU's own features == the HIP path, token for token
    r_gpu = paraformer_infer(feats[:, : int(tout.max())], tout, w, cfg, keep_logits=True)
    assert got == r_gpu["tokens"]

    # (2) the frontend alone: pfm_fbank reproduces the knf-pinned restatement (oracle/fbank_ref) to float rounding,
    # so the oracle on the restatement's features decodes the same tokens
    ref_feats = [fbank_ref.frontend(x) for x in wavs]
    assert [f.shape[0] for f in ref_feats] == tout.tolist()
    for i, f in enumerate(ref_feats):
        assert float((feats[i, : f.shape[0]] == f).mean()) >= 0.999, i
    T = max(f.shape[0] for f in ref_feats)
    x = np.zeros((len(wavs), T, 560), np.float32)
    for i, f in enumerate(ref_feats):
        x[i, : f.shape[0]] = f
    r_ref = paraformer_infer(x, tout, w, cfg)
    assert r_ref["tokens"] == got


@pytest.mark.parametrize("name", ["c1", "w3", "w7"])
def test_automodel_wav_large_matches_reference_generate(name):
    """Config C1 end to end: Paraformer-large (seeded weights), one wav per generate() call, EXACT mode, waveform in
    -> text out; equal to the reference AutoModel.generate result dict (make_golden.py automodel_wav_large)."""
    from funasr_amd.config import paraformer_large
    cfg = paraformer_large()
    gj = json.load(open(f"{GOLD}/automodel_wav_large.json", encoding="utf-8"))[name]
    am = _large_wav_automodel(cfg)
    res = am.generate(input=waveform(gj["seed"], gj["n"]), key=[name])
    assert res == gj["result"], (res[0]["text"], gj["result"][0]["text"])


_LARGE_AM = {}


def _large_wav_automodel(cfg):
    from funasr_amd.auto_model import AutoModel
    if "am" not in _LARGE_AM:
        am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                       tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), device="cuda", mode="exact",
                       **cfg.reference_kwargs())
        am.kwargs["frontend"].cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
        _LARGE_AM["am"] = am
    return _LARGE_AM["am"]


def test_model_dir_matches_synthetic_seed(tmp_path):
    """A model dir written the way the hub layout stores it (config.yaml, model.pt {"state_dict"}, tokens.json,
    am.mvn) decodes exactly like AutoModel(model="Paraformer", synthetic_seed=0) with the same token list and
    CMVN."""
    import yaml
    from funasr_amd.weights import make_weights
    cfg = paraformer_tiny()
    toks = token_list(cfg.vocab_size)
    cmvn = np.load(f"{GOLD}/lfr_cmvn.npz")["cmvn"]
    d = tmp_path / "paraformer_tiny"
    d.mkdir()
    conf = cfg.reference_kwargs()
    conf.pop("vocab_size")
    conf.update(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), frontend="WavFrontend",
                frontend_conf=dict(fs=16000, window="hamming", n_mels=80, frame_length=25, frame_shift=10,
                                   lfr_m=7, lfr_n=6),
                tokenizer="CharTokenizer", tokenizer_conf=dict(unk_symbol="<unk>", split_with_space=True))
    (d / "config.yaml").write_text(yaml.safe_dump(conf, allow_unicode=True), encoding="utf-8")
    torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in make_weights(cfg, 0).items()}}, d / "model.pt")
    (d / "tokens.json").write_text(json.dumps(toks, ensure_ascii=False), encoding="utf-8")
    with open(d / "am.mvn", "w") as f:
        f.write("<Nnet>\n<Splice> 560 560\n[ 0 ]\n<AddShift> 560 560\n<LearnRateCoef> 0 [ "
                + " ".join(repr(float(v)) for v in cmvn[0]) + " ]\n<Rescale> 560 560\n<LearnRateCoef> 0 [ "
                + " ".join(repr(float(v)) for v in cmvn[1]) + " ]\n</Nnet>\n")
    from funasr_amd.auto_model import AutoModel
    am_dir = AutoModel(model=str(d), device="cuda", mode="exact")
    am_seed = _automodel(tokenizer_conf=dict(token_list=toks), frontend_conf=dict(cmvn_file=str(d / "am.mvn")))
    wavs = [waveform(51, 16000 * 4), waveform(52, 16000 * 2 + 900)]
    a = am_dir.generate(input=wavs, batch_size=2, key=["x", "y"])
    b = am_seed.generate(input=wavs, batch_size=2, key=["x", "y"])
    assert a == b
    assert all(r["text"] for r in a)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, paths, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)   # both ranks share the one card of the box
        am = _automodel()
        res = am.generate(input=paths, batch_size=1)
        from funasr_amd.distributed import item_lengths, length_sorted_shards
        mine = length_sorted_shards(item_lengths(paths), world)[rank]
        q.put((rank, res, mine, am.last_gather))
    finally:
        dist.destroy_process_group()


def test_dp_world2_shared_device_matches_single_rank(tmp_path):
    import torch.multiprocessing as mp
    paths = _wav_files(tmp_path)
    # batch_size 1 on both sides: each utterance is decoded alone in either run, so the comparison is
    # bitwise (a batch's padded length changes the GEMM tile policy, which may move an f32 rounding and
    # flip a near-tie token of the random-weight model: that is batching, not sharding)
    one = _automodel().generate(input=paths, batch_size=1)
    assert [r["key"] for r in one] == [f"utt{i}" for i in range(len(paths))]
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, paths, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = [m for _, _, m, _ in out]
    assert sorted(shards[0] + shards[1]) == list(range(len(paths)))
    assert min(len(s) for s in shards) >= len(paths) // world
    for rank, res, _, how in out:
        assert how == "tensor", (rank, how)   # the greedy token matrices went over the collective as int32 tensors
        assert res == one, rank   # gathered in input order, token for token


def test_load_flat_device_matches_host_load():
    """pfm_set_weight_device (the DP ranks' path: weights stay in HBM after the RCCL broadcast) gives the same
    decode as pfm_set_weight from host memory, including the Conv1d / depthwise-tap re-layouts."""
    from funasr_amd.runtime import PfmEngine
    from funasr_amd.weights import make_weights, param_layout
    from tests.golden.inputs import fbank_input
    cfg = paraformer_tiny()
    sd = make_weights(cfg, 5)
    a = PfmEngine(cfg, 0)
    a.load_state_dict(sd)
    lay = param_layout(cfg)
    flat = torch.cat([torch.from_numpy(np.ascontiguousarray(sd[k], np.float32)).reshape(-1) for k, *_ in lay]).cuda()
    b = PfmEngine(cfg, 0)
    b.load_flat_device(flat, lay)
    assert b.missing_weights == 0
    feats, lens = fbank_input(seed=12, B=3, T=60, lens=[60, 41, 17])
    x, ln = torch.from_numpy(feats).cuda(), torch.from_numpy(lens).cuda()
    ra, rb = a.run(x, ln, mode="exact"), b.run(x, ln, mode="exact")
    torch.cuda.synchronize()
    for k in ("tokens", "ntok"):
        assert torch.equal(ra[k], rb[k]), k
    with pytest.raises(Exception):
        b.load_flat_device(flat[:100], lay)


@pytest.mark.parametrize("xw", [7, 0])
@pytest.mark.parametrize("large", [False, True])
def test_bf16_wire_weights_fast_mode_bit_identical(monkeypatch, large, xw):
    """broadcast_state_dict(wire="bf16") (the fast-mode data-parallel broadcast: 520 instead of 880 MB for
    Paraformer-large) leaves every rank bf16-rounded matrices; fast mode reads those only through bf16 copies (or,
    for the decoder w_2 / CIF projection, receives them in f32), so its decode is bit-identical to the f32-loaded
    engine's (under PFM_FAST_XW the split-plane weights travel as f32); EXACT mode is refused on such an engine."""
    monkeypatch.setenv("PFM_FAST_XW", str(xw))
    from funasr_amd.config import paraformer_large
    from funasr_amd.distributed import bf16_wire_round
    from funasr_amd.runtime import PfmEngine, PfmError
    from funasr_amd.weights import make_weights, param_layout
    from tests.golden.inputs import fbank_input
    cfg = paraformer_large() if large else paraformer_tiny()
    sd = make_weights(cfg, 5)
    a = PfmEngine(cfg, 0)
    a.load_state_dict(sd)
    lay = param_layout(cfg)
    flat = torch.cat([torch.from_numpy(np.ascontiguousarray(sd[k], np.float32)).reshape(-1) for k, *_ in lay]).cuda()
    b = PfmEngine(cfg, 0)
    b.load_flat_device(bf16_wire_round(flat, lay), lay, fast_only=True)
    B, T = (24, 500) if large else (3, 60)
    feats, lens = fbank_input(seed=12, B=B, T=T, lens=[T - 7 * i for i in range(B)])
    x, ln = torch.from_numpy(feats).cuda(), torch.from_numpy(lens).cuda()
    ra = a.run(x, ln, mode="fast", want_enc=True, want_alphas=True)
    rb = b.run(x, ln, mode="fast", want_enc=True, want_alphas=True)
    torch.cuda.synchronize()
    for k in ("tokens", "ntok", "enc", "alphas"):
        assert torch.equal(ra[k], rb[k]), k
    with pytest.raises(PfmError):
        b.run(x, ln, mode="exact")


def _large_tokint_automodel():
    from funasr_amd.auto_model import AutoModel
    from funasr_amd.config import paraformer_large
    return AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), synthetic_seed=0,
                     device="cuda", mode="exact", **paraformer_large().reference_kwargs())


def _dp_worker_large(rank, world, port, paths, bs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        am = _large_tokint_automodel()
        q.put((rank, am.generate(input=paths, batch_size=bs), am.last_gather))
    finally:
        dist.destroy_process_group()


def test_exact_tile_policy_batch_invariant_large():
    """EXACT mode's GEMM tiles do not change any row's arithmetic (verdict r5 item 6): 24 Paraformer-large utterances of
    equal length (T = 500 LFR frames, no padding differences) decode to the same tokens, counts and CIF alphas in one
    batch of 24 (M = 12,000 rows: 256 x 256 tiles, two encoder groups) as one at a time (M = 500: 128 x 256 tiles).
    Before round 6 the policy switched MFMA shapes with the grid (32x32x16 below 256 tiles, 16x16x32 above)."""
    from funasr_amd.config import paraformer_large
    from funasr_amd.runtime import PfmEngine
    from funasr_amd.weights import make_weights
    from tests.golden.inputs import fbank_input
    cfg = paraformer_large()
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    B, T = 24, 500
    x, l = fbank_input(seed=77, B=B, T=T, lens=[T] * B)
    xs, ls = torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda()
    rb = e.run(xs, ls, mode="exact", want_alphas=True)
    torch.cuda.synchronize()
    tb, nb, ab = rb["tokens"].cpu(), rb["ntok"].cpu(), rb["alphas"].cpu()
    for i in range(B):
        r1 = e.run(xs[i:i + 1], ls[i:i + 1], mode="exact", want_alphas=True)
        torch.cuda.synchronize()
        assert int(r1["ntok"][0]) == int(nb[i]), i
        n = int(nb[i])
        assert torch.equal(r1["tokens"][0, :n].cpu(), tb[i, :n]), i
        assert torch.equal(r1["alphas"][0].cpu(), ab[i]), i


def _dp_worker_large(rank, world, port, paths, bs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        am = _large_tokint_automodel()
        q.put((rank, am.generate(input=paths, batch_size=bs), am.last_gather))
    finally:
        dist.destroy_process_group()


def test_exact_dp_shards_decode_as_their_batches_large(tmp_path):
    """Data parallelism adds nothing to batching (SURVEY §4's multi-GPU token matrix): ragged Paraformer-large waveforms
    through the world-2 shared-device path at batch_size 7 (each rank decodes its length-sorted shard as one batch)
    equal one process decoding the same shards as the same batches, utterance for utterance. (Across DIFFERENT
    batchings of ragged input the reference itself differs: CifPredictorV2.forward, cif_predictor.py:212-224, convolves
    the unmasked encoder output, so an utterance's last frame sees the first padded frame of its batch; the path
    reproduces that, as the ragged reference goldens show, and the tile policy adds nothing, as the test above shows.)"""
    import torch.multiprocessing as mp
    from funasr_amd.distributed import item_lengths, length_sorted_shards
    paths = _wav_files(tmp_path)
    world = 2
    shards = length_sorted_shards(item_lengths(paths), world)
    am = _large_tokint_automodel()
    want = [None] * len(paths)
    for sh in shards:
        res = am.generate(input=[paths[i] for i in sh], batch_size=7)
        for i, r in zip(sh, res):
            want[i] = r
    del am
    torch.cuda.empty_cache()
    assert all(w is not None and len(w["token_int"]) > 0 for w in want)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker_large, args=(r, world, port, paths, 7, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, how in out:
        assert how == "tensor", (rank, how)
        assert res == want, rank
