"""Multi-process data-parallel plumbing on CPU with gloo (world_size 2): the same
funasr_amd.distributed functions bench.py / AutoModel run over RCCL on the GPU node."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from funasr_amd.distributed import broadcast_state_dict, gather_results, length_sorted_shards, shard_range


def test_shard_range_covers_exactly():
    for n in [1, 2, 5, 64, 513]:
        for world in [1, 2, 3, 4, 8]:
            spans = [shard_range(n, world, r) for r in range(world)]
            got = [i for a, b in spans for i in range(a, b)]
            assert got == list(range(n))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_length_sorted_shards_balance():
    lens = [500, 83, 431, 500, 120, 300, 222, 17]
    sh = length_sorted_shards(lens, 2)
    assert sorted(sum(sh, [])) == list(range(len(lens)))
    tot = [sum(lens[i] for i in s) for s in sh]
    assert abs(tot[0] - tot[1]) <= max(lens)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        layout = [("encoder.encoders.0.feed_forward.w_1.weight", (3, 4), 4), ("b.bias", (5,), 4),
                  ("decoder.decoders.0.feed_forward.w_2.weight", (2, 2, 2), 8)]
        sd = None
        if rank == 0:
            rng = np.random.default_rng(0)
            sd = {k: rng.standard_normal(s).astype(np.float32) for k, s, _ in layout}
        got = broadcast_state_dict(layout, sd)
        got16 = broadcast_state_dict(layout, sd, wire="bf16")
        items = list(range(11))
        lo, hi = shard_range(len(items), world, rank)
        local = [{"key": f"u{i}", "rank": rank} for i in items[lo:hi]]
        allres = gather_results(local)
        q.put((rank, {k: v.tolist() for k, v in got.items()}, allres, {k: v.tolist() for k, v in got16.items()}))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_broadcast_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda x: x[0])
    rng = np.random.default_rng(0)
    want = {k: rng.standard_normal(s).astype(np.float32).tolist() for k, s in
            [("encoder.encoders.0.feed_forward.w_1.weight", (3, 4)), ("b.bias", (5,)),
             ("decoder.decoders.0.feed_forward.w_2.weight", (2, 2, 2))]}
    # bf16 wire: the encoder FFN matrix arrives bf16-rounded; the bias and the decoder w_2 (read in f32 by fast
    # mode's folded LayerNorm) exact
    want16 = {k: (torch.tensor(v).to(torch.bfloat16).float().tolist() if ".w_1." in k else v)
              for k, v in want.items()}
    for rank, sd, allres, sd16 in out:
        assert sd == want
        assert sd16 == want16
        assert [r["key"] for r in allres] == [f"u{i}" for i in range(11)]
        assert [r["rank"] for r in allres] == [0] * 6 + [1] * 5


class _EchoModel:
    """Stands in for the HIP model inside AutoModel.inference: one result per input, tagged with the rank."""

    def eval(self):
        return self

    def inference(self, data_in, key=None, **kw):
        rank = dist.get_rank() if dist.is_initialized() else 0
        return [{"key": k, "n": int(len(x)), "rank": rank} for k, x in zip(key, data_in)], {}


def _infer_worker(rank, world, port, items, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from funasr_amd.auto_model import AutoModel
        am = AutoModel.__new__(AutoModel)
        am.kwargs, am.model = {"batch_size": 2}, _EchoModel()
        q.put((rank, am.inference(items, key=None)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_automodel_inference_length_sorted_order_restored():
    """AutoModel.inference under world 2: longest-first round-robin shards (both ranks get similar padded
    work), results all-gathered back into input order; identical to the one-process run minus the rank tag."""
    from funasr_amd.auto_model import AutoModel
    lens = [500, 83, 431, 500, 120, 300, 222, 17, 260]
    items = [np.zeros(n, np.float32) for n in lens]
    single = AutoModel.__new__(AutoModel)
    single.kwargs, single.model = {"batch_size": 2}, _EchoModel()
    want = [{k: v for k, v in r.items() if k != "rank"} for r in single.inference(items)]
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_infer_worker, args=(r, world, port, items, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out:
        assert [r["n"] for r in res] == lens
        assert [{k: v for k, v in r.items() if k not in ("rank", "key")} for r in res] == \
            [{k: v for k, v in r.items() if k != "key"} for r in want]
        per_rank = [sum(r["n"] for r in res if r["rank"] == k) for k in range(world)]
        assert abs(per_rank[0] - per_rank[1]) <= max(lens)
        assert {r["rank"] for r in res if r["n"] == 500} == {0, 1}   # the two longest go to different ranks


class _NbestModel(_EchoModel):
    """An n-best model: two results per input (best first), none for a 17-sample input (a search that ended no
    hypothesis), with meta["owner"] naming each result's batch index (what Paraformer.inference returns)."""

    def inference(self, data_in, key=None, **kw):
        rank = dist.get_rank() if dist.is_initialized() else 0
        res, owner = [], []
        for i, (k, x) in enumerate(zip(key, data_in)):
            if len(x) == 17:
                continue
            for n in range(2):
                res.append({"key": k, "n": int(len(x)), "hyp": n, "rank": rank})
                owner.append(i)
        return res, {"owner": owner}


def _nbest_worker(rank, world, port, items, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from funasr_amd.auto_model import AutoModel
        am = AutoModel.__new__(AutoModel)
        am.kwargs, am.model = {"batch_size": 3}, _NbestModel()
        # rank 1 sees every input as empty: the shard plan must still be rank 0's (broadcast), not its own
        mine = items if rank == 0 else [np.zeros(0, np.float32) for _ in items]
        from funasr_amd.distributed import shard_items
        q.put((rank, shard_items(mine, world, rank), am.inference(items, key=None)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_automodel_nbest_grouped_by_input():
    """AutoModel.inference under world 2 with an n-best model: results are grouped by the input they belong to
    (meta owner), inputs without a hypothesis contribute none, n-best order inside an input is kept; equal to
    the one-process run. The shard plan is rank 0's on every rank."""
    from funasr_amd.auto_model import AutoModel
    from funasr_amd.distributed import item_lengths
    lens = [500, 83, 17, 431, 500, 120, 300, 222, 260]
    items = [np.zeros(n, np.float32) for n in lens]
    single = AutoModel.__new__(AutoModel)
    single.kwargs, single.model = {"batch_size": 3}, _NbestModel()
    want = [{k: v for k, v in r.items() if k not in ("rank", "key")} for r in single.inference(items)]
    assert len(want) == 2 * (len(lens) - 1)
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_nbest_worker, args=(r, world, port, items, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    plan = length_sorted_shards(item_lengths(items), world)
    for rank, shard, res in out:
        assert shard == plan[rank]
        assert [{k: v for k, v in r.items() if k not in ("rank", "key")} for r in res] == want


class _TokenModel(_EchoModel):
    """A greedy model: per input a row of token ids (position p of input with n samples -> (n + 7 p) % 97, with
    the specials 0 / 1 / 2 among them), count = n % 13; results built from the token matrix like
    Paraformer.results_from_token_matrix, and the matrix returned in meta["token_matrix"]."""
    L = 16

    def _mat(self, data_in):
        b = len(data_in)
        t = torch.full((b, self.L), -1, dtype=torch.int32)
        nt = torch.zeros(b, dtype=torch.int32)
        for i, x in enumerate(data_in):
            n = len(x)
            nt[i] = n % 13
            t[i, :] = torch.tensor([(n + 7 * p) % 97 for p in range(self.L)], dtype=torch.int32)
        return t, nt

    def results_from_token_matrix(self, toks, ntok, key, tokenizer=None, **kw):
        return [{"key": key[i], "ids": [int(v) for v in toks[i, :int(ntok[i])] if v not in (0, 1, 2)]}
                for i in range(len(ntok))]

    def inference(self, data_in, key=None, **kw):
        t, nt = self._mat(data_in)
        return self.results_from_token_matrix(t.numpy(), nt.numpy(), key), {"token_matrix": (t, nt)}


def _token_worker(rank, world, port, items, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from funasr_amd.auto_model import AutoModel
        am = AutoModel.__new__(AutoModel)
        am.kwargs, am.model = {"batch_size": 2}, _TokenModel()
        called = []
        import funasr_amd.distributed as D
        orig = D.gather_results
        D.gather_results = lambda local: called.append(1) or orig(local)
        res = am.inference(items, key=[f"k{i}" for i in range(len(items))])
        err = None
        try:   # rank 1 sees one input fewer: every rank must raise instead of entering different collectives
            am.inference(items if rank == 0 else items[:-1], key=None)
        except RuntimeError as e:
            err = str(e)
        q.put((rank, res, len(called), err))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_token_matrix_tensor_gather():
    """Greedy results under world 2 come from the token matrices gathered as int32 tensors (no pickled result
    objects) and equal the one-process run in input order; mismatched input counts raise on every rank."""
    from funasr_amd.auto_model import AutoModel
    lens = [500, 83, 17, 431, 500, 120, 300, 222, 260]
    items = [np.zeros(n, np.float32) for n in lens]
    single = AutoModel.__new__(AutoModel)
    single.kwargs, single.model = {"batch_size": 2}, _TokenModel()
    want = single.inference(items, key=[f"k{i}" for i in range(len(items))])
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_token_worker, args=(r, world, port, items, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, n_obj_gathers, err in out:
        assert res == want
        assert n_obj_gathers == 0
        assert err is not None and "different input counts" in err


class _WriterModel(_EchoModel):
    """Writes output_dir files like Paraformer.inference (model_writer: {n}best_recog/{token,text})."""

    def inference(self, data_in, key=None, **kw):
        from funasr_amd.writer import model_writer
        w = model_writer(self, kw)
        res = []
        for k, x in zip(key, data_in):
            if w is not None:
                w["1best_recog"]["token"][k] = " ".join(["t"] * (len(x) % 5 + 1))
                w["1best_recog"]["text"][k] = f"len{len(x)}"
            res.append({"key": k, "n": int(len(x))})
        return res, {}


def _writer_worker(rank, world, port, items, out_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from funasr_amd.auto_model import AutoModel
        am = AutoModel.__new__(AutoModel)
        am.kwargs, am.model = {"batch_size": 2}, _WriterModel()
        res = am.inference(items, key=None, output_dir=out_dir)
        # dp=False: a call on one rank alone enters no collective (it would hang here otherwise)
        solo = am.inference(items[:3], key=None, dp=False) if rank == 0 else None
        q.put((rank, res, solo))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_output_dir_merged_in_input_order(tmp_path):
    """generate(..., output_dir) under world 2: each rank writes its share into a directory of its own and rank 0
    merges them into output_dir/1best_recog/{token,text} in input order -- the files a one-process run writes,
    nothing truncated or overwritten; the rank directories are gone afterwards. dp=False calls are rank-local."""
    from funasr_amd.auto_model import AutoModel
    lens = [500, 83, 17, 431, 500, 120, 300, 222, 260]
    items = [np.zeros(n, np.float32) for n in lens]
    d1, d2 = tmp_path / "one", tmp_path / "two"
    single = AutoModel.__new__(AutoModel)
    single.kwargs, single.model = {"batch_size": 2}, _WriterModel()
    want_res = single.inference(items, key=None, output_dir=str(d1))
    single.model.writer.close()
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_writer_worker, args=(r, world, port, items, str(d2), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys = None
    for rank, res, solo in out:
        assert [r["n"] for r in res] == lens
        keys = [r["key"] for r in res] if keys is None else keys
        assert [r["key"] for r in res] == keys   # one key list on every rank (rank 0's)
        if rank == 0:
            assert [r["n"] for r in solo] == lens[:3]
    assert sorted(os.listdir(d2)) == ["1best_recog"]
    for name in ("token", "text"):
        got = (d2 / "1best_recog" / name).read_text(encoding="utf-8").splitlines()
        ref = (d1 / "1best_recog" / name).read_text(encoding="utf-8").splitlines()
        assert [g.split(" ", 1)[0] for g in got] == keys
        assert [g.split(" ", 1)[1] for g in got] == [r.split(" ", 1)[1] for r in ref]
    assert [r["n"] for r in want_res] == lens


def _xw_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["PFM_FAST_XW"] = "7" if rank == 0 else "0"   # the ranks disagree: src's bits must win
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        layout = [("encoder.encoders.3.self_attn.linear_q_k_v.weight", (6, 4), 4), ("b.bias", (5,), 4)]
        sd = None
        if rank == 0:
            rng = np.random.default_rng(1)
            sd = {k: rng.standard_normal(s).astype(np.float32) for k, s, _ in layout}
        got, xw = broadcast_state_dict(layout, sd, wire="bf16", with_xw=True)
        q.put((rank, xw, {k: v.tolist() for k, v in got.items()}))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bf16_wire_uses_src_xw_bits():
    """broadcast_state_dict(wire="bf16") splits by the source rank's PFM_FAST_XW even where another rank's
    environment says otherwise (the two would post collectives of different sizes): with bit 4 the q|k rows of an
    encoder QKV arrive bf16-rounded and the v rows exact on every rank, and both report xw = 7."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_xw_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(1)
    w = rng.standard_normal((6, 4)).astype(np.float32)
    want = torch.tensor(w)
    want[:4] = want[:4].to(torch.bfloat16).float()
    for rank, xw, got in out:
        assert xw == 7
        assert got["encoder.encoders.3.self_attn.linear_q_k_v.weight"] == want.tolist()
