"""Utterance data parallelism over one process per GPU (torch.distributed: RCCL on MI355X,
gloo on CPU for tests).

The Paraformer path has no exchange inside a forward pass: utterances are
independent. So the only collectives are
  * one weight broadcast from rank 0 at start-up (`broadcast_state_dict`: one flat fp32 buffer, 880 MB for
    Paraformer-large, or for fast-mode serving the bf16-only matrix rows as bf16 and the rest as f32, 520 MB; large RCCL
    broadcasts over xGMI),
  * (API path only) after the rank's batches, an all-gather of its greedy token matrices as tensors
    (`gather_token_matrices`: [n, L] int32 ids + counts + input indices, RCCL on the GPU), from which every rank
    builds the results; result kinds that are not a function of the token matrix (timestamps, n-best, SenseVoice)
    are all-gathered as Python objects (`gather_results`).
The timed benchmark step has no collective at all: each rank decodes its own shard.
The reference's only multi-GPU inference is one process per GPU over a split scp list
(examples/aishell/paraformer/run.sh:136-170); `shard_range` is that split, in-process.
AutoModel.inference deals utterances longest-first round-robin instead (`length_sorted_shards`
over `item_lengths`), so every rank gets a similar amount of padded audio, and all-gathers
(index, result) pairs to restore the input order.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced utterance slice [start, end) of n items for `rank`."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def length_sorted_shards(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Balance padded work: sort by length, deal round-robin so every rank gets similar T."""
    order = np.argsort(-np.asarray(lengths), kind="stable")
    return [order[r::world].tolist() for r in range(world)]


def shard_items(items: Sequence, world: int, rank: int) -> List[int]:
    """This rank's input indices: rank 0 measures the items (item_lengths) and deals them with
    length_sorted_shards; the deal is broadcast, so every rank shards identically even where its own view of
    the inputs differs (node-local paths, a file still being written)."""
    import torch.distributed as dist
    plan = [length_sorted_shards(item_lengths(items), world) if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(plan, src=0)
    shards = plan[0]
    if sorted(i for s in shards for i in s) != list(range(len(items))):
        raise RuntimeError(f"data-parallel shard plan does not cover the {len(items)} inputs of rank {rank}")
    return shards[rank]


def item_lengths(items: Sequence) -> List[int]:
    """Cheap per-item work estimate for sharding without decoding anything: samples / frames of
    in-memory arrays, the byte size of files and byte strings, 0 when unknown."""
    import os
    out = []
    for x in items:
        if hasattr(x, "shape") and len(getattr(x, "shape", ())) > 0:
            out.append(int(x.shape[0]))
        elif isinstance(x, (bytes, bytearray)):
            out.append(len(x))
        elif isinstance(x, str) and os.path.isfile(x):
            out.append(int(os.path.getsize(x)))
        elif isinstance(x, (list, tuple)):
            out.append(len(x))
        else:
            out.append(0)
    return out


# The matrices fast mode reads ONLY through their bf16 copies (the library's GEMM-flagged weights, pfm_api.hip
# add_entry(..., true)), minus the decoder FFNs' w_2 (their LayerNorm is folded through it in f32:
# W2g = bf16(W2 diag(gamma)), c2 = W2 beta). Everything else -- FSMN taps (f32 depthwise arithmetic), the CIF alpha
# projection, biases, LayerNorms -- is read in f32 and travels as f32.
_BF16_WIRE_SUFFIXES = ("self_attn.linear_out.weight", "self_attn.linear_q_k_v.weight", "feed_forward.w_1.weight",
                       "src_attn.linear_q.weight", "src_attn.linear_k_v.weight", "src_attn.linear_out.weight",
                       "decoder.output_layer.weight", "ctc.ctc_lo.weight", "predictor.cif_conv1d.weight")


def fast_xw_bits() -> int:
    """The library's PFM_FAST_XW (default 7; bit 8 implies 4), as pfm_api.hip reads it."""
    import os
    v = os.environ.get("PFM_FAST_XW", "")
    b = (int(v) if v.strip() else 7) & 15
    return b | 4 if b & 8 else b


def bf16_wire_rows(key: str, shape, xw: int = None):
    """Rows [r0, r1) of weight `key` that fast mode reads only through their bf16 copies (sent as bf16 by
    wire="bf16"; the rest of the tensor travels as f32). Under PFM_FAST_XW the split-plane weights are read in f32
    (their lo planes w - bf16(w)): bit 1 the predictor conv, bit 2 encoder layer 0 (and layer 1's QKV GEMM), bit 4
    the v rows of every encoder QKV projection, bit 8 every encoder out-projection."""
    xw = fast_xw_bits() if xw is None else xw
    rows = int(shape[0]) if len(shape) else 0
    bf = key.endswith(_BF16_WIRE_SUFFIXES) or (key.startswith("encoder.") and key.endswith("feed_forward.w_2.weight"))
    if not bf:
        return 0, 0
    if (xw & 1) and key.startswith("predictor."):
        return 0, 0
    if (xw & 2) and key.startswith("encoder.encoders0."):
        return 0, 0
    if (xw & 8) and key.startswith("encoder.") and key.endswith("self_attn.linear_out.weight"):
        return 0, 0
    if (xw & 4) and key.startswith("encoder.") and key.endswith("self_attn.linear_q_k_v.weight"):
        return 0, 2 * rows // 3   # q | k rows bf16, the v rows f32
    return 0, rows


def bf16_wire_key(key: str, shape, xw: int = None) -> bool:
    """True when every element of the weight travels as bf16 under wire="bf16"."""
    r0, r1 = bf16_wire_rows(key, shape, xw)
    return r1 > r0 and r1 - r0 == int(shape[0])


def _wire_index(layout, dev, xw: int = None):
    """Flat indices of the bf16-wire elements and of the f32 ones."""
    import torch
    sizes = [int(np.prod(s)) for _, s, *_ in layout]
    mat = np.zeros(int(sum(sizes)), dtype=bool)
    off = 0
    for (k, s, *_), n in zip(layout, sizes):
        r0, r1 = bf16_wire_rows(k, s, xw)
        if r1 > r0:
            row = n // int(s[0])
            mat[off + r0 * row:off + r1 * row] = True
        off += n
    return torch.from_numpy(np.nonzero(mat)[0]).to(dev), torch.from_numpy(np.nonzero(~mat)[0]).to(dev)


def bf16_wire_round(flat, layout, xw: int = None):
    """What a receiving rank holds after broadcast_state_dict(wire="bf16"): `flat` (f32, layout order) with the
    bf16-wire elements rounded to bf16 (in place; returned)."""
    import torch
    mi, _ = _wire_index(layout, flat.device, xw)
    flat[mi] = flat[mi].to(torch.bfloat16).to(torch.float32)
    return flat


def broadcast_state_dict(layout, sd: Optional[Dict[str, np.ndarray]], device=None, src: int = 0,
                         keep_on_device: bool = False, wire: str = "f32", with_xw: bool = False):
    """Broadcast a state_dict from `src` in one (f32) or two (bf16 wire) flat collectives; returns it on every rank.

    layout: [(key, shape, ...)] in a fixed order known to all ranks (weights.param_layout).
    sd: the dict on `src` (ignored elsewhere). device: torch device of the collective
    (cuda for RCCL, cpu for gloo). keep_on_device: return the flat f32 tensor itself (for
    PfmEngine.load_flat_device: no device -> host -> device round trip) instead of a host dict.
    wire: "f32" sends every weight as f32 (880 MB for Paraformer-large); "bf16" sends the matrix rows fast mode reads
    only through their bf16 copies (`bf16_wire_rows`, for the PFM_FAST_XW in effect) as bf16 and the rest as f32
    (486 MB at PFM_FAST_XW=0, 520 MB at the default 7). The
    receiving ranks' matrices are then bf16-rounded, which fast mode does not see (bf16(bf16(w)) = bf16(w): its
    decode is bit-identical, tests/test_gpu_automodel.py) but EXACT mode would: load them with
    PfmEngine.load_flat_device(..., fast_only=True, wire_xw=xw).
    The bf16 / f32 split depends on PFM_FAST_XW (its split-plane rows travel as f32), so under wire="bf16" the bits
    of `src` are broadcast first and every rank splits by them, whatever its own environment says (ranks that
    disagreed would otherwise post collectives of different sizes). with_xw=True returns (state, xw): pass xw to
    load_flat_device, which then refuses fast runs under any other PFM_FAST_XW (their split planes would be built
    from bf16-rounded weights with zero lo planes).
    """
    import torch
    import torch.distributed as dist
    if wire not in ("f32", "bf16"):
        raise ValueError(f"broadcast_state_dict: wire {wire!r} (f32 | bf16)")
    rank = dist.get_rank()
    sizes = [int(np.prod(s)) for _, s, *_ in layout]
    total = int(sum(sizes))
    dev = torch.device("cpu") if device is None else torch.device(device)
    flat = torch.empty(total, dtype=torch.float32, device=dev)
    if rank == src:
        host = np.empty(total, dtype=np.float32)
        off = 0
        for (k, s, *_), n in zip(layout, sizes):
            host[off:off + n] = np.asarray(sd[k], dtype=np.float32).reshape(-1)
            off += n
        flat.copy_(torch.from_numpy(host))
    xw = fast_xw_bits()
    if wire == "f32":
        dist.broadcast(flat, src)
    else:
        xwt = torch.tensor([xw], dtype=torch.int64, device=dev)
        dist.broadcast(xwt, src)
        xw = int(xwt.item())
        mi, vi = _wire_index(layout, dev, xw)
        mb = flat[mi].to(torch.bfloat16) if rank == src else torch.empty(mi.numel(), dtype=torch.bfloat16, device=dev)
        vf = flat[vi] if rank == src else torch.empty(vi.numel(), dtype=torch.float32, device=dev)
        dist.broadcast(mb, src)
        dist.broadcast(vf, src)
        flat[mi] = mb.to(torch.float32)   # every rank, src included: all hold the same bf16-rounded matrices
        flat[vi] = vf
    if keep_on_device:
        return (flat, xw) if with_xw else flat
    host = flat.cpu().numpy() if dev.type != "cpu" else flat.numpy()
    out, off = {}, 0
    for (k, s, *_), n in zip(layout, sizes):
        out[k] = host[off:off + n].reshape(s)
        off += n
    return (out, xw) if with_xw else out


def agree_item_count(n_items: int) -> int:
    """The ranks' input counts, all-gathered before any data-parallel collective; every rank raises when they differ
    (ranks whose views of the inputs differ would otherwise enter different collectives and hang)."""
    import torch
    import torch.distributed as dist
    dev = _coll_device()
    world = dist.get_world_size()
    mine = torch.tensor([n_items], dtype=torch.int64, device=dev)
    allc = torch.empty(world, dtype=torch.int64, device=dev)
    _all_gather_flat(allc, mine)
    counts = allc.cpu().tolist()
    if len(set(counts)) != 1:
        raise RuntimeError(f"data-parallel inference: the ranks see different input counts {counts}")
    return counts[0]


def _coll_device():
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":   # RCCL: device tensors over xGMI
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_token_matrices(parts, index: Sequence[int]):
    """All-gather this rank's greedy token matrices as tensors.

    parts: [(tokens [b, L_b] int32 device tensor, ntok [b] int32)] in decode order; index: the input index of every
    row (len = sum b). Returns host arrays (tokens [N, L] int32 padded with -1, ntok [N], index [N]) of all ranks,
    rows in rank order. Two collectives: the per-rank (rows, width) pair, then one padded [rows_max, width + 2]
    int32 block per rank (ids | ntok | input index) with all_gather_into_tensor (RCCL) / all_gather (gloo)."""
    import torch
    import torch.distributed as dist
    dev = _coll_device()
    world = dist.get_world_size()
    n = int(sum(int(t.shape[0]) for t, _ in parts))
    L = max([int(t.shape[1]) for t, _ in parts] + [1])
    shape = torch.tensor([n, L], dtype=torch.int64, device=dev)
    shapes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    _all_gather_flat(shapes, shape)
    sh = shapes.view(world, 2).cpu().numpy()
    nmax, Lmax = int(sh[:, 0].max()), int(sh[:, 1].max())
    blk = torch.full((max(nmax, 1), Lmax + 2), -1, dtype=torch.int32, device=dev)
    r0 = 0
    for t, nt in parts:
        b, lb = int(t.shape[0]), int(t.shape[1])
        blk[r0:r0 + b, :lb] = t.to(device=dev, dtype=torch.int32)
        blk[r0:r0 + b, Lmax] = nt.reshape(-1).to(device=dev, dtype=torch.int32)
        r0 += b
    if n:
        blk[:n, Lmax + 1] = torch.as_tensor(np.asarray(index, np.int32), device=dev)
    allb = torch.empty((world * blk.shape[0], Lmax + 2), dtype=torch.int32, device=dev)
    _all_gather_flat(allb, blk)
    allh = allb.view(world, blk.shape[0], Lmax + 2).cpu().numpy()
    rows = np.concatenate([allh[r, :int(sh[r, 0])] for r in range(world)], 0)
    return rows[:, :Lmax], rows[:, Lmax], rows[:, Lmax + 1]


def _all_gather_flat(out, t):
    """out = concat of t over ranks (rank order): all_gather_into_tensor where the backend has it."""
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, t.contiguous())
        return
    world = dist.get_world_size()
    chunks = list(out.view(world, *t.shape).unbind(0))
    dist.all_gather(chunks, t.contiguous())


def gather_results(local: list) -> list:
    """All-gather python result lists (rank order) — API path only, never in the timed step."""
    import torch.distributed as dist
    world = dist.get_world_size()
    bucket = [None] * world
    dist.all_gather_object(bucket, local)
    return [x for part in bucket for x in part]
