"""Utterance data parallelism over one process per GPU (torch.distributed: RCCL on MI355X,
gloo on CPU for tests).

The Paraformer path has no exchange inside a forward pass: utterances are
independent. So the only collectives are
  * one weight broadcast from rank 0 at start-up (`broadcast_state_dict`, one flat fp32
    buffer — 880 MB for Paraformer-large, a single large RCCL broadcast over xGMI),
  * (API path only) an all-gather of the per-rank results after a batch (`gather_results`).
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


def broadcast_state_dict(layout, sd: Optional[Dict[str, np.ndarray]], device=None, src: int = 0,
                         keep_on_device: bool = False):
    """Broadcast a state_dict from `src` as ONE flat fp32 tensor; returns it on every rank.

    layout: [(key, shape, ...)] in a fixed order known to all ranks (weights.param_layout).
    sd: the dict on `src` (ignored elsewhere). device: torch device of the collective
    (cuda for RCCL, cpu for gloo). keep_on_device: return the flat tensor itself (for
    PfmEngine.load_flat_device: no device -> host -> device round trip) instead of a host dict.
    """
    import torch
    import torch.distributed as dist
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
    dist.broadcast(flat, src)
    if keep_on_device:
        return flat
    host = flat.cpu().numpy() if dev.type != "cpu" else flat.numpy()
    out, off = {}, 0
    for (k, s, *_), n in zip(layout, sizes):
        out[k] = host[off:off + n].reshape(s)
        off += n
    return out


def gather_results(local: list) -> list:
    """All-gather python result lists (rank order) — API path only, never in the timed step."""
    import torch.distributed as dist
    world = dist.get_world_size()
    bucket = [None] * world
    dist.all_gather_object(bucket, local)
    return [x for part in bucket for x in part]
