"""ORACLE — CPU restatement of the reference FSMN-VAD encoder (TEST INFRASTRUCTURE).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module, and
only as the checker. The product path (`funasr_amd.*`) never imports it.

Pinning: tests/test_oracle_golden.py checks it against tests/golden/vad.npz, the silence posteriors the
real reference FsmnVADStreaming.inference computed (tests/golden/make_golden.py, `vad`), on features from
oracle/streaming_ref.FrontendOnline with LFR (5, 1).

  vad_forward   funasr/models/fsmn_vad_streaming/encoder.py:241-279 (FSMN.forward with its cache dict):
                in_linear1 -> in_linear2 -> ReLU -> fsmn_layers x BasicBlock (linear (no bias) ->
                FSMNBlock (:36-90: x + Conv2d[lorder,1] over [cache ; x], the cache keeps the last
                (lorder-1) rows) -> affine -> ReLU) -> out_linear1 -> out_linear2 -> softmax
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .paraformer_ref import as_torch_weights


@torch.no_grad()
def vad_forward(feats, w, cfg, cache=None):
    """feats [T, input_dim] (one chunk of one stream), cache: dict carried between chunks (created when
    None) -> (posteriors [T, output_dim], cache)."""
    w = as_torch_weights(w)
    x = torch.as_tensor(np.asarray(feats, np.float32))
    cache = {} if cache is None else cache

    def aff(h, name, bias=True):
        return F.linear(h, w[f"{name}.linear.weight"], w[f"{name}.linear.bias"] if bias else None)

    h = torch.relu(aff(aff(x, "encoder.in_linear1"), "encoder.in_linear2"))
    L = cfg.lorder
    for i in range(cfg.fsmn_layers):
        p = f"encoder.fsmn.{i}"
        a = aff(h, f"{p}.linear", bias=False)                       # [T, P]
        prev = cache.get(i, torch.zeros((L - 1, a.shape[1])))
        full = torch.cat([prev, a])                                  # [L-1+T, P]
        cache[i] = full[-(L - 1):] if L > 1 else prev
        wt = w[f"{p}.fsmn_block.conv_left.weight"][:, 0, :, 0]       # [P, L]
        conv = F.conv1d(full.t()[None], wt[:, None, :], groups=wt.shape[0])[0].t()
        h = torch.relu(aff(a + conv, f"{p}.affine"))
    logits = aff(aff(h, "encoder.out_linear1"), "encoder.out_linear2")
    return torch.softmax(logits, dim=-1), cache
