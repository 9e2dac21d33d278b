"""ORACLE — CPU restatement of the reference CT-Transformer punctuation forward (TEST INFRASTRUCTURE).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this module,
and only as the checker. The product path (`funasr_amd.*`) never imports it.

Pinning: tests/test_oracle_golden.py checks it against tests/golden/punc_tiny.npz, the logits of every
`punc_forward` call the real reference `CTTransformer.inference` made (tests/golden/make_golden.py, `punc`).

  punc_forward   funasr/models/ct_transformer/model.py:81-93: embed (Embedding) -> SANMEncoder
                 (sanm/encoder.py:361-430, input_layer "pe": x * sqrt(output_size) + PE, layer 0 keeps its
                 residual since input_size == output_size) -> decoder Linear(att_unit, len(punc_list));
                 the caller takes topk(1) = argmax (first index on ties) per token (model.py:264-266)
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .paraformer_ref import as_torch_weights, encoder


@torch.no_grad()
def punc_forward(ids, lens, w, cfg):
    """ids [B, T] int, lens [B] -> logits [B, T, n_punc] f32 (torch-CPU)."""
    w = as_torch_weights(w)
    ids = torch.as_tensor(np.asarray(ids), dtype=torch.int64)
    lens = torch.as_tensor(np.asarray(lens), dtype=torch.int64)
    x = F.embedding(ids, w["embed.weight"])
    enc, _ = encoder(x, lens, w, cfg)
    return F.linear(enc, w["decoder.weight"], w["decoder.bias"])
