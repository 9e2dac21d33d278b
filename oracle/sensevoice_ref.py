"""ORACLE — CPU restatement of the reference SenseVoiceSmall inference path (TEST INFRASTRUCTURE).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker. The product path never imports it.

Pinning: tests/test_oracle_golden.py checks it against goldens produced by the real reference
`SenseVoiceSmall` (tests/golden/make_golden.py, sense_voice_*.npz).

ATen fp32 on CPU, one function per reference stage:

  query rows + concat   funasr/models/sense_voice/model.py:851-876 (inference)
  encoder               funasr/models/sense_voice/model.py:553-585 (SenseVoiceEncoderSmall.forward)
  encoder layer         funasr/models/sense_voice/model.py:329-405 (EncoderLayerSANM, eps 1e-5 :275-287)
  SAN-M attention       funasr/models/sense_voice/model.py:129-233 (same algebra as
                        oracle.paraformer_ref.sanm_self_attention)
  CTC head              funasr/models/ctc/ctc.py:173-184 (log_softmax(ctc_lo(x)))
  greedy CTC            funasr/models/sense_voice/model.py:893-906 (argmax, unique_consecutive,
                        drop blank)
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

from .paraformer_ref import as_torch_weights, encoder_layer, layer_norm, pad_mask, pos_encoding

Tensor = torch.Tensor


def query_ids(cfg, language: str = "auto", use_itn: bool = False, text_norm=None) -> List[int]:
    """Embedding rows prepended to every utterance: [language, 1 (event), 2 (emotion), textnorm]
    (model.py:851-876)."""
    lid = cfg.lid_dict[language] if language in cfg.lid_dict else 0
    if text_norm is None:
        text_norm = "withitn" if use_itn else "woitn"
    return [lid, 1, 2, cfg.textnorm_dict[text_norm]]


def build_input(feats: Tensor, lens: Tensor, w: Dict[str, Tensor], qids: List[int]):
    """[B,T,I] -> [B,T+4,I] with the four query embeddings in front; lens + 4."""
    B = feats.shape[0]
    q = w["embed.weight"][torch.as_tensor(qids)]                 # [4, I]
    x = torch.cat([q[None].expand(B, -1, -1), feats], dim=1)
    return x, lens + 4


def encoder(x: Tensor, olens: Tensor, w: Dict[str, Tensor], cfg) -> Tensor:
    B, T, I = x.shape
    m = pad_mask(olens, T)
    x = x * cfg.d_model ** 0.5
    x = x + pos_encoding(T, I)[None]
    x = encoder_layer(x, m, w, "encoder.encoders0.0", cfg)
    for i in range(cfg.enc_blocks - 1):
        x = encoder_layer(x, m, w, f"encoder.encoders.{i}", cfg)
    x = layer_norm(x, w["encoder.after_norm.weight"], w["encoder.after_norm.bias"], cfg.ln_eps)
    for i in range(cfg.tp_blocks):
        x = encoder_layer(x, m, w, f"encoder.tp_encoders.{i}", cfg)
    return layer_norm(x, w["encoder.tp_norm.weight"], w["encoder.tp_norm.bias"], cfg.ln_eps)


def ctc_greedy(frame_ids: Tensor, olens: Tensor, blank: int) -> List[List[int]]:
    out = []
    for i in range(frame_ids.shape[0]):
        y = torch.unique_consecutive(frame_ids[i, : int(olens[i])], dim=-1)
        out.append(y[y != blank].tolist())
    return out


@torch.no_grad()
def sensevoice_infer(feats, lens, w, cfg, language="auto", use_itn=False, text_norm=None,
                     ban_emo_unk=False, keep_logits=False) -> dict:
    """SenseVoiceSmall.inference for data_type='fbank' up to token_int (model.py:809-906)."""
    feats = feats if isinstance(feats, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(feats))
    lens = (lens if isinstance(lens, torch.Tensor) else torch.as_tensor(lens)).to(torch.int64).reshape(-1)
    w = as_torch_weights(w)
    x, olens = build_input(feats.to(torch.float32), lens, w, query_ids(cfg, language, use_itn, text_norm))
    enc = encoder(x, olens, w, cfg)
    logits = F.linear(enc, w["ctc.ctc_lo.weight"], w["ctc.ctc_lo.bias"])
    logp = torch.log_softmax(logits, dim=2)
    if ban_emo_unk:
        logp[:, :, cfg.emo_unk] = -float("inf")
    frame_ids = logp.argmax(dim=-1)
    res = dict(enc=enc, enc_lens=olens, frame_ids=frame_ids, tokens=ctc_greedy(frame_ids, olens, cfg.blank_id))
    if keep_logits:
        res["logp"] = logp
    return res
