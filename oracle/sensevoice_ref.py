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
  timestamps            funasr/models/sense_voice/model.py:917-945 (softmax emission, blank zeroed where it
                        wins, ctc_forced_align of funasr/models/sense_voice/utils/ctc_alignment.py:2-60,
                        frame groups -> [token, start s, end s]) and post() (model.py:949-965)
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


def ctc_forced_align(emis: np.ndarray, targets: List[int], blank: int = 0) -> np.ndarray:
    """ctc_alignment.py:2-60 for one utterance (the batch of one the reference builds per utterance): Viterbi over
    the extended label sequence [blank, y1, blank, y2, ..., blank] of score + emis[t, label] in float32 (SenseVoice
    passes softmax probabilities, not logs), predecessors stay / previous / skip (skip only between different
    labels), ties to the first; the end state is the better of the last label and the final blank (first on a tie);
    back-tracking gives one extended state per frame, returned as its label id."""
    emis = np.asarray(emis, dtype=np.float32)
    T = emis.shape[0]
    L = len(targets)
    ext = [blank]
    for y in targets:
        ext += [int(y), blank]
    ext = np.asarray(ext, dtype=np.int64)
    S = len(ext)
    diff = np.zeros(S, dtype=bool)
    diff[2:] = ext[2:] != ext[:-2]
    ninf = np.float32(-np.inf)
    best = np.full(S + 2, ninf, dtype=np.float32)
    best[2] = emis[0, blank]
    best[3] = emis[0, ext[1]]          # IndexError for L == 0, as the reference
    bp = np.zeros((T, S + 2), dtype=np.int64)
    for t in range(1, T):
        prev = np.stack((best[2:], best[1:-1], np.where(diff, best[:-2], ninf)))
        idx = np.argmax(prev, axis=0)                       # first maximum (torch.max(dim=0) on CPU)
        val = prev[idx, np.arange(S)]
        best[2:] = (emis[t, ext] + val).astype(np.float32)
        bp[t, 2:] = idx
    l1l2 = best[[2 + 2 * L - 1, 2 + 2 * L]]
    path = np.zeros(T, dtype=np.int64)
    path[T - 1] = 2 + 2 * L - 1 + int(np.argmax(l1l2))
    for t in range(T - 1, 0, -1):
        path[t - 1] += path[t] - bp[t, path[t]]
    return ext[np.clip(path - 2, 0, None)]


def timestamp_emission(logits: np.ndarray, blank: int = 0) -> np.ndarray:
    """model.py:920-922: softmax of the CTC head over the utterance's speech frames, with the blank probability
    set to 0 on frames whose argmax is the blank."""
    p = torch.softmax(torch.as_tensor(np.asarray(logits, dtype=np.float32)), dim=-1)
    pred = p.argmax(-1)
    p[pred == blank, blank] = 0
    return p.numpy()


def timestamp_groups(align: np.ndarray, n_frames: int, ts_max: int, pieces: List[str]) -> list:
    """model.py:929-944: one [piece, start s, end s] per run of equal non-blank frames of align[:n_frames]
    (60 ms LFR frames, centred: -30 ms), the end clipped to the last frame as the reference's float32 tensor."""
    from itertools import groupby
    out, start, tid = [], 0, 0
    cap = np.float32(ts_max * 60 - 30) / np.float32(1000)    # (encoder_out_lens[i] - 4) * 60 - 30) / 1000, f32
    for tok, frames in groupby(align[:n_frames].tolist()):
        end = start + len(list(frames))
        if tok != 0:
            left = max((start * 60 - 30) / 1000, 0)
            right = (end * 60 - 30) / 1000
            if cap < np.float32(right):
                right = cap
            out.append([pieces[tid], left, right])
            tid += 1
        start = end
    return out


def timestamp_post(ts: list) -> list:
    """SenseVoiceSmall.post (model.py:949-965): word-level [start ms, end ms] from piece-level timestamps."""
    res = []
    for i, (word, start, end) in enumerate(ts):
        if word == "\u2581":
            continue
        if i == 0 or word.startswith("\u2581") or len(word) == 1 or not word[1].isalpha():
            res.append([int(start * 1000), int(end * 1000)])
        else:
            res[-1][1] = int(end * 1000)
    return res
