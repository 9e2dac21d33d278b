"""ORACLE — CPU restatement of the reference Paraformer inference path (TEST INFRASTRUCTURE).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import this module, and only as the checker / the timed CPU baseline. The
product path (`funasr_amd.*`) never imports it and has no CPU fallback.

Pinning: tests/test_oracle_golden.py checks this restatement against golden
vectors produced by the real reference modules (tests/golden/make_golden.py).

Arithmetic is ATen fp32 on CPU — the same library the reference calls — written
as plain functions over a state_dict, one function per reference stage:

  pos_encoding        funasr/models/transformer/embedding.py:389-413
  layer_norm          funasr/models/transformer/layer_norm.py:13-39 (eps 1e-12)
  fsmn                funasr/models/sanm/attention.py:207-223 (encoder),
                      funasr/models/sanm/attention.py:499-547 (decoder, tgt mask)
  sanm_self_attention funasr/models/sanm/attention.py:225-311
  encoder             funasr/models/sanm/encoder.py:72-148, 361-430
  predictor / cif     funasr/models/paraformer/cif_predictor.py:202-253, 346-370, 668-735
  decoder             funasr/models/paraformer/decoder.py:78-121, 359-411;
                      cross attention funasr/models/sanm/attention.py:631-717;
                      FFN funasr/models/sanm/positionwise_feed_forward.py:12-33
  greedy              funasr/models/paraformer/model.py:513-565
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def _t(w, key) -> Tensor:
    v = w[key]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))


def as_torch_weights(w: Dict[str, np.ndarray]) -> Dict[str, Tensor]:
    return {k: (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v)))
            for k, v in w.items()}


def pad_mask(lens: Tensor, T: int) -> Tensor:
    """1.0 on valid frames, 0.0 on padding: [B, T] (make_pad_mask negated, nets_utils.py:104)."""
    return (torch.arange(T)[None, :] < lens[:, None]).to(torch.float32)


def pos_encoding(T: int, depth: int) -> Tensor:
    """Sinusoidal PE, positions 1..T, [sin | cos] halves (embedding.py:389-413), fp32."""
    pos = torch.arange(1, T + 1, dtype=torch.float32)
    inc = torch.log(torch.tensor([10000.0], dtype=torch.float32)) / (depth / 2 - 1)
    inv = torch.exp(torch.arange(depth / 2).to(torch.float32) * (-inc))
    st = pos[:, None] * inv[None, :]
    return torch.cat([torch.sin(st), torch.cos(st)], dim=1)


def layer_norm(x: Tensor, g: Tensor, b: Tensor, eps: float) -> Tensor:
    return F.layer_norm(x, (x.shape[-1],), g, b, eps)


def fsmn(v: Tensor, m: Tensor, wconv: Tensor, shift: int) -> Tensor:
    """mask * (depthwise_conv(mask*v) + mask*v); v [B,T,D], m [B,T], wconv [D,1,K]."""
    K = wconv.shape[-1]
    left = (K - 1) // 2 + (shift if shift > 0 else 0)
    right = K - 1 - left
    mm = m[:, :, None]
    vin = v * mm
    x = F.pad(vin.transpose(1, 2), (left, right))
    x = F.conv1d(x, wconv, groups=wconv.shape[0]).transpose(1, 2)
    return (x + vin) * mm


def _attend(q: Tensor, k: Tensor, v: Tensor, key_valid: Tensor, heads: int) -> Tensor:
    """softmax((q*dk^-0.5) k^T, -inf on padded keys) v, padded-key probs zeroed; returns [B,Tq,D]."""
    B, Tq, D = q.shape
    Tk = k.shape[1]
    dk = D // heads
    qh = q.reshape(B, Tq, heads, dk).transpose(1, 2) * dk ** (-0.5)
    kh = k.reshape(B, Tk, heads, dk).transpose(1, 2)
    vh = v.reshape(B, Tk, heads, dk).transpose(1, 2)
    s = torch.matmul(qh, kh.transpose(-2, -1))
    pad = (key_valid == 0)[:, None, None, :]
    p = torch.softmax(s.masked_fill(pad, -float("inf")), dim=-1).masked_fill(pad, 0.0)
    o = torch.matmul(p, vh)
    return o.transpose(1, 2).reshape(B, Tq, D)


def sanm_self_attention(x: Tensor, m: Tensor, w: Dict[str, Tensor], p: str, heads: int, shift: int) -> Tensor:
    D = w[f"{p}.linear_out.weight"].shape[0]
    qkv = F.linear(x, w[f"{p}.linear_q_k_v.weight"], w[f"{p}.linear_q_k_v.bias"])
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    mem = fsmn(v, m, w[f"{p}.fsmn_block.weight"], shift)
    att = _attend(q, k, v, m, heads)
    return F.linear(att, w[f"{p}.linear_out.weight"], w[f"{p}.linear_out.bias"]) + mem


def encoder_layer(x: Tensor, m: Tensor, w: Dict[str, Tensor], p: str, cfg) -> Tensor:
    din = x.shape[-1]
    h = layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps)
    a = sanm_self_attention(h, m, w, f"{p}.self_attn", cfg.heads, cfg.enc_sanm_shift)
    x = x + a if din == cfg.d_model else a
    h = layer_norm(x, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
    h = F.linear(F.relu(F.linear(h, w[f"{p}.feed_forward.w_1.weight"], w[f"{p}.feed_forward.w_1.bias"])),
                 w[f"{p}.feed_forward.w_2.weight"], w[f"{p}.feed_forward.w_2.bias"])
    return x + h


def encoder(feats: Tensor, lens: Tensor, w: Dict[str, Tensor], cfg, return_layers=False):
    B, T, I = feats.shape
    m = pad_mask(lens, T)
    x = feats * cfg.d_model ** 0.5
    x = x + pos_encoding(T, I)[None]
    layers = []
    x = encoder_layer(x, m, w, "encoder.encoders0.0", cfg)
    layers.append(x)
    for i in range(cfg.enc_blocks - 1):
        x = encoder_layer(x, m, w, f"encoder.encoders.{i}", cfg)
        layers.append(x)
    x = layer_norm(x, w["encoder.after_norm.weight"], w["encoder.after_norm.bias"], cfg.ln_eps)
    olens = m.sum(1).to(torch.int64)
    if return_layers:
        return x, olens, layers
    return x, olens


def cif_alphas(enc: Tensor, lens: Tensor, w: Dict[str, Tensor], cfg) -> Tensor:
    """conv1d(k=l+r+1) + ReLU + Linear(512->1) + sigmoid, then relu(a*smooth - noise) * mask: [B,T]."""
    m = pad_mask(lens, enc.shape[1])
    q = F.pad(enc.transpose(1, 2), (cfg.cif_l_order, cfg.cif_r_order))
    h = torch.relu(F.conv1d(q, w["predictor.cif_conv1d.weight"], w["predictor.cif_conv1d.bias"])).transpose(1, 2)
    a = torch.sigmoid(F.linear(h, w["predictor.cif_output.weight"], w["predictor.cif_output.bias"]))
    a = torch.relu(a * cfg.smooth_factor - cfg.noise_threshold)
    return (a.squeeze(-1) * m)


def tail_process(hidden: Tensor, alphas: Tensor, lens: Tensor, tail: float):
    """Append tail_threshold at frame `len` and a zero hidden frame (cif_predictor.py:346-370)."""
    B, T, D = hidden.shape
    m = pad_mask(lens, T)
    z = torch.zeros((B, 1), dtype=torch.float32)
    tail_m = torch.cat([torch.ones_like(z), m], 1) - torch.cat([m, z], 1)
    a = torch.cat([alphas, z], 1) + tail_m * tail
    h = torch.cat([hidden, torch.zeros((B, 1, D), dtype=hidden.dtype)], 1)
    token_num = torch.floor(a.sum(-1))
    return h, a, token_num


def cif(hidden: Tensor, alphas: Tensor, threshold: float):
    """Continuous integrate-and-fire (cif_v1, cif_predictor.py:668-735).

    Fire at frame t iff floor(P_t) > floor(P_{t-1}), P = fp64 cumsum of alphas cast to fp32.
    Token k = PH[t_k] - PH[t_{k-1}] + r[t_{k-1}] h[t_{k-1}] - r[t_k] h[t_k], PH = cumsum(alpha*h),
    r = frac part of the fire value. Rows beyond the fire count are zero; padded to round(sum a).max().
    """
    B, T, D = hidden.shape
    P = torch.cumsum(alphas, dim=1, dtype=torch.float64).to(torch.float32)
    Pf = torch.floor(P)
    prevf = torch.roll(Pf, 1, dims=1)
    prevf[:, 0] = 0
    fire = (Pf - prevf) > 0
    fires = fire.to(torch.float32) + (P - Pf)
    PH = torch.cumsum(alphas[:, :, None] * hidden, dim=1)
    rem = fires - torch.floor(fires)
    L = int(torch.round(alphas.sum(-1)).int().max())
    n_fire = fire.sum(1)
    out = torch.zeros((B, max(L, 0), D), dtype=torch.float32)
    for b in range(B):
        idx = torch.nonzero(fire[b]).squeeze(-1)
        prev_ph = torch.zeros(D)
        prev_rh = torch.zeros(D)
        for k, t in enumerate(idx.tolist()):
            rh = rem[b, t] * hidden[b, t]
            out[b, k] = PH[b, t] - prev_ph + prev_rh - rh
            prev_ph, prev_rh = PH[b, t], rh
    return out, fires, n_fire


def predictor(enc: Tensor, lens: Tensor, w: Dict[str, Tensor], cfg):
    alphas = cif_alphas(enc, lens, w, cfg)
    h, a, token_num = tail_process(enc, alphas, lens, cfg.tail_threshold)
    embeds, peak, n_fire = cif(h, a, cfg.cif_threshold)
    Lmax = int(torch.max(token_num).to(torch.int32))
    return embeds[:, :Lmax], token_num, a, peak, n_fire


def decoder_ffn(x: Tensor, w: Dict[str, Tensor], p: str, cfg) -> Tensor:
    h = torch.relu(F.linear(x, w[f"{p}.w_1.weight"], w[f"{p}.w_1.bias"]))
    h = layer_norm(h, w[f"{p}.norm.weight"], w[f"{p}.norm.bias"], cfg.ln_eps)
    return F.linear(h, w[f"{p}.w_2.weight"])


def decoder(enc: Tensor, enc_lens: Tensor, embeds: Tensor, ys_lens: Tensor, w: Dict[str, Tensor], cfg,
            return_hidden=False) -> Tensor:
    B, L, D = embeds.shape
    tm = pad_mask(ys_lens, L)
    mm = pad_mask(enc_lens, enc.shape[1])
    x = embeds
    for i in range(cfg.dec_blocks):
        p = f"decoder.decoders.{i}"
        r = x
        t = decoder_ffn(layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                        w, f"{p}.feed_forward", cfg)
        t = layer_norm(t, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
        x = r + fsmn(t, tm, w[f"{p}.self_attn.fsmn_block.weight"], cfg.dec_sanm_shift)
        h = layer_norm(x, w[f"{p}.norm3.weight"], w[f"{p}.norm3.bias"], cfg.ln_eps)
        q = F.linear(h, w[f"{p}.src_attn.linear_q.weight"], w[f"{p}.src_attn.linear_q.bias"])
        kv = F.linear(enc, w[f"{p}.src_attn.linear_k_v.weight"], w[f"{p}.src_attn.linear_k_v.bias"])
        a = _attend(q, kv[..., :D], kv[..., D:], mm, cfg.heads)
        x = x + F.linear(a, w[f"{p}.src_attn.linear_out.weight"], w[f"{p}.src_attn.linear_out.bias"])
    p = "decoder.decoders3.0"
    x = decoder_ffn(layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                    w, f"{p}.feed_forward", cfg)
    hidden = layer_norm(x, w["decoder.after_norm.weight"], w["decoder.after_norm.bias"], cfg.ln_eps)
    logits = F.linear(hidden, w["decoder.output_layer.weight"], w["decoder.output_layer.bias"])
    if return_hidden:
        return logits, hidden
    return logits


def greedy(logp: Tensor, ntok: Tensor, cfg) -> List[List[int]]:
    """Per-utterance argmax over the first ntok rows, drop {blank, sos, eos} (model.py:527-565)."""
    out = []
    for i in range(logp.shape[0]):
        ids = logp[i, : int(ntok[i])].argmax(dim=-1).tolist()
        out.append([t for t in ids if t not in (cfg.eos, cfg.sos, cfg.blank_id)])
    return out


@torch.no_grad()
def paraformer_infer(feats, lens, w, cfg, keep_logits=False) -> dict:
    """Full fbank -> token-id path (Paraformer.inference with data_type='fbank')."""
    feats = feats if isinstance(feats, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(feats))
    lens = (lens if isinstance(lens, torch.Tensor) else torch.as_tensor(lens)).to(torch.int64).reshape(-1)
    w = as_torch_weights(w)
    enc, olens = encoder(feats.to(torch.float32), lens, w, cfg)
    embeds, token_num, alphas, peak, n_fire = predictor(enc, olens, w, cfg)
    ntok = token_num.round().long()
    res = dict(enc=enc, enc_lens=olens, alphas=alphas, cif_peak=peak, token_num=token_num,
               n_fire=n_fire, ntok=ntok, embeds=embeds)
    if int(ntok.max()) < 1:
        res["tokens"] = [[] for _ in range(feats.shape[0])]
        return res
    logits = decoder(enc, olens, embeds, ntok, w, cfg)
    logp = torch.log_softmax(logits, dim=-1)
    res["tokens"] = greedy(logp, ntok, cfg)
    res["argmax"] = logits.argmax(-1)
    if keep_logits:
        res["logits"] = logits
    return res
