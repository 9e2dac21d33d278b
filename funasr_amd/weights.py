"""Deterministic synthetic Paraformer weights + state_dict key layout.

Pretrained checkpoints cannot be fetched offline, so every parity
run uses weights from this counter-seeded generator: each tensor is drawn from
its own PCG64 stream keyed by (seed, crc32(state_dict key)), so any subset of
tensors can be regenerated independently, on any host, bit-identically.

Distribution follows torch's default module init (what the survey's reference
timings used): Linear/Conv weights and biases ~ U(-1/sqrt(fan_in), +1/sqrt(fan_in)).
LayerNorm gamma/beta are perturbed off (1, 0) so the affine path is exercised.

Key names and shapes are exactly the reference `model.state_dict()` of
`funasr/models/paraformer/model.py:29`, so these dicts load
into the reference with `load_state_dict(strict=True)` and a real `model.pt`
state_dict can be fed to the HIP path unchanged.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterator, List, Tuple

import numpy as np

from .config import CTTransformerConfig, FsmnVADConfig, ParaformerConfig, SenseVoiceConfig

Shape = Tuple[int, ...]


def param_layout(cfg) -> List[Tuple[str, Shape, int]]:
    """(key, shape, fan_in) for every parameter, in state_dict order.

    Negative fan_in codes: -1 LayerNorm gamma, -2 LayerNorm beta, -3 embedding table.
    """
    if isinstance(cfg, SenseVoiceConfig):
        return sense_voice_layout(cfg)
    if isinstance(cfg, CTTransformerConfig):
        return ct_transformer_layout(cfg)
    if isinstance(cfg, FsmnVADConfig):
        return fsmn_vad_layout(cfg)
    D, F, K, I, V = cfg.d_model, cfg.ffn, cfg.kernel_size, cfg.input_size, cfg.vocab_size
    out: List[Tuple[str, Shape, int]] = []

    def lin(name, o, i, bias=True):
        out.append((f"{name}.weight", (o, i), i))
        if bias:
            out.append((f"{name}.bias", (o,), i))

    def ln(name, n):
        out.append((f"{name}.weight", (n,), -1))
        out.append((f"{name}.bias", (n,), -2))

    def enc_layer(p, din):
        lin(f"{p}.self_attn.linear_out", D, D)
        lin(f"{p}.self_attn.linear_q_k_v", 3 * D, din)
        out.append((f"{p}.self_attn.fsmn_block.weight", (D, 1, K), K))
        lin(f"{p}.feed_forward.w_1", F, D)
        lin(f"{p}.feed_forward.w_2", D, F)
        ln(f"{p}.norm1", din)
        ln(f"{p}.norm2", D)

    enc_layer("encoder.encoders0.0", I)
    for i in range(cfg.enc_blocks - 1):
        enc_layer(f"encoder.encoders.{i}", D)
    ln("encoder.after_norm", D)

    out.append(("decoder.embed.0.weight", (V, D), -3))
    ln("decoder.after_norm", D)
    lin("decoder.output_layer", V, D)
    for i in range(cfg.dec_blocks):
        p = f"decoder.decoders.{i}"
        out.append((f"{p}.self_attn.fsmn_block.weight", (D, 1, K), K))
        lin(f"{p}.src_attn.linear_q", D, D)
        lin(f"{p}.src_attn.linear_k_v", 2 * D, D)
        lin(f"{p}.src_attn.linear_out", D, D)
        lin(f"{p}.feed_forward.w_1", F, D)
        lin(f"{p}.feed_forward.w_2", D, F, bias=False)
        ln(f"{p}.feed_forward.norm", F)
        ln(f"{p}.norm1", D)
        ln(f"{p}.norm2", D)
        ln(f"{p}.norm3", D)
    p = "decoder.decoders3.0"
    lin(f"{p}.feed_forward.w_1", F, D)
    lin(f"{p}.feed_forward.w_2", D, F, bias=False)
    ln(f"{p}.feed_forward.norm", F)
    ln(f"{p}.norm1", D)

    kp = cfg.cif_l_order + cfg.cif_r_order + 1
    out.append(("predictor.cif_conv1d.weight", (D, D, kp), D * kp))
    out.append(("predictor.cif_conv1d.bias", (D,), D * kp))
    lin("predictor.cif_output", 1, D)
    if getattr(cfg, "ctc_weight", 0.0) > 0.0:   # ctc/ctc.py:33 (paraformer/model.py:95-100)
        lin("ctc.ctc_lo", V, D)
    return out


def _enc_layer(out, p: str, din: int, D: int, F: int, K: int):
    """EncoderLayerSANM parameters (sanm/encoder.py:72-148 == sense_voice/model.py:301-327)."""
    out += [(f"{p}.self_attn.linear_out.weight", (D, D), D), (f"{p}.self_attn.linear_out.bias", (D,), D),
            (f"{p}.self_attn.linear_q_k_v.weight", (3 * D, din), din),
            (f"{p}.self_attn.linear_q_k_v.bias", (3 * D,), din),
            (f"{p}.self_attn.fsmn_block.weight", (D, 1, K), K),
            (f"{p}.feed_forward.w_1.weight", (F, D), D), (f"{p}.feed_forward.w_1.bias", (F,), D),
            (f"{p}.feed_forward.w_2.weight", (D, F), F), (f"{p}.feed_forward.w_2.bias", (D,), F),
            (f"{p}.norm1.weight", (din,), -1), (f"{p}.norm1.bias", (din,), -2),
            (f"{p}.norm2.weight", (D,), -1), (f"{p}.norm2.bias", (D,), -2)]


def sense_voice_layout(cfg: SenseVoiceConfig) -> List[Tuple[str, Shape, int]]:
    """SenseVoiceSmall state_dict keys (sense_voice/model.py:445-663; ctc/ctc.py:33):
    encoder.{encoders0.0, encoders.*, tp_encoders.*}, after_norm, tp_norm, ctc.ctc_lo, embed."""
    D, F, K, I, V = cfg.d_model, cfg.ffn, cfg.kernel_size, cfg.input_size, cfg.vocab_size
    out: List[Tuple[str, Shape, int]] = []
    _enc_layer(out, "encoder.encoders0.0", I, D, F, K)
    for i in range(cfg.enc_blocks - 1):
        _enc_layer(out, f"encoder.encoders.{i}", D, D, F, K)
    for i in range(cfg.tp_blocks):
        _enc_layer(out, f"encoder.tp_encoders.{i}", D, D, F, K)
    out += [("encoder.after_norm.weight", (D,), -1), ("encoder.after_norm.bias", (D,), -2),
            ("encoder.tp_norm.weight", (D,), -1), ("encoder.tp_norm.bias", (D,), -2),
            ("ctc.ctc_lo.weight", (V, D), D), ("ctc.ctc_lo.bias", (V,), D),
            ("embed.weight", (cfg.n_embed, I), -3)]
    return out


def ct_transformer_layout(cfg: CTTransformerConfig) -> List[Tuple[str, Shape, int]]:
    """CTTransformer state_dict keys (ct_transformer/model.py:63-68): embed, encoder (SANMEncoder with
    input_layer "pe": encoders0.0, encoders.*, after_norm), decoder (Linear att_unit -> punc classes)."""
    D, F, K, I = cfg.d_model, cfg.ffn, cfg.kernel_size, cfg.input_size
    out: List[Tuple[str, Shape, int]] = [("embed.weight", (cfg.vocab_size, I), -3)]
    _enc_layer(out, "encoder.encoders0.0", I, D, F, K)
    for i in range(cfg.enc_blocks - 1):
        _enc_layer(out, f"encoder.encoders.{i}", D, D, F, K)
    out += [("encoder.after_norm.weight", (D,), -1), ("encoder.after_norm.bias", (D,), -2),
            ("decoder.weight", (cfg.n_punc, D), D), ("decoder.bias", (cfg.n_punc,), D)]
    return out


def fsmn_vad_layout(cfg: FsmnVADConfig) -> List[Tuple[str, Shape, int]]:
    """FsmnVADStreaming state_dict keys (fsmn_vad_streaming/encoder.py:200-241): the FSMN encoder only."""
    out: List[Tuple[str, Shape, int]] = []

    def aff(name, o, i, bias=True):
        out.append((f"{name}.linear.weight", (o, i), i))
        if bias:
            out.append((f"{name}.linear.bias", (o,), i))

    aff("encoder.in_linear1", cfg.input_affine_dim, cfg.input_dim)
    aff("encoder.in_linear2", cfg.linear_dim, cfg.input_affine_dim)
    for i in range(cfg.fsmn_layers):
        aff(f"encoder.fsmn.{i}.linear", cfg.proj_dim, cfg.linear_dim, bias=False)
        out.append((f"encoder.fsmn.{i}.fsmn_block.conv_left.weight", (cfg.proj_dim, 1, cfg.lorder, 1), cfg.lorder))
        aff(f"encoder.fsmn.{i}.affine", cfg.linear_dim, cfg.proj_dim)
    aff("encoder.out_linear1", cfg.output_affine_dim, cfg.linear_dim)
    aff("encoder.out_linear2", cfg.output_dim, cfg.output_affine_dim)
    return out


def _stream(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def gen_tensor(seed: int, key: str, shape: Shape, fan_in: int) -> np.ndarray:
    n = int(np.prod(shape))
    u = _stream(seed, key).random(n, dtype=np.float32) * np.float32(2.0) - np.float32(1.0)
    if fan_in > 0:
        a = u * np.float32(1.0 / np.sqrt(fan_in))
    elif fan_in == -1:          # LayerNorm gamma
        a = np.float32(1.0) + np.float32(0.1) * u
    elif fan_in == -2:          # LayerNorm beta
        a = np.float32(0.1) * u
    else:                       # embedding tables: U(-1, 1)
        a = u
    return a.astype(np.float32).reshape(shape)


def iter_weights(cfg, seed: int = 0) -> Iterator[Tuple[str, np.ndarray]]:
    for key, shape, fan_in in param_layout(cfg):
        yield key, gen_tensor(seed, key, shape, fan_in)


def make_weights(cfg, seed: int = 0) -> Dict[str, np.ndarray]:
    """Full synthetic state_dict as fp32 numpy arrays (220.08M params for Paraformer-large;
    SenseVoiceSmall layout when cfg is a SenseVoiceConfig)."""
    return dict(iter_weights(cfg, seed))


def num_params(cfg) -> int:
    return int(sum(int(np.prod(s)) for _, s, _ in param_layout(cfg)))


def vad_test_weights(cfg: FsmnVADConfig, seed: int = 0, sil_scale: float = -2000.0, sil_bias: float = 0.0):
    """Synthetic FSMN-VAD weights for segment tests: the silence-pdf row of out_linear2 scaled (and its bias
    shifted) so p(sil) follows the signal level across the speech/noise threshold; with plain random
    weights p(sil) ~ 1/248 for every frame and the detector sees one all-speech segment."""
    w = make_weights(cfg, seed)
    wk, bk = "encoder.out_linear2.linear.weight", "encoder.out_linear2.linear.bias"
    w[wk] = w[wk].copy()
    w[wk][0] *= np.float32(sil_scale)
    w[bk] = w[bk].copy()
    w[bk][0] += np.float32(sil_bias)
    return w
