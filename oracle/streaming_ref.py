"""ORACLE — CPU restatement of the reference streaming Paraformer chunk path (TEST INFRASTRUCTURE).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module, and only as the checker. The product path (`funasr_amd.*`) never imports it.

Pinning: tests/test_oracle_golden.py checks it against tests/golden/stream_*.npz, produced by the
real reference `ParaformerStreaming.generate_chunk` / `inference` and `WavFrontendOnline`
(tests/golden/make_golden.py, `stream` part).

One stream (the reference is batch 1, paraformer_streaming/model.py:598), fp32 ATen on CPU:

  StreamState.__init__   paraformer_streaming/model.py:435-466 (init_cache)
  encoder_chunk          scama/encoder.py:448-499 (_add_overlap_chunk, forward_chunk),
                         embedding.py:416-444 (StreamSinusoidalPositionEncoder),
                         scama/encoder.py:150-186 + sanm/attention.py:313-339 (layer / attention with
                         the encoder_chunk_look_back K/V cache)
  cif_chunk              paraformer/cif_predictor.py:255-344 (CifPredictorV2.forward_chunk)
  decoder_chunk          paraformer/decoder.py:181-221, 461-528; sanm/attention.py:499-547 (FSMN cache),
                         719-740 (cross attention with the decoder_chunk_look_back K/V cache)
  chunk_step             paraformer_streaming/model.py:468-554 (generate_chunk, greedy path)
  FrontendOnline         frontends/wav_frontend.py:211-478 (WavFrontendOnline.forward, apply_lfr,
                         init_cache); fbank frames from oracle/fbank_ref.py
  stream_infer           paraformer_streaming/model.py:556-642 (inference: 600 ms sample chunks,
                         tail chunk, prev_samples)
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import fbank_ref
from .paraformer_ref import _attend, as_torch_weights, decoder_ffn, layer_norm

Tensor = torch.Tensor


class StreamState:
    """The reference cache dict of one stream (init_cache), as plain fields."""

    def __init__(self, cfg, chunk_size=(0, 10, 5), enc_look_back=0, dec_look_back=0):
        self.chunk_size = list(chunk_size)
        self.elb, self.dlb = int(enc_look_back), int(dec_look_back)
        self.start_idx = 0
        self.feats = torch.zeros((chunk_size[0] + chunk_size[2], cfg.input_size))
        self.enc_kv: List[Optional[tuple]] = [None] * cfg.enc_blocks
        self.cif_hidden = torch.zeros((cfg.d_model,))
        self.cif_alpha = torch.zeros(())
        self.dec_fsmn: List[Optional[Tensor]] = [None] * cfg.dec_blocks
        self.dec_kv: List[Optional[tuple]] = [None] * cfg.dec_blocks
        self.tail_chunk = False


def stream_pe(start: int, T: int, depth: int) -> Tensor:
    """StreamSinusoidalPositionEncoder rows start+1 .. start+T (embedding.py:422-444)."""
    pos = torch.arange(1, T + start + 1, dtype=torch.float32)
    inc = torch.log(torch.tensor([10000], dtype=torch.float32)) / (depth / 2 - 1)
    inv = torch.exp(torch.arange(depth / 2).type(torch.float32) * (-inc))
    st = pos[:, None] * inv[None, :]
    return torch.cat([torch.sin(st), torch.cos(st)], dim=1)[start:start + T]


def _enc_layer_chunk(x: Tensor, w, p: str, cfg, st: StreamState, li: int) -> Tensor:
    D = cfg.d_model
    cs = st.chunk_size
    din = x.shape[-1]
    h = layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps)
    a = f"{p}.self_attn"
    qkv = F.linear(h, w[f"{a}.linear_q_k_v.weight"], w[f"{a}.linear_q_k_v.bias"])
    q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
    kf, vf = k, v
    if st.elb > 0 or st.elb == -1:
        c = st.enc_kv[li]
        if c is not None:
            kf, vf = torch.cat((c[0], k)), torch.cat((c[1], v))
            ck, cv = torch.cat((c[0], k[: -cs[2]])), torch.cat((c[1], v[: -cs[2]]))
            if st.elb != -1:
                ck, cv = ck[-(st.elb * cs[1]):], cv[-(st.elb * cs[1]):]
            st.enc_kv[li] = (ck, cv)
        else:
            st.enc_kv[li] = (k[: -cs[2]], v[: -cs[2]])
    # FSMN memory over the window, zero padded, no mask (attention.py:207-223 with mask None)
    K = cfg.kernel_size
    left = (K - 1) // 2 + (cfg.enc_sanm_shift if cfg.enc_sanm_shift > 0 else 0)
    mem = F.conv1d(F.pad(v.t()[None], (left, K - 1 - left)), w[f"{a}.fsmn_block.weight"], groups=D)[0].t() + v
    att = _attend(q[None], kf[None], vf[None], torch.ones((1, kf.shape[0])), cfg.heads)[0]
    o = F.linear(att, w[f"{a}.linear_out.weight"], w[f"{a}.linear_out.bias"]) + mem
    x = x + o if din == D else o
    h = layer_norm(x, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
    h = F.linear(F.relu(F.linear(h, w[f"{p}.feed_forward.w_1.weight"], w[f"{p}.feed_forward.w_1.bias"])),
                 w[f"{p}.feed_forward.w_2.weight"], w[f"{p}.feed_forward.w_2.bias"])
    return x + h


def encoder_chunk(x_new: Optional[Tensor], st: StreamState, w, cfg) -> Tensor:
    """x_new [n, input_size] LFR+CMVN feats of the chunk, or None for the tail chunk. Returns the
    after_norm window [Tw, D] (Tw = cached overlap frames + n; 5 for the tail chunk)."""
    scale = cfg.d_model ** 0.5
    if st.tail_chunk or x_new is None:
        # forward_chunk scales its input in place (encoder.py:463) and the tail chunk's input IS
        # cache["feats"] (model.py:604-605), so the tail window is the cached overlap x sqrt(d)
        st.start_idx += st.feats.shape[0]
        x = st.feats * scale
    else:
        n = x_new.shape[0]
        xe = x_new * scale + stream_pe(st.start_idx, n, x_new.shape[1])
        st.start_idx += n
        x = torch.cat((st.feats, xe))
        st.feats = x[-(st.chunk_size[0] + st.chunk_size[2]):]
    x = _enc_layer_chunk(x, w, "encoder.encoders0.0", cfg, st, 0)
    for i in range(cfg.enc_blocks - 1):
        x = _enc_layer_chunk(x, w, f"encoder.encoders.{i}", cfg, st, i + 1)
    return layer_norm(x, w["encoder.after_norm.weight"], w["encoder.after_norm.bias"], cfg.ln_eps)


def cif_alphas_chunk(enc: Tensor, w, cfg) -> Tensor:
    q = F.pad(enc.t()[None], (cfg.cif_l_order, cfg.cif_r_order))
    h = torch.relu(F.conv1d(q, w["predictor.cif_conv1d.weight"], w["predictor.cif_conv1d.bias"]))[0].t()
    a = torch.sigmoid(F.linear(h, w["predictor.cif_output.weight"], w["predictor.cif_output.bias"]))
    return torch.relu(a * cfg.smooth_factor - cfg.noise_threshold).squeeze(-1)


def cif_chunk(enc: Tensor, st: StreamState, w, cfg, is_final: bool):
    """Returns (acoustic embeds [ntok, D], alphas of the window after chunk masking)."""
    alphas = cif_alphas_chunk(enc, w, cfg)
    cs = st.chunk_size
    alphas[: cs[0]] = 0.0
    if not is_final:
        alphas[sum(cs[:2]):] = 0.0
    a_win = alphas.clone()
    hidden = torch.cat((st.cif_hidden[None], enc))
    alphas = torch.cat((st.cif_alpha.reshape(1), alphas))
    if is_final:
        hidden = torch.cat((hidden, torch.zeros((1, enc.shape[1]))))
        alphas = torch.cat((alphas, torch.tensor([cfg.tail_threshold], dtype=torch.float32)))
    integrate = 0.0
    frames = torch.zeros((enc.shape[1],))
    out = []
    for t in range(alphas.shape[0]):
        alpha = alphas[t]
        if alpha + integrate < cfg.cif_threshold:
            integrate += alpha
            frames += alpha * hidden[t]
        else:
            frames += (cfg.cif_threshold - integrate) * hidden[t]
            out.append(frames)
            integrate += alpha
            integrate -= cfg.cif_threshold
            frames = integrate * hidden[t]
    st.cif_alpha = torch.as_tensor(integrate, dtype=torch.float32).reshape(())
    st.cif_hidden = frames / integrate if integrate > 0.0 else frames
    emb = torch.stack(out) if out else torch.zeros((0, enc.shape[1]))
    return emb, a_win


def _dec_fsmn_chunk(t: Tensor, wconv: Tensor, cache: Optional[Tensor], cfg):
    """MultiHeadedAttentionSANMDecoder.forward with mask None (attention.py:499-547); t [L, D]."""
    K = cfg.kernel_size
    left = (K - 1) // 2 + (cfg.dec_sanm_shift if cfg.dec_sanm_shift > 0 else 0)
    x = t.t()[None]
    L = x.shape[2]
    if cache is None:
        x = F.pad(x, (left, K - 1 - left))
    else:
        x = torch.cat((cache[:, :, 1:], x), dim=2)[:, :, -(K + L - 1):]
    cache = x
    y = F.conv1d(x, wconv, groups=wconv.shape[0])[0].t()
    inp = t if y.shape[0] == t.shape[0] else t[-1:]
    return y + inp, cache


def decoder_chunk(enc: Tensor, emb: Tensor, st: StreamState, w, cfg) -> Tensor:
    D = cfg.d_model
    x = emb
    for i in range(cfg.dec_blocks):
        p = f"decoder.decoders.{i}"
        r = x
        t = decoder_ffn(layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                        w, f"{p}.feed_forward", cfg)
        t = layer_norm(t, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
        y, st.dec_fsmn[i] = _dec_fsmn_chunk(t, w[f"{p}.self_attn.fsmn_block.weight"], st.dec_fsmn[i], cfg)
        x = r + y
        h = layer_norm(x, w[f"{p}.norm3.weight"], w[f"{p}.norm3.bias"], cfg.ln_eps)
        q = F.linear(h, w[f"{p}.src_attn.linear_q.weight"], w[f"{p}.src_attn.linear_q.bias"])
        kv = F.linear(enc, w[f"{p}.src_attn.linear_k_v.weight"], w[f"{p}.src_attn.linear_k_v.bias"])
        k, v = kv[:, :D], kv[:, D:]
        if st.dlb > 0:
            n = st.dlb * st.chunk_size[1]
            c = st.dec_kv[i]
            if c is not None:
                k, v = torch.cat((c[0], k)), torch.cat((c[1], v))
            st.dec_kv[i] = (k[-n:], v[-n:])
        a = _attend(q[None], k[None], v[None], torch.ones((1, k.shape[0])), cfg.heads)[0]
        x = x + F.linear(a, w[f"{p}.src_attn.linear_out.weight"], w[f"{p}.src_attn.linear_out.bias"])
    p = "decoder.decoders3.0"
    x = decoder_ffn(layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                    w, f"{p}.feed_forward", cfg)
    x = layer_norm(x, w["decoder.after_norm.weight"], w["decoder.after_norm.bias"], cfg.ln_eps)
    return F.linear(x, w["decoder.output_layer.weight"], w["decoder.output_layer.bias"])


@torch.no_grad()
def chunk_step(x_new, st: StreamState, w, cfg, is_final: bool, keep=False):
    """generate_chunk for one stream: token ids of this chunk (blank/sos/eos dropped)."""
    w = as_torch_weights(w)
    if x_new is not None and not isinstance(x_new, torch.Tensor):
        x_new = torch.from_numpy(np.ascontiguousarray(x_new, dtype=np.float32))
    enc = encoder_chunk(x_new, st, w, cfg)
    emb, a_win = cif_chunk(enc, st, w, cfg, is_final)
    res = dict(enc=enc, alphas=a_win, ntok=emb.shape[0], tokens=[])
    if emb.shape[0] < 1:
        return res
    logits = decoder_chunk(enc, emb, st, w, cfg)
    ids = logits.argmax(-1).tolist()
    res["argmax"] = ids
    res["tokens"] = [t for t in ids if t not in (cfg.eos, cfg.sos, cfg.blank_id)]
    if keep:
        res["logits"] = logits
    return res


# ------------------------------------------------------------------ online frontend
class FrontendOnline:
    """WavFrontendOnline.forward for one stream (dither 0): fbank frames over the carried samples,
    LFR with the splice-frame cache, CMVN. `cmvn` [2, 560] or None."""
    FL, FS = 400, 160

    def __init__(self, cmvn=None, lfr_m=7, lfr_n=6):
        self.cmvn, self.m, self.n = cmvn, lfr_m, lfr_n
        self.input_cache = np.zeros((0,), np.float32)
        self.reserve = np.zeros((0,), np.float32)   # reserve_waveforms
        self.splice: Optional[np.ndarray] = None      # lfr_splice_cache[0]

    def _lfr(self, x: np.ndarray, is_final: bool):
        """apply_lfr (wav_frontend.py:275-310): rows, splice cache, splice_idx."""
        m, n = self.m, self.n
        T = x.shape[0]
        T_lfr = int(np.ceil((T - (m - 1) // 2) / n))
        splice_idx = T_lfr
        last_idx = (T - m) // n + 1
        num_padding = m - (T - last_idx * n)
        rows = T_lfr
        inp = x
        if is_final:
            if num_padding > 0:
                num_padding = (2 * m - 2 * T + (T_lfr - 1 + last_idx) * n) / 2 * (T_lfr - last_idx)
                inp = np.concatenate([x] + [x[-1:]] * int(num_padding))
        elif num_padding > 0:
            rows = last_idx
            splice_idx = last_idx
        splice_idx = min(T - 1, splice_idx * n)
        # as_strided on inputs[:splice_idx] addresses the storage of `inputs`, so the last row may
        # read frames at or beyond splice_idx (still inside `inputs`)
        src = inp.reshape(-1)
        d = x.shape[1]
        out = np.stack([src[i * n * d: i * n * d + m * d] for i in range(rows)]) if rows > 0 else \
            np.zeros((0, m * d), np.float32)
        assert all(r.shape[0] == m * d for r in out), "as_strided would read past the input frames"
        return out.astype(np.float32), x[splice_idx:], splice_idx

    def __call__(self, wav: np.ndarray, is_final: bool) -> np.ndarray:
        x = np.concatenate([self.input_cache, np.asarray(wav, np.float32)])
        nfr = int((x.shape[0] - self.FL) / self.FS + 1)
        nfr = nfr if nfr >= 1 and x.shape[0] >= self.FL else 0
        self.input_cache = x[-(x.shape[0] - nfr * self.FS):]
        empty = np.zeros((0, 80 * self.m), np.float32)
        if nfr:
            used = x[: (nfr - 1) * self.FS + self.FL]
            fb = fbank_ref.fbank(used)
            waves = np.concatenate([self.reserve, used])
            if self.splice is None:
                self.splice = np.repeat(fb[:1], (self.m - 1) // 2, axis=0)
            if fb.shape[0] + self.splice.shape[0] >= self.m:
                feats = np.concatenate([self.splice, fb])
                from_w = int((waves.shape[0] - self.FL) / self.FS + 1)
                minus = (self.m - 1) // 2 if self.reserve.size == 0 else 0
                out, self.splice, sidx = self._lfr(feats, is_final)
                self.reserve = waves[(sidx - minus) * self.FS: from_w * self.FS]
            else:
                self.reserve = waves[: -(self.FL - self.FS)]
                self.splice = np.concatenate([self.splice, fb])
                return empty
        else:
            if not is_final:
                return empty
            out, _, _ = self._lfr(self.splice, is_final)
        if self.cmvn is not None and out.shape[0]:
            out = fbank_ref.apply_cmvn(out, self.cmvn)
        return out


CHUNK_SAMPLES_PER_FRAME = 960   # model.py:582: chunk_size[1] * 960 samples (60 ms per LFR frame)


@torch.no_grad()
def stream_infer(wav: np.ndarray, w, cfg, cmvn=None, chunk_size=(0, 10, 5), enc_look_back=0,
                 dec_look_back=0, is_final=True, state=None):
    """ParaformerStreaming.inference for one call (all samples of `wav`); returns (token ids per
    600 ms chunk, state). state = (StreamState, FrontendOnline, prev_samples) to continue a stream."""
    if state is None:
        state = (StreamState(cfg, chunk_size, enc_look_back, dec_look_back), FrontendOnline(cmvn), np.zeros(0, np.float32))
    st, fe, prev = state
    stride = int(chunk_size[1] * CHUNK_SAMPLES_PER_FRAME)
    audio = np.concatenate([prev, np.asarray(wav, np.float32)])
    n = int(len(audio) // stride + int(is_final))
    m = int(len(audio) % stride * (1 - int(is_final)))
    out = []
    for i in range(n):
        fin = is_final and i == n - 1
        seg = audio[i * stride:(i + 1) * stride]
        if fin and len(seg) < 960:
            st.tail_chunk = True
            r = chunk_step(None, st, w, cfg, fin)
        else:
            feats = fe(seg, fin)
            if feats.shape[0] == 0:
                # generate_chunk on an empty fbank: encoder over the overlap cache only happens with
                # tail_chunk; the reference would fail here, so such chunks never occur in practice
                out.append([])
                continue
            r = chunk_step(feats, st, w, cfg, fin)
        out.append(r["tokens"])
    prev = audio[:-m] if m else audio[len(audio):]
    if is_final:
        state = None
    else:
        state = (st, fe, prev)
    return out, state
