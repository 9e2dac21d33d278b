"""Fast-mode (bf16) rounding-point emulation on the CPU (diagnostic tool, not product code).

Runs the oracle's Paraformer restatement (oracle/paraformer_ref.py, torch-CPU fp32) with the FAST path's bf16
rounding points switched on one at a time, and scores each variant against a reference headline golden
(tests/golden/para_large_b24.npz / _b64.npz: the reference's per-position top-k log-probs) with the same statistics
the GPU parity test uses (tests/fast_parity.py): flip fraction on equal-count utterances, mean / max regret.

Rounding points (names used on the command line):
  G     every GEMM operand (activation rows and weights) in bf16, f32 accumulate  ("ideal bf16");
        GE / GP / GD / GO the same for the encoder / predictor conv / decoder (incl. memory K|V) / vocabulary only
  QKV   the q | k | v projection outputs stored as bf16 (attention + FSMN operands), decoder q too
  KV    the decoder's memory K | V projection output stored as bf16
  P     the attention's unnormalised probabilities exp(s - max) rounded to bf16 before P.V (normaliser in f32)
  F     the encoder FSMN memory output stored as bf16 (it is added to the f32 residual)
  DH    the decoder FFN's 2048-wide hidden rounded to bf16 BEFORE its LayerNorm (LN folded through W2:
        y = rstd (W2g h - mu c1) + c2 with W2g = bf16(W2 diag(gamma)))
  DF    the decoder FSMN's input (LN2 output) and output stored as bf16
  WONLY / AONLY  with a G* scope: round only the weights / only the activation rows
  A16   EXACT-mode x4 candidate: every GEMM activation as two bf16 planes (~2^-16), weights f32 (attention f32)
  XW:<s>  keep the weights of scope s exact (s = enc0 encq (encqq / encqk / encqv: its q / k / v rows) enco enc1w enc2w pred dec out; a split-bf16 weight)

    python tools/fast_emul.py b24 G G,QKV G,QKV,P ...
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from funasr_amd.config import paraformer_large  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from oracle import paraformer_ref as R  # noqa: E402
from tests.fast_parity import paraformer_stats  # noqa: E402
from tests.golden.inputs import fbank_input  # noqa: E402

ALL = ("G", "GE", "GP", "GD", "GO", "QKV", "KV", "P", "F", "DH", "DF")
SCOPE = {"G": ("enc", "pred", "dec", "out"), "GE": ("enc",), "GP": ("pred",), "GD": ("dec",), "GO": ("out",),
         "GE0": ("enc0",), "GE1": ("enc1",), "GEQ": ("encq",), "GEO": ("enco",), "GE1W": ("enc1w",), "GE2W": ("enc2w",)}
ALL = ALL + ("GE0", "GE1", "GEQ", "GEO", "GE1W", "GE2W", "WONLY", "AONLY", "A16")


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def bf2(x):
    """x0 + x1 (two bf16 planes, ~16 significant bits): the A operand of an EXACT-mode x4 GEMM"""
    x0 = bf(x)
    return x0 + bf(x - x0)


class Emu:
    def __init__(self, w, cfg, knobs):
        self.xw = {kk[3:] for kk in knobs if kk.startswith("XW:")}   # weights kept exact in these scopes
        knobs = [kk for kk in knobs if not kk.startswith("XW:")]
        self.w, self.cfg, self.k = w, cfg, set(knobs)
        self.g = {s for kk in self.k if kk in SCOPE for s in SCOPE[kk]}
        self.wb = {}

    def _wscope(self, key):
        """fine scope of a weight for XW: enc0 (enc0q / enc0o / enc0f: its QKV / out-proj / FFN) / encq / enco /
        enc1w / enc2w / pred / dec / out"""
        if key.startswith("encoder."):
            if key.startswith("encoder.encoders0."):
                for tag, sub in (("enc0q", "linear_q_k_v"), ("enc0o", "linear_out"), ("enc0f", "feed_forward")):
                    if sub in key and tag in self.xw:
                        return tag
                return "enc0"
            for tag, sub in (("encq", "linear_q_k_v"), ("enco", "linear_out"), ("enc1w", "w_1"), ("enc2w", "w_2")):
                if sub in key:
                    return tag
        return self._scope(key)

    def _scope(self, key):
        if key.startswith("encoder."):
            if "enc" in self.g:
                return "enc"
            if key.startswith("encoder.encoders0."):
                return "enc0"
            if "enc1" in self.g:
                return "enc1"
            for tag, sub in (("encq", "linear_q_k_v"), ("enco", "linear_out"), ("enc1w", "w_1"), ("enc2w", "w_2")):
                if sub in key:
                    return tag
            return "enc"
        if key.startswith("predictor."):
            return "pred"
        return "out" if key.startswith("decoder.output_layer") else "dec"

    def W(self, key):
        if self._scope(key) not in self.g or "AONLY" in self.k or self._wscope(key) in self.xw:
            return self.w[key]
        if key not in self.wb:
            wq = bf(self.w[key])
            if "linear_q_k_v" in key and key.startswith("encoder.encoders."):
                D = wq.shape[0] // 3
                layer = int(key.split(".")[2])
                lim = [int(x[6:]) for x in self.xw if x.startswith("encqv<")]   # encqv<N: layers 1..N-1 only
                for i, part in enumerate(("encqq", "encqk", "encqv")):
                    if part in self.xw or (part == "encqv" and lim and layer + 1 < lim[0]):
                        wq[i * D:(i + 1) * D] = self.w[key][i * D:(i + 1) * D]
            self.wb[key] = wq
        return self.wb[key]

    def lin(self, x, wkey, bkey=None):
        if "A16" in self.k:   # EXACT x4: activations as two bf16 planes, f32 weights
            return F.linear(bf2(x), self.w[wkey], self.w[bkey] if bkey else None)
        a = bf(x) if self._scope(wkey) in self.g and "WONLY" not in self.k else x
        return F.linear(a, self.W(wkey), self.w[bkey] if bkey else None)

    def attend(self, q, k, v, key_valid, heads, round_p):
        B, Tq, D = q.shape
        Tk = k.shape[1]
        dk = D // heads
        qh = q.reshape(B, Tq, heads, dk).transpose(1, 2) * dk ** (-0.5)
        kh = k.reshape(B, Tk, heads, dk).transpose(1, 2)
        vh = v.reshape(B, Tk, heads, dk).transpose(1, 2)
        s = torch.matmul(qh, kh.transpose(-2, -1))
        pad = (key_valid == 0)[:, None, None, :]
        s = s.masked_fill(pad, -float("inf"))
        if round_p:
            m = s.amax(-1, keepdim=True)
            p = torch.exp(s - m).masked_fill(pad, 0.0)
            l = p.sum(-1, keepdim=True)
            o = torch.matmul(bf(p), vh) / l
        else:
            o = torch.matmul(torch.softmax(s, -1).masked_fill(pad, 0.0), vh)
        return o.transpose(1, 2).reshape(B, Tq, D)

    def enc_layer(self, x, m, p):
        cfg, w = self.cfg, self.w
        din = x.shape[-1]
        h = R.layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps)
        a = f"{p}.self_attn"
        D = w[f"{a}.linear_out.weight"].shape[0]
        qkv = self.lin(h, f"{a}.linear_q_k_v.weight", f"{a}.linear_q_k_v.bias")
        if "QKV" in self.k:
            qkv = bf(qkv)
        q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
        mem = R.fsmn(v, m, w[f"{a}.fsmn_block.weight"], cfg.enc_sanm_shift)
        if "F" in self.k:
            mem = bf(mem)
        att = self.attend(q, k, v, m, cfg.heads, "P" in self.k)
        y = self.lin(att, f"{a}.linear_out.weight", f"{a}.linear_out.bias") + mem
        x = x + y if din == cfg.d_model else y
        h = R.layer_norm(x, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
        h = torch.relu(self.lin(h, f"{p}.feed_forward.w_1.weight", f"{p}.feed_forward.w_1.bias"))
        return x + self.lin(h, f"{p}.feed_forward.w_2.weight", f"{p}.feed_forward.w_2.bias")

    def encoder(self, feats, lens):
        cfg, w = self.cfg, self.w
        B, T, I = feats.shape
        m = R.pad_mask(lens, T)
        x = feats * cfg.d_model ** 0.5 + R.pos_encoding(T, I)[None]
        x = self.enc_layer(x, m, "encoder.encoders0.0")
        for i in range(cfg.enc_blocks - 1):
            x = self.enc_layer(x, m, f"encoder.encoders.{i}")
        x = R.layer_norm(x, w["encoder.after_norm.weight"], w["encoder.after_norm.bias"], cfg.ln_eps)
        return x, m.sum(1).to(torch.int64)

    def alphas(self, enc, lens):
        cfg, w = self.cfg, self.w
        m = R.pad_mask(lens, enc.shape[1])
        e = bf2(enc) if "A16" in self.k else bf(enc) if "pred" in self.g else enc
        q = F.pad(e.transpose(1, 2), (cfg.cif_l_order, cfg.cif_r_order))
        wc = (bf(w["predictor.cif_conv1d.weight"]) if "pred" in self.g and "pred" not in self.xw
              else w["predictor.cif_conv1d.weight"])
        h = torch.relu(F.conv1d(q, wc, w["predictor.cif_conv1d.bias"])).transpose(1, 2)
        a = torch.sigmoid(F.linear(h, w["predictor.cif_output.weight"], w["predictor.cif_output.bias"]))
        a = torch.relu(a * cfg.smooth_factor - cfg.noise_threshold)
        return a.squeeze(-1) * m

    def dec_ffn(self, x, p):
        cfg, w = self.cfg, self.w
        h = torch.relu(self.lin(x, f"{p}.w_1.weight", f"{p}.w_1.bias"))
        g, b = w[f"{p}.norm.weight"], w[f"{p}.norm.bias"]
        if "DH" in self.k:
            hb = bf(h)
            mu = hb.mean(-1, keepdim=True)
            var = ((hb - mu) ** 2).mean(-1, keepdim=True)
            rstd = torch.rsqrt(var + cfg.ln_eps)
            W2 = w[f"{p}.w_2.weight"]
            W2g = bf(W2 * g[None, :])
            c1 = W2g.sum(1)
            c2 = W2 @ b
            return rstd * (F.linear(hb, W2g) - mu * c1) + c2
        h = R.layer_norm(h, g, b, cfg.ln_eps)
        return self.lin(h, f"{p}.w_2.weight")

    def decoder(self, enc, enc_lens, embeds, ys_lens):
        cfg, w = self.cfg, self.w
        B, L, D = embeds.shape
        tm = R.pad_mask(ys_lens, L)
        mm = R.pad_mask(enc_lens, enc.shape[1])
        x = embeds
        for i in range(cfg.dec_blocks):
            p = f"decoder.decoders.{i}"
            r = x
            t = self.dec_ffn(R.layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                             f"{p}.feed_forward")
            t = R.layer_norm(t, w[f"{p}.norm2.weight"], w[f"{p}.norm2.bias"], cfg.ln_eps)
            if "DF" in self.k:
                t = bf(t)
            f = R.fsmn(t, tm, w[f"{p}.self_attn.fsmn_block.weight"], cfg.dec_sanm_shift)
            if "DF" in self.k:
                f = bf(f)
            x = r + f
            h = R.layer_norm(x, w[f"{p}.norm3.weight"], w[f"{p}.norm3.bias"], cfg.ln_eps)
            q = self.lin(h, f"{p}.src_attn.linear_q.weight", f"{p}.src_attn.linear_q.bias")
            kv = self.lin(enc, f"{p}.src_attn.linear_k_v.weight", f"{p}.src_attn.linear_k_v.bias")
            if "QKV" in self.k:
                q = bf(q)
            if "KV" in self.k:
                kv = bf(kv)
            a = self.attend(q, kv[..., :D], kv[..., D:], mm, cfg.heads, "P" in self.k)
            x = x + self.lin(a, f"{p}.src_attn.linear_out.weight", f"{p}.src_attn.linear_out.bias")
        p = "decoder.decoders3.0"
        x = self.dec_ffn(R.layer_norm(x, w[f"{p}.norm1.weight"], w[f"{p}.norm1.bias"], cfg.ln_eps),
                         f"{p}.feed_forward")
        hidden = R.layer_norm(x, w["decoder.after_norm.weight"], w["decoder.after_norm.bias"], cfg.ln_eps)
        return self.lin(hidden, "decoder.output_layer.weight", "decoder.output_layer.bias")

    @torch.no_grad()
    def run(self, feats, lens):
        cfg = self.cfg
        enc, olens = self.encoder(feats, lens)
        alphas = self.alphas(enc, olens)
        h, a, token_num = R.tail_process(enc, alphas, olens, cfg.tail_threshold)
        embeds, _, _ = R.cif(h, a, cfg.cif_threshold)
        embeds = embeds[:, : int(torch.max(token_num).to(torch.int32))]
        ntok = token_num.round().long()
        logits = self.decoder(enc, olens, embeds, ntok)
        return enc, ntok, logits.argmax(-1)


def score(golden, ntok, ids, enc=None):
    g = np.load(golden)
    s = paraformer_stats(ids.numpy().astype(np.int32), ntok.numpy(), g, margin=0.5)
    off = np.concatenate([[0], np.cumsum(g["ntok"])])
    flips, tot = 0, 0
    for b in range(len(g["ntok"])):
        if int(ntok[b]) != int(g["ntok"][b]):
            continue
        n = int(ntok[b])
        flips += int((ids[b, :n].numpy() != g["argmax"][off[b]:off[b] + n]).sum())
        tot += n
    s["flip_frac_equal_counts"] = flips / max(1, tot)
    if enc is not None:
        lens = g["lens"]
        rows = np.stack([enc[b, [0, int(lens[b]) // 2, int(lens[b]) - 1]].numpy() for b in range(len(lens))])
        s["enc_rows_rel"] = float(np.linalg.norm(rows - g["enc_rows"]) / np.linalg.norm(g["enc_rows"]))
    return s


def main():
    name = sys.argv[1]
    variants = [v.split(",") if v not in ("-", "none") else [] for v in sys.argv[2:]]
    torch.set_num_threads(int(os.environ.get("EMUL_THREADS", "8")))
    gpath = f"{ROOT}/tests/golden/para_large_{name}.npz"
    g = np.load(gpath)
    cfg = paraformer_large()
    w = R.as_torch_weights(make_weights(cfg, seed=0))
    feats, lens = fbank_input(seed=int(g["seed"]), B=int(g["B"]), T=int(g["T"]), lens=g["lens"])
    x, ln = torch.from_numpy(feats), torch.from_numpy(lens.astype(np.int64))
    out_json = os.environ.get("EMUL_JSON")
    res, toks = {}, {}
    for knobs in variants:
        for kk in knobs:
            assert kk in ALL or kk.startswith("XW:"), kk
        t0 = time.time()
        enc, ntok, ids = Emu(w, cfg, knobs).run(x, ln)
        s = score(gpath, ntok, ids, enc)
        res["+".join(knobs) or "f32"] = s
        toks[("+".join(knobs) or "f32") + "/ids"] = ids.numpy().astype(np.int16)
        toks[("+".join(knobs) or "f32") + "/ntok"] = ntok.numpy().astype(np.int16)
        print(f"{'+'.join(knobs) or 'f32':22s} flips {s['flip_frac_equal_counts']:.4f} "
              f"mean_regret {s['mean_regret']:.4f} max_regret {s['max_regret']:.3f} "
              f"outside_top5 {s['outside_topk']} equal_counts {s['equal_counts']:.3f} "
              f"enc_rel {s['enc_rows_rel']:.2e} ({time.time() - t0:.0f} s)", flush=True)
    if out_json:   # merge into a JSON file: {golden: {variant: stats}}
        import json
        allr = json.load(open(out_json)) if os.path.exists(out_json) else {}
        allr.setdefault(f"para_large_{name}", {}).update(res)
        with open(out_json, "w") as f:
            json.dump(allr, f, indent=1)
        # the emulated decisions themselves, so later statistics can be recomputed without re-running the emulation
        tpath = os.path.join(os.path.dirname(out_json), f"fast_emul_tokens_{name}.npz")
        old = dict(np.load(tpath)) if os.path.exists(tpath) else {}
        np.savez_compressed(tpath, **(old | toks))


if __name__ == "__main__":
    main()
