"""Seeded synthetic inputs shared by the golden generator, the tests and bench.py.

Fbank-input convention: post-CMVN LFR features ~ N(0,1) fp32 [B,T,560],
drawn from numpy PCG64(seed); padded frames (t >= len) are zero.
"""
from __future__ import annotations

import numpy as np


def fbank_input(seed: int, B: int, T: int, lens=None, dim: int = 560):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, T, dim), dtype=np.float32)
    lens = np.full((B,), T, dtype=np.int32) if lens is None else np.asarray(lens, dtype=np.int32)
    for b in range(B):
        x[b, int(lens[b]):] = 0.0
    return x, lens


def waveform(seed: int, n: int, fs: int = 16000):
    """Seeded 16 kHz test signal in [-1, 1): three tones + N(0, 0.05) noise, quantised to s16/32768."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    x = 0.3 * np.sin(2 * np.pi * 220.0 * t) + 0.2 * np.sin(2 * np.pi * 1375.0 * t + 0.3) \
        + 0.1 * np.sin(2 * np.pi * 4100.0 * t + 1.1) + rng.normal(0.0, 0.05, n)
    q = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return (q.astype(np.float32) / 32768.0)


def token_list(vocab: int):
    """Synthetic CharTokenizer vocabulary: <blank>,<s>,</s>, CJK chars, <unk>."""
    return ["<blank>", "<s>", "</s>"] + [chr(0x4E00 + i) for i in range(vocab - 4)] + ["<unk>"]


def vad_waveform(seed: int, seconds: float, gaps):
    """Seeded 16 kHz signal for the VAD goldens: the tone+noise test signal with quiet gaps (N(0, 0.002),
    s16-quantised) at `gaps` [(beg_s, end_s)]."""
    x = waveform(seed=seed, n=int(seconds * 16000)).copy()
    rng = np.random.default_rng(seed + 100)
    for b, e in gaps:
        i0, i1 = int(b * 16000), int(e * 16000)
        x[i0:i1] = np.round(rng.normal(0.0, 0.002, i1 - i0) * 32768.0).clip(-32768, 32767) / 32768.0
    return x.astype(np.float32)
