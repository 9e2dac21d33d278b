"""ORACLE — numpy restatement of the WavFrontend math (TEST INFRASTRUCTURE ONLY).

  fbank      kaldi-native-fbank as vendored by the reference (feature-window.cc:25-55,121-247;
             feature-fbank.cc:73-118; mel-computations.cc:107-257; feature-functions.cc:28-47)
             with the options of runtime/onnxruntime/src/paraformer.cpp:21-31
  apply_lfr  funasr/frontends/wav_frontend.py:58-74
  apply_cmvn funasr/frontends/wav_frontend.py:41-55
Pinned against oracle/_ref/knf_fbank (the reference C++ compiled from its own sources) via
tests/golden/fbank_knf.npz, and against the reference apply_lfr/apply_cmvn via lfr_cmvn.npz.
"""
from __future__ import annotations

import numpy as np

FL, FS, NFFT, NMEL = 400, 160, 512, 80


def _mel(f):
    return np.float32(1127.0) * np.log(np.float32(1.0) + np.asarray(f, np.float32) / np.float32(700.0)).astype(np.float32)


def mel_banks() -> np.ndarray:
    """[80, 256] triangular weights computed in f32 like knf MelBanks."""
    w = np.zeros((NMEL, NFFT // 2), np.float32)
    lo, hi = _mel(20.0), _mel(8000.0)
    delta = (hi - lo) / np.float32(NMEL + 1)
    freqs = np.float32(16000.0 / NFFT) * np.arange(NFFT // 2, dtype=np.float32)
    m = _mel(freqs)
    for b in range(NMEL):
        left, center, right = lo + b * delta, lo + (b + 1) * delta, lo + (b + 2) * delta
        up = (m > left) & (m <= center)
        down = (m > center) & (m < right)
        w[b, up] = ((m[up] - left) / (center - left)).astype(np.float32)
        w[b, down] = ((right - m[down]) / (right - center)).astype(np.float32)
    return w


def hamming() -> np.ndarray:
    a = 2.0 * np.pi / (FL - 1)
    return (0.54 - 0.46 * np.cos(a * np.arange(FL))).astype(np.float32)


def fbank(wav: np.ndarray) -> np.ndarray:
    """wav: float samples in [-1, 1). Returns log-mel [N, 80] f32 (N = 1 + (S-400)//160)."""
    x = np.asarray(wav, np.float32) * np.float32(32768.0)
    n = 0 if len(x) < FL else 1 + (len(x) - FL) // FS
    if n == 0:
        return np.zeros((0, NMEL), np.float32)
    idx = np.arange(n)[:, None] * FS + np.arange(FL)[None, :]
    fr = x[idx].astype(np.float32)
    fr = fr - fr.mean(axis=1, keepdims=True, dtype=np.float64).astype(np.float32)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = (fr - np.float32(0.97) * prev) * hamming()[None, :]
    spec = np.fft.rfft(fr.astype(np.float64), n=NFFT, axis=1)[:, : NFFT // 2]
    re, im = spec.real.astype(np.float32), spec.imag.astype(np.float32)
    p = re * re + im * im
    e = p @ mel_banks().T
    return np.log(np.maximum(e, np.float32(1.1920928955078125e-07))).astype(np.float32)


def apply_lfr(x: np.ndarray, m: int = 7, n: int = 6) -> np.ndarray:
    """LFR row i = frames clamp(n*i + j - (m-1)//2, 0, N-1), j < m, concatenated."""
    N = x.shape[0]
    T = (N + n - 1) // n
    idx = np.clip(np.arange(T)[:, None] * n + np.arange(m)[None, :] - (m - 1) // 2, 0, N - 1)
    return x[idx].reshape(T, m * x.shape[1]).astype(np.float32)


def apply_cmvn(x: np.ndarray, cmvn: np.ndarray) -> np.ndarray:
    d = x.shape[1]
    return ((x + cmvn[0:1, :d]) * cmvn[1:2, :d]).astype(np.float32)


def frontend(wav: np.ndarray, cmvn: np.ndarray = None) -> np.ndarray:
    y = apply_lfr(fbank(wav))
    return apply_cmvn(y, cmvn) if cmvn is not None else y
