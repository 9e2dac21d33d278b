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

import ctypes
import ctypes.util

import numpy as np

FL, FS, NFFT, NMEL = 400, 160, 512, 80

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]


def _mel(f) -> np.float32:
    """MelScale (mel-computations.h:72-74): 1127 * logf(1 + f / 700) in f32 with the C library's logf,
    evaluated at run time as knf does (numpy's own f32 log, or a compile-time-folded logf, differ by an
    ulp on some bins and move the triangle edges)."""
    return np.float32(1127.0) * np.float32(_libm.logf(float(np.float32(1.0) + np.float32(f) / np.float32(700.0))))


def mel_banks() -> np.ndarray:
    """[80, 256] triangular weights, knf MelBanks (mel-computations.cc:107-221) operation by operation."""
    w = np.zeros((NMEL, NFFT // 2), np.float32)
    lo, hi = _mel(20.0), _mel(8000.0)
    delta = np.float32((hi - lo) / np.float32(NMEL + 1))
    width = np.float32(16000.0) / np.float32(NFFT)
    m = [_mel(np.float32(width * np.float32(k))) for k in range(NFFT // 2)]
    for b in range(NMEL):
        left = np.float32(lo + np.float32(b) * delta)
        center = np.float32(lo + np.float32(b + 1) * delta)
        right = np.float32(lo + np.float32(b + 2) * delta)
        for k in range(NFFT // 2):
            mk = m[k]
            if left < mk < right:
                w[b, k] = (mk - left) / (center - left) if mk <= center else (right - mk) / (right - center)
    return w


def hamming() -> np.ndarray:
    """feature-window.cc:32-42: 0.54 - 0.46 cos(2 pi i / (N - 1)) in f64, stored as f32."""
    a = 2.0 * np.pi / (FL - 1)
    return (0.54 - 0.46 * np.cos(a * np.arange(FL))).astype(np.float32)


def fbank(wav: np.ndarray) -> np.ndarray:
    """wav: float samples in [-1, 1). Returns log-mel [N, 80] f32 (N = 1 + (S-400)//160).

    Follows knf's float / double boundaries: the DC mean is a sequential f32 sum / 400
    (feature-window.cc:179-190; np.cumsum accumulates sequentially), pre-emphasis and window in f32
    (:200-211, :57-63), the rfft in f64 (rfft.cc:41-47: float -> double -> float; numpy's pocketfft and
    Ooura's rdft agree after the f32 rounding), |X|^2 in f32 (feature-functions.cc:28-47), mel sums
    sequential in f32 over each bin's support (mel-computations.cc:224-247), log(max(e, FLT_EPSILON))
    (feature-fbank.cc:102-108) as the f64 log rounded to f32 (the correctly rounded logf; glibc's logf
    differs from it on ~0.03 % of the energies)."""
    x = np.asarray(wav, np.float32) * np.float32(32768.0)
    n = 0 if len(x) < FL else 1 + (len(x) - FL) // FS
    if n == 0:
        return np.zeros((0, NMEL), np.float32)
    idx = np.arange(n)[:, None] * FS + np.arange(FL)[None, :]
    fr = x[idx].astype(np.float32)
    mean = np.cumsum(fr, axis=1, dtype=np.float32)[:, -1:] / np.float32(FL)
    fr = (fr - mean.astype(np.float32)).astype(np.float32)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = ((fr - np.float32(0.97) * prev).astype(np.float32) * hamming()[None, :]).astype(np.float32)
    spec = np.fft.rfft(fr.astype(np.float64), n=NFFT, axis=1)[:, : NFFT // 2]
    re, im = spec.real.astype(np.float32), spec.imag.astype(np.float32)
    p = (re * re + im * im).astype(np.float32)
    W = mel_banks()
    e = np.zeros((n, NMEL), np.float32)
    for b in range(NMEL):
        nz = np.nonzero(W[b])[0]
        acc = np.zeros(n, np.float32)
        for k in range(int(nz[0]), int(nz[-1]) + 1):
            acc = (acc + W[b, k] * p[:, k]).astype(np.float32)
        e[:, b] = acc
    t = np.maximum(e, np.float32(1.1920928955078125e-07))
    return np.log(t.astype(np.float64)).astype(np.float32)


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
