"""WavFrontend on the HIP path: waveform -> fbank -> LFR -> CMVN via pfm_fbank.

Host responsibilities mirrored from funasr/frontends/wav_frontend.py:
  load_cmvn  (:15-38)  Kaldi nnet1 text file: <AddShift> / <Rescale> vectors -> [2, D] f32
  WavFrontend(fs, window, n_mels, frame_length, frame_shift, lfr_m, lfr_n, dither, cmvn_file)
  forward    (:118-158) batch of waveforms -> (feats [B,T,560], lens [B])
The per-sample arithmetic (fbank, LFR, CMVN) runs in funasr_amd/csrc/k_fbank.hip.
Audio input: float arrays in [-1, 1), or 16-bit PCM WAV files (stdlib `wave`; the reference
uses torchaudio/librosa, which are not part of this build).
"""
from __future__ import annotations

import os
import wave
from typing import List, Optional, Sequence

import numpy as np


def load_cmvn(cmvn_file: str) -> np.ndarray:
    """Parse am.mvn: the vector after <AddShift>'s <LearnRateCoef> line is the shift, the one after
    <Rescale>'s is the scale. Returns float32 [2, D]."""
    with open(cmvn_file, encoding="utf-8") as f:
        lines = f.readlines()
    shift, scale = None, None
    for i, line in enumerate(lines):
        tok = line.split()
        if not tok or i + 1 >= len(lines):
            continue
        nxt = lines[i + 1].split()
        if tok[0] in ("<AddShift>", "<Rescale>") and nxt and nxt[0] == "<LearnRateCoef>":
            vec = np.array(nxt[3:-1], dtype=np.float32)   # "<LearnRateCoef> 0 [ v0 v1 ... ]"
            if tok[0] == "<AddShift>":
                shift = vec
            else:
                scale = vec
    if shift is None or scale is None:
        raise ValueError(f"{cmvn_file}: missing <AddShift>/<Rescale> blocks")
    return np.stack([shift, scale]).astype(np.float32)


def read_wav(path: str, fs: int = 16000) -> np.ndarray:
    """16-bit PCM WAV -> float32 in [-1, 1) (first channel)."""
    with wave.open(path, "rb") as w:
        if w.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM WAV is supported")
        if w.getframerate() != fs:
            raise ValueError(f"{path}: sample rate {w.getframerate()} != {fs} (resampling is not supported)")
        n, ch = w.getnframes(), w.getnchannels()
        x = np.frombuffer(w.readframes(n), dtype="<i2").reshape(-1, ch)[:, 0]
    return x.astype(np.float32) / 32768.0


class WavFrontend:
    """Offline Kaldi-fbank + LFR + CMVN frontend (options of wav_frontend.py:80-97)."""

    def __init__(self, cmvn_file: Optional[str] = None, fs: int = 16000, window: str = "hamming", n_mels: int = 80,
                 frame_length: int = 25, frame_shift: int = 10, lfr_m: int = 7, lfr_n: int = 6,
                 dither: float = 0.0, snip_edges: bool = True, upsacle_samples: bool = True, **kwargs):
        if (fs, window, n_mels, frame_length, frame_shift, lfr_m, lfr_n) != (16000, "hamming", 80, 25, 10, 7, 6):
            raise ValueError("the HIP frontend implements fs=16000, hamming, 80 mel, 25/10 ms, LFR 7/6")
        if not snip_edges or not upsacle_samples:
            raise ValueError("the HIP frontend implements snip_edges=True, upsacle_samples=True")
        if dither != 0.0:
            # the reference default dither=1.0 adds Gaussian noise per call (non-deterministic);
            # the C++ runtime forces 0 (runtime/onnxruntime/src/paraformer.cpp:24) and so does this build
            dither = 0.0
        self.fs, self.frame_shift, self.lfr_n = fs, frame_shift, lfr_n
        self.cmvn_file = cmvn_file
        self.cmvn = load_cmvn(cmvn_file) if cmvn_file else None

    def output_size(self) -> int:
        return 560

    def load(self, item) -> np.ndarray:
        if isinstance(item, str):
            return read_wav(item, self.fs)
        if hasattr(item, "detach"):
            item = item.detach().cpu().numpy()
        return np.asarray(item, dtype=np.float32).reshape(-1)

    def __call__(self, engine, wavs: Sequence, device=None):
        """List of waveforms -> (feats [B,T,560] cuda f32, lens [B] cuda int32) via pfm_fbank."""
        import torch
        arrs: List[np.ndarray] = [self.load(w) for w in wavs]
        S = max(1, max(len(a) for a in arrs))
        buf = np.zeros((len(arrs), S), dtype=np.float32)
        for i, a in enumerate(arrs):
            buf[i, : len(a)] = a
        ns = np.array([len(a) for a in arrs], dtype=np.int32)
        if (ns < 400).any():
            raise ValueError("waveforms shorter than one 25 ms frame (400 samples) are not supported")
        dev = torch.device("cuda", engine.device)
        feats, t_out = engine.fbank(torch.from_numpy(buf).to(dev), torch.from_numpy(ns).to(dev), self.cmvn)
        return feats, t_out, ns
