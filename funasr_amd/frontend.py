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


class WavFrontendOnline(WavFrontend):
    """Online fbank + LFR + CMVN (WavFrontendOnline, funasr/frontends/wav_frontend.py:211-478), batched
    over streams. Per stream the cache holds what the reference's does, reduced to what its outputs
    depend on: the carried samples (`input_cache`, forward_fbank :322-333), the length of
    `reserve_waveforms` (its contents are never read, only its size and emptiness, :424-445), and the
    LFR splice frames (`lfr_splice_cache`, kept on the device). The integer bookkeeping of apply_lfr
    (:275-310) runs on the host; the fbank frames (pfm_fbank_raw) and the LFR/CMVN row gather
    (pfm_lfr_gather) run in k_fbank.hip.
    """
    FL, FS = 400, 160

    def __init__(self, cmvn_file: Optional[str] = None, lfr_m: int = 7, lfr_n: int = 6, **kwargs):
        # the fbank options are checked by WavFrontend; LFR (m, n) is free here (ASR 7/6, FSMN-VAD 5/1)
        super().__init__(cmvn_file=cmvn_file, **kwargs)
        if lfr_m < 1 or lfr_n < 1:
            raise ValueError("lfr_m / lfr_n must be >= 1")
        self.lfr_m, self.lfr_n = int(lfr_m), int(lfr_n)
        self._cmvn_dev = {}

    def output_size(self) -> int:
        return 80 * self.lfr_m

    @staticmethod
    def init_cache(cache: dict) -> dict:
        """init_cache (wav_frontend.py:468-476): carried samples, reserve_waveforms, splice frames; `waveforms`
        = the samples of the last call's frames (cache["waveforms"], read by the VAD's decibel pass)."""
        cache.clear()
        cache.update(input_cache=np.zeros((0,), np.float32), reserve=np.zeros((0,), np.float32), splice=None,
                     waveforms=None)
        return cache

    def _cmvn_on(self, torch, dev):
        if self.cmvn is None:
            return None
        k = str(dev)
        if k not in self._cmvn_dev:
            self._cmvn_dev[k] = torch.from_numpy(np.ascontiguousarray(self.cmvn, dtype=np.float32)).to(dev)
        return self._cmvn_dev[k]

    def _lfr_index(self, T: int, is_final: bool):
        """apply_lfr on T frames: (frame index per output row [rows, m], splice_idx). Padded frames of the
        final chunk repeat the last frame (:285-293)."""
        m, n = self.lfr_m, self.lfr_n
        T_lfr = int(np.ceil((T - (m - 1) // 2) / n))
        splice_idx = T_lfr
        last_idx = (T - m) // n + 1
        num_padding = m - (T - last_idx * n)
        rows, T_in = T_lfr, T
        if is_final:
            if num_padding > 0:
                num_padding = (2 * m - 2 * T + (T_lfr - 1 + last_idx) * n) / 2 * (T_lfr - last_idx)
                T_in = T + int(num_padding)
        elif num_padding > 0:
            rows = last_idx
            splice_idx = last_idx
        splice_idx = min(T - 1, splice_idx * n)
        rows = max(rows, 0)
        idx = np.arange(rows)[:, None] * n + np.arange(m)[None, :]
        if rows and idx.max() >= T_in:
            raise ValueError("online LFR would read past the input frames (apply_lfr as_strided)")
        return np.minimum(idx, T - 1).astype(np.int32), splice_idx

    def step(self, engine, items):
        """items: list of (wav chunk (1-D f32), is_final, cache) -> list of feats [rows, 560] cuda f32
        (rows may be 0), one pfm_fbank_raw launch and one pfm_lfr_gather launch for all streams."""
        import torch
        dev = torch.device("cuda", engine.device)
        xs, nfrs = [], []
        for wav, _, cache in items:
            if not cache:
                self.init_cache(cache)
            w = self.load(wav)
            x = np.concatenate([cache["input_cache"], w]) if cache["input_cache"].size else w   # (no copy of a fresh chunk)
            nfr = int((x.shape[0] - self.FL) / self.FS + 1)
            nfr = nfr if nfr >= 1 and x.shape[0] >= self.FL else 0
            keep = x.shape[0] - nfr * self.FS
            cache["input_cache"] = (x[-keep:] if keep else x).copy()     # x[-0:] is all of x (:331-333); never a view
                                                                        # of the caller's buffer
            xs.append(x[: (nfr - 1) * self.FS + self.FL] if nfr else x[:0])
            nfrs.append(nfr)
        fb = None
        if any(nfrs):
            S = max(len(u) for u in xs)
            if len(xs) == 1:   # one stream (the VAD, batch 1): no padded staging copy
                buf = np.ascontiguousarray(xs[0], dtype=np.float32)[None]
            else:
                buf = np.zeros((len(xs), S), np.float32)
                for k, u in enumerate(xs):
                    buf[k, : len(u)] = u
            fb = engine.fbank_raw(torch.from_numpy(buf).to(dev), [len(u) for u in xs])
        srcs, idxs, offs, out_rows = [], [], 0, []
        for k, (wav, is_final, cache) in enumerate(items):
            nfr, used = nfrs[k], xs[k]
            rows_k = 0
            if nfr:
                fbk = fb[k, :nfr]
                waves = np.concatenate([cache["reserve"], used])          # (:424)
                cache["waveforms"] = waves
                if cache["splice"] is None:
                    cache["splice"] = fbk[:1].repeat((self.lfr_m - 1) // 2, 1)
                if nfr + cache["splice"].shape[0] >= self.lfr_m:
                    feats = torch.cat([cache["splice"], fbk])
                    idx, sidx = self._lfr_index(feats.shape[0], is_final)
                    from_w = int((len(waves) - self.FL) / self.FS + 1)
                    minus = (self.lfr_m - 1) // 2 if cache["reserve"].size == 0 else 0
                    lo = (sidx - minus) * self.FS
                    cache["reserve"] = waves[lo:from_w * self.FS]                              # (:447-452)
                    cache["waveforms"] = waves[:(from_w - 1) * self.FS + self.FL]               # (:453-456)
                    cache["splice"] = feats[sidx:].clone()
                    srcs.append(feats)
                    idxs.append(idx + offs)
                    offs += feats.shape[0]
                    rows_k = idx.shape[0]
                else:
                    cache["reserve"] = waves[:-(self.FL - self.FS)]                              # (:458-461)
                    cache["splice"] = torch.cat([cache["splice"], fbk])
            elif is_final and cache["splice"] is not None:
                # (:474-483): the frames of the call are the reserve (or none)
                cache["waveforms"] = cache["reserve"] if cache["reserve"].size else np.zeros((0,), np.float32)
                idx, _ = self._lfr_index(cache["splice"].shape[0], True)
                srcs.append(cache["splice"])
                idxs.append(idx + offs)
                offs += cache["splice"].shape[0]
                rows_k = idx.shape[0]
            out_rows.append(rows_k)
        if not srcs or sum(out_rows) == 0:
            return [torch.zeros((0, 80 * self.lfr_m), dtype=torch.float32, device=dev) for _ in items]
        frames = torch.cat(srcs) if len(srcs) > 1 else srcs[0]
        allf = engine.lfr_gather(frames, np.concatenate(idxs), self.lfr_m, self._cmvn_on(torch, dev))
        return list(torch.split(allf, out_rows))
