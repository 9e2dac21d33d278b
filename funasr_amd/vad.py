"""`FsmnVADStreaming` voice-activity detector with the reference's plugin contract, backed by libpfm_hip.so.

Contract (funasr/models/fsmn_vad_streaming/model.py:281-916):
  * registered as tables.model_classes["FsmnVADStreaming"]; constructed as cls(encoder="FSMN",
    encoder_conf=..., **vad options); state_dict keys of the reference FSMN encoder;
  * inference(data_in, key, frontend, cache={}, **kwargs) -> ([{"key", "value": [[beg_ms, end_ms], ...]}], meta)
    over 60 s sample chunks (chunk_size 60000) with the online frontend (LFR 5/1) and its caches; offline
    (is_streaming_input False) segments are [beg, end] pairs.
The FSMN encoder (the per-frame silence posteriors) runs in the HIP library (pfm_vad_run) with its
memory caches in HBM; the detection state machine over those per-frame values is host code, as in the
reference (E2EVadModel: GetFrameState, WindowDetector, DetectOneFrame and the output-buffer bookkeeping),
native in the library (pfm_vad_detector_*). `VadDetector` below is its Python statement (frame decibels
and the same state machine), kept as the readable specification the native one is tested against.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import FsmnVADConfig
from .frontend import WavFrontendOnline
from .model import HipModel
from .register import tables
from .writer import model_writer

# VadStateMachine / FrameState / AudioChangeState (model.py:22-41)
START_NOT_DETECTED, IN_SPEECH, END_DETECTED = 1, 2, 3
F_INVALID, F_SIL, F_SPEECH = -1, 0, 1
C_S2S, C_SP2SIL, C_SIL2SIL, C_SIL2SP, C_INVALID = 0, 1, 2, 3, 5
SINGLE_UTT, MULTI_UTT = 0, 1


class WindowDetector:
    """model.py:159-241: a sliding window of frame decisions with two thresholds (hysteresis)."""

    def __init__(self, window_ms, sil2speech_ms, speech2sil_ms, frame_ms):
        self.win = int(window_ms / frame_ms)
        self.s2p = int(sil2speech_ms / frame_ms)
        self.p2s = int(speech2sil_ms / frame_ms)
        self.reset()

    def reset(self):
        self.pos, self.sum, self.state, self.pre = 0, 0, [0] * self.win, F_SIL

    def detect(self, frame_state: int) -> int:
        if frame_state not in (F_SPEECH, F_SIL):
            return C_INVALID
        cur = 1 if frame_state == F_SPEECH else 0
        self.sum += cur - self.state[self.pos]
        self.state[self.pos] = cur
        self.pos = (self.pos + 1) % self.win
        if self.pre == F_SIL and self.sum >= self.s2p:
            self.pre = F_SPEECH
            return C_SIL2SP
        if self.pre == F_SPEECH and self.sum <= self.p2s:
            self.pre = F_SIL
            return C_SP2SIL
        return C_SIL2SIL if self.pre == F_SIL else C_S2S


class Segment:
    __slots__ = ("start_ms", "end_ms", "has_start", "has_end")

    def __init__(self, start_ms):
        self.start_ms = self.end_ms = start_ms
        self.has_start = self.has_end = False


class VadDetector:
    """The per-stream E2E VAD state (model.py Stats + cache) and its frame loop. Frame values are kept
    with absolute indices (the reference drops consumed frames from the front of its arrays and indexes
    them relative to the drop count: the same element)."""

    def __init__(self, opts: Dict):
        self.o = dict(opts)
        self.frame_ms = int(self.o["frame_in_ms"])
        self.win = WindowDetector(self.o["window_size_ms"], self.o["sil_to_speech_time_thres"],
                                  self.o["speech_to_sil_time_thres"], self.frame_ms)
        self.max_end_sil = self.o["max_end_silence_time"] - self.o["speech_to_sil_time_thres"]
        self.p_sil: List[float] = []
        self.decibel: List[float] = []
        self.data_buf_start_frame = 0
        self.frm_cnt = 0
        self.latest_speech = 0
        self.latest_sil = -1
        self.cont_sil = 0
        self.state = START_NOT_DETECTED
        self.conf_start = -1
        self.conf_end = -1
        self.n_end = 0
        self.noise_db = -100.0
        self.next_seg = True
        self.out: List[Segment] = []
        self.out_offset = 0
        self.last_drop = 0

    # ---- per-chunk inputs (ComputeDecibel :326-348, ComputeScores :350-360)
    def frame_decibels(self, w: np.ndarray) -> np.ndarray:
        """ComputeDecibel (:326-348) over one chunk's waveform, float32 as the reference. The frames
        are a strided view (no gather copy); np.square materialises the same contiguous [n, fl]
        block the reference sums, so the values are bit-identical to its fancy-indexed frames."""
        fl = int(self.o["frame_length_ms"] * self.o["sample_rate"] / 1000)
        fs = int(self.frame_ms * self.o["sample_rate"] / 1000)
        w = np.asarray(w, np.float32).reshape(-1)
        if len(w) < fl:
            return np.zeros((0,), np.float32)
        frames = np.lib.stride_tricks.sliding_window_view(w, fl)[::fs]
        return 10 * np.log10(np.sum(np.square(frames), axis=1) + 0.000001)

    def add_waveform(self, w: np.ndarray):
        self.decibel.extend(self.frame_decibels(w).tolist())

    def add_scores(self, p_sil: np.ndarray):
        self.p_sil.extend(float(x) for x in np.asarray(p_sil, np.float32))
        self.frm_cnt += len(p_sil)

    # ---- GetFrameState (:493-546)
    def frame_state(self, t: int) -> int:
        db = self.decibel[t]
        snr = db - self.noise_db
        if db < self.o["decibel_thres"]:
            # (:498-499) the reference also runs the detector here, at the drop-relative frame index
            self.detect_one(F_SIL, t - self.last_drop, False)
            return F_SIL
        s = self.p_sil[t]
        noise_prob = math.log(s) * self.o["speech_2_noise_ratio"]
        speech_prob = math.log(1.0 - s)
        if math.exp(speech_prob) >= math.exp(noise_prob) + self.o["speech_noise_thres"]:
            if snr >= self.o["snr_thres"] and db >= self.o["decibel_thres"]:
                return F_SPEECH
            return F_SIL
        if self.noise_db < -99.9:
            self.noise_db = db
        else:
            n = self.o["noise_frame_num_used_for_snr"]
            self.noise_db = (db + self.noise_db * (n - 1)) / n
        return F_SIL

    # ---- output buffer (:362-441)
    def pop_till(self, frame: int):
        if self.data_buf_start_frame < frame:
            self.data_buf_start_frame = frame

    def pop_to_output(self, start, cnt, first_is_start, last_is_end):
        self.pop_till(start)
        if not self.out or first_is_start:
            self.out.append(Segment(start * self.frame_ms))
        seg = self.out[-1]
        self.data_buf_start_frame += cnt
        seg.end_ms = (start + cnt) * self.frame_ms
        if first_is_start:
            seg.has_start = True
        if last_is_end:
            seg.has_end = True

    def on_silence(self, frame):
        self.latest_sil = frame
        if self.state == START_NOT_DETECTED:
            self.pop_till(frame)

    def on_voice(self, frame):
        self.latest_speech = frame
        self.pop_to_output(frame, 1, False, False)

    def on_voice_start(self, frame, fake=False):
        if self.conf_start == -1:
            self.conf_start = frame
        if not fake and self.state == START_NOT_DETECTED:
            self.pop_to_output(self.conf_start, 1, True, False)

    def on_voice_end(self, frame, fake, is_last):
        for t in range(self.latest_speech + 1, frame):
            self.on_voice(t)
        if self.conf_end == -1:
            self.conf_end = frame
        if not fake:
            self.pop_to_output(self.conf_end, 1, False, True)
        self.n_end += 1

    def maybe_end_if_last(self, is_final, idx):
        if is_final:
            self.on_voice_end(idx, False, True)
            self.state = END_DETECTED

    def latency(self) -> int:
        v = self.win.win
        if self.o["do_extend"]:
            v += int(self.o["lookback_time_start_point"] / self.frame_ms)
        return v

    def reset_detection(self):   # ResetDetection (:303-324)
        self.cont_sil = 0
        self.latest_speech = 0
        self.latest_sil = -1
        self.conf_start = -1
        self.conf_end = -1
        self.state = START_NOT_DETECTED
        self.win.reset()
        if self.out:
            if not self.out[-1].has_end:
                raise RuntimeError("VAD reset with an open segment")
            self.last_drop = int(self.out[-1].end_ms / self.frame_ms)

    # ---- DetectOneFrame (:782-916)
    def detect_one(self, frm_state: int, idx: int, is_final: bool):
        tmp = F_INVALID
        if frm_state == F_SPEECH:
            tmp = F_SPEECH if math.fabs(1.0) > self.o["fe_prior_thres"] else F_SIL
        elif frm_state == F_SIL:
            tmp = F_SIL
        ch = self.win.detect(tmp)
        max_seg = self.o["max_single_segment_time"] / self.frame_ms
        if ch == C_SIL2SP:
            self.cont_sil = 0
            if self.state == START_NOT_DETECTED:
                start = max(self.data_buf_start_frame, idx - self.latency())
                self.on_voice_start(start)
                self.state = IN_SPEECH
                for t in range(start + 1, idx + 1):
                    self.on_voice(t)
            elif self.state == IN_SPEECH:
                for t in range(self.latest_speech + 1, idx):
                    self.on_voice(t)
                if idx - self.conf_start + 1 > max_seg:
                    self.on_voice_end(idx, False, False)
                    self.state = END_DETECTED
                elif not is_final:
                    self.on_voice(idx)
                else:
                    self.maybe_end_if_last(is_final, idx)
        elif ch == C_SP2SIL:
            self.cont_sil = 0
            if self.state == IN_SPEECH:
                if idx - self.conf_start + 1 > max_seg:
                    self.on_voice_end(idx, False, False)
                    self.state = END_DETECTED
                elif not is_final:
                    self.on_voice(idx)
                else:
                    self.maybe_end_if_last(is_final, idx)
        elif ch == C_S2S:
            self.cont_sil = 0
            if self.state == IN_SPEECH:
                if idx - self.conf_start + 1 > max_seg:
                    self.on_voice_end(idx, False, False)
                    self.state = END_DETECTED
                elif not is_final:
                    self.on_voice(idx)
                else:
                    self.maybe_end_if_last(is_final, idx)
        elif ch == C_SIL2SIL:
            self.cont_sil += 1
            if self.state == START_NOT_DETECTED:
                if ((self.o["detect_mode"] == SINGLE_UTT
                     and self.cont_sil * self.frame_ms > self.o["max_start_silence_time"])
                        or (is_final and self.n_end == 0)):
                    for t in range(self.latest_sil + 1, idx):
                        self.on_silence(t)
                    self.on_voice_start(0, True)
                    self.on_voice_end(0, True, False)
                    self.state = END_DETECTED
                elif idx >= self.latency():
                    self.on_silence(idx - self.latency())
            elif self.state == IN_SPEECH:
                if self.cont_sil * self.frame_ms >= self.max_end_sil:
                    look = int(self.max_end_sil / self.frame_ms)
                    if self.o["do_extend"]:
                        look -= int(self.o["lookahead_time_end_point"] / self.frame_ms)
                        look -= 1
                        look = max(0, look)
                    self.on_voice_end(idx - look, False, False)
                    self.state = END_DETECTED
                elif idx - self.conf_start + 1 > max_seg:
                    self.on_voice_end(idx, False, False)
                    self.state = END_DETECTED
                elif self.o["do_extend"] and not is_final:
                    if self.cont_sil <= int(self.o["lookahead_time_end_point"] / self.frame_ms):
                        self.on_voice(idx)
                else:
                    self.maybe_end_if_last(is_final, idx)
        if self.state == END_DETECTED and self.o["detect_mode"] == MULTI_UTT:
            self.reset_detection()

    # ---- DetectCommonFrames / DetectLastFrames (:755-780) over the chunk's n new frames
    def detect_chunk(self, n: int, is_final: bool):
        if self.state == END_DETECTED:
            return
        for i in range(n - 1, -1, -1):
            t = self.frm_cnt - 1 - i
            st = self.frame_state(t)
            self.detect_one(st, t, is_final and i == 0)

    def segments(self, is_final: bool, streaming: bool) -> List[List[int]]:
        """forward() output (:566-613) for one call."""
        segs = []
        for i in range(self.out_offset, len(self.out)):
            s = self.out[i]
            if streaming:
                if not s.has_start:
                    continue
                if not self.next_seg and not s.has_end:
                    continue
                beg = s.start_ms if self.next_seg else -1
                if s.has_end:
                    end = s.end_ms
                    self.next_seg = True
                    self.out_offset += 1
                else:
                    end = -1
                    self.next_seg = False
                segs.append([beg, end])
            else:
                if not is_final and (not s.has_start or not s.has_end):
                    continue
                segs.append([s.start_ms, s.end_ms])
                self.out_offset += 1
        return segs


@tables.register("model_classes", "FsmnVADStreaming")
class FsmnVADStreaming(HipModel):
    family = "fsmn_vad"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.cfg = FsmnVADConfig.from_kwargs(**kwargs)
        self._init_common(kwargs)
        self._vad = None

    def engine(self):   # the VAD has its own small C-ABI object (pfm_vad), not a pfm_handle
        from .runtime import PfmError, PfmVad
        dev = self._device_index()
        if self._engine is None or self._engine_dev != dev:
            v = PfmVad(self.cfg, dev)
            if self._host_sd:
                v.load_state_dict(self._host_sd)
            self._engine, self._engine_dev = v, dev
        if self._engine.missing_weights:
            raise PfmError(f"{self._engine.missing_weights} FSMN-VAD weights not loaded")
        return self._engine

    def init_cache(self, cache: dict, **kwargs) -> dict:
        cache.clear()
        opts = dict(self.cfg.vad_opts)
        if kwargs.get("max_end_silence_time") is not None:
            opts["max_end_silence_time"] = kwargs["max_end_silence_time"]
        from .runtime import PfmVadDetector
        cache.update(frontend={}, prev_samples=np.zeros((0,), np.float32), detector=PfmVadDetector(opts),
                     db_calc=VadDetector(opts))
        self.engine().reset()
        return cache

    @torch.no_grad()
    def inference(self, data_in, data_lengths=None, key: List[str] = None, tokenizer=None, frontend=None,
                  cache: Optional[dict] = None, **kwargs):
        cache = {} if cache is None else cache
        if len(cache) == 0:
            self.init_cache(cache, **kwargs)
        fe = frontend if isinstance(frontend, WavFrontendOnline) and frontend.lfr_m == self.cfg.lfr_m else \
            WavFrontendOnline(cmvn_file=None, lfr_m=self.cfg.lfr_m, lfr_n=self.cfg.lfr_n)
        if frontend is not None and fe is not frontend and getattr(frontend, "cmvn", None) is not None:
            fe.cmvn = np.asarray(frontend.cmvn, np.float32)
        chunk_ms = kwargs.get("chunk_size", 60000)
        streaming = kwargs.get("is_streaming_input", False if chunk_ms >= 15000 else True)
        is_final = kwargs.get("is_final", False) if streaming else kwargs.get("is_final", True)
        x = data_in[0] if isinstance(data_in, (list, tuple)) else data_in
        if isinstance(x, str):
            from .frontend import read_wav
            x, is_final = read_wav(x), True
        x = x.detach().cpu().numpy() if hasattr(x, "detach") else x
        x = np.asarray(x, np.float32).reshape(-1)   # no copy of a float32 waveform (300 s: 19 MB)
        prev = cache["prev_samples"]
        audio = np.concatenate([prev, x]) if prev.size else x
        stride = int(chunk_ms * fe.fs / 1000)
        n = int(len(audio) // stride + int(is_final))
        m = int(len(audio) % stride * (1 - int(is_final)))
        eng = self.engine()
        det = cache["detector"]          # native state machine (pfm_vad_detector)
        dbc: VadDetector = cache["db_calc"]
        fl_s = int(dbc.o["frame_length_ms"] * dbc.o["sample_rate"] / 1000)
        fs_s = int(dbc.frame_ms * dbc.o["sample_rate"] / 1000)
        segments: List[List[int]] = []
        for i in range(n):
            fin = is_final and i == n - 1
            seg = audio[i * stride:(i + 1) * stride]
            feats = fe.step(eng, [(seg, fin, cache["frontend"])])[0]
            wv = cache["frontend"].get("waveforms")
            # ComputeDecibel: the frame energies on the device (numpy's float32 summation order), the log in numpy
            # float32 as the reference (dbc.frame_decibels is the host statement of the same values)
            if wv is not None and len(wv) >= fl_s:
                db_new = (10 * np.log10(eng.frame_energy(wv, fl_s, fs_s) + 0.000001)).astype(np.float64)
            else:
                db_new = np.zeros((0,))
            p = eng.run(feats).cpu().numpy() if feats.shape[0] else np.zeros((0,), np.float32)
            segments.extend(det.push(db_new, p, fin, streaming))
        # (a copy: the caller's waveform is neither kept alive nor aliased by the cache)
        cache["prev_samples"] = audio[:-m].copy() if m else np.zeros((0,), np.float32)
        if is_final:
            self.init_cache(cache, **kwargs)
        key = self._keys(key, 1)
        writer = model_writer(self, kwargs)   # output_dir: 1best_recog/text (fsmn_vad_streaming/model.py:730-744)
        if writer is not None:
            writer["1best_recog"]["text"][key[0]] = segments
        return [{"key": key[0], "value": segments}], {}
