"""ctypes binding of libpfm_hip.so (include/pfm.h) + a torch-facing engine wrapper.

The HIP library is the only compute path: importing this module does not require a GPU,
but constructing a `PfmEngine` does, and there is no CPU fallback anywhere in the
product — a missing library or device raises `PfmError`.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import numpy as np

from .config import CTTransformerConfig, ParaformerConfig, SenseVoiceConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PFM_LIB", os.path.join(_HERE, "_lib", "libpfm_hip.so"))

PFM_F32, PFM_BF16 = 0, 1
ARCH_PARAFORMER, ARCH_SENSEVOICE, ARCH_PUNC = 0, 1, 2
MODE_EXACT, MODE_FAST = 0, 1
MODES = {"exact": MODE_EXACT, "fp32": MODE_EXACT, "fast": MODE_FAST, "bf16": MODE_FAST}

# every symbol include/pfm.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = ("pfm_config_default", "pfm_config_sensevoice", "pfm_create", "pfm_run_beam", "pfm_set_weight", "pfm_set_weight_device",
               "pfm_missing_weights", "pfm_reserve", "pfm_run", "pfm_run_ctc", "pfm_ctc_align", "pfm_op_ctc_collapse", "pfm_fbank", "pfm_lfr_frames", "pfm_last_error", "pfm_destroy", "pfm_op_gemm",
               "pfm_op_attention", "pfm_op_layernorm", "pfm_op_ln_gemm", "pfm_op_fsmn", "pfm_op_cif", "pfm_op_ctc_beam", "pfm_profile", "pfm_op_ffn", "pfm_op_ffn_op", "pfm_op_ffn_op_qkv", "pfm_op_ffn_dec", "pfm_op_fsmn_bf16", "pfm_op_layernorm_bf16",
               "pfm_profile_read", "pfm_streams_create", "pfm_streams_reset", "pfm_stream_step", "pfm_stream_step_beam",
               "pfm_streams_destroy", "pfm_fbank_raw", "pfm_lfr_gather", "pfm_config_punc", "pfm_run_punc", "pfm_vad_config_default", "pfm_vad_create",
               "pfm_vad_set_weight", "pfm_vad_missing_weights", "pfm_vad_reset", "pfm_vad_run", "pfm_vad_destroy", "pfm_vad_fbank_raw", "pfm_vad_frame_energy", "pfm_run_punc_host",
               "pfm_vad_opts_default", "pfm_vad_detector_create", "pfm_vad_detector_push", "pfm_vad_detector_destroy")


class PfmError(RuntimeError):
    pass


class PfmConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("input_size", "d_model", "heads", "ffn", "enc_blocks", "dec_blocks",
                                               "kernel_size", "enc_sanm_shift", "dec_sanm_shift", "vocab_size",
                                               "cif_l_order", "cif_r_order")] + \
              [(n, ctypes.c_float) for n in ("cif_threshold", "tail_threshold", "smooth_factor", "noise_threshold",
                                             "ln_eps")] + \
              [(n, ctypes.c_int32) for n in ("arch", "tp_blocks", "n_embed", "ctc_head")]

    @classmethod
    def from_config(cls, c) -> "PfmConfig":
        if isinstance(c, CTTransformerConfig):
            return cls(c.input_size, c.d_model, c.heads, c.ffn, c.enc_blocks, 0, c.kernel_size, c.enc_sanm_shift, 0,
                       c.n_punc, 1, 1, 1.0, 0.45, 1.0, 0.0, c.ln_eps, ARCH_PUNC, 0, c.vocab_size, 0)
        if isinstance(c, SenseVoiceConfig):
            return cls(c.input_size, c.d_model, c.heads, c.ffn, c.enc_blocks, 0, c.kernel_size, c.enc_sanm_shift, 0,
                       c.vocab_size, 1, 1, 1.0, 0.45, 1.0, 0.0, c.ln_eps, ARCH_SENSEVOICE, c.tp_blocks, c.n_embed, 0)
        return cls(c.input_size, c.d_model, c.heads, c.ffn, c.enc_blocks, c.dec_blocks, c.kernel_size,
                   c.enc_sanm_shift, c.dec_sanm_shift, c.vocab_size, c.cif_l_order, c.cif_r_order,
                   c.cif_threshold, c.tail_threshold, c.smooth_factor, c.noise_threshold, c.ln_eps,
                   ARCH_PARAFORMER, 0, 0, 1 if getattr(c, "ctc_weight", 0.0) > 0.0 else 0)


class PfmVadConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("input_dim", "input_affine_dim", "fsmn_layers", "linear_dim", "proj_dim",
                                               "lorder", "output_affine_dim", "output_dim")]


class PfmVadOpts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("detect_mode", "max_end_silence_time", "max_start_silence_time",
                                               "window_size_ms", "sil_to_speech_time_thres",
                                               "speech_to_sil_time_thres", "do_extend", "lookback_time_start_point",
                                               "lookahead_time_end_point", "max_single_segment_time",
                                               "noise_frame_num_used_for_snr", "frame_in_ms")] + \
              [(n, ctypes.c_double) for n in ("speech_2_noise_ratio", "snr_thres", "decibel_thres",
                                              "speech_noise_thres", "fe_prior_thres")]


_lib = None


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and prototype libpfm_hip.so. Raises PfmError if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise PfmError(f"{p} not found: build it with `python -m funasr_amd.build` (hipcc, gfx950)")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    vp, i32, f32p, i32p = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p
    lib.pfm_config_default.argtypes = [ctypes.POINTER(PfmConfig)]
    lib.pfm_config_default.restype = None
    lib.pfm_config_sensevoice.argtypes = [ctypes.POINTER(PfmConfig)]
    lib.pfm_config_sensevoice.restype = None
    lib.pfm_run_ctc.argtypes = [vp, vp, i32, f32p, i32p, i32, i32, ctypes.POINTER(ctypes.c_int32), i32, i32p, i32,
                                i32p, f32p, i32p]
    lib.pfm_op_ctc_collapse.argtypes = [vp, i32p, ctypes.c_int64, i32p, i32, i32, i32p, i32, i32p]
    lib.pfm_ctc_align.argtypes = [vp, vp, f32p, i32, i32, i32p, i32p, i32, i32p, i32, i32p]
    lib.pfm_create.argtypes = [ctypes.POINTER(PfmConfig), i32, ctypes.POINTER(vp)]
    lib.pfm_set_weight.argtypes = [vp, ctypes.c_char_p, vp, i32, ctypes.POINTER(ctypes.c_int64), i32]
    lib.pfm_set_weight_device.argtypes = [vp, ctypes.c_char_p, vp, i32, ctypes.POINTER(ctypes.c_int64), i32, vp]
    lib.pfm_missing_weights.argtypes = [vp]
    lib.pfm_reserve.argtypes = [vp, i32, i32]
    lib.pfm_run.argtypes = [vp, vp, i32, f32p, i32p, i32, i32, i32p, i32, i32p, f32p, f32p, f32p]
    lib.pfm_run_beam.argtypes = [vp, vp, i32, f32p, i32p, i32, i32, i32, ctypes.c_float, ctypes.c_float, i32, i32,
                                 i32, i32, i32, i32p, i32, i32p, f32p, f32p, f32p]
    lib.pfm_fbank.argtypes = [vp, vp, f32p, i32p, i32, i32, f32p, f32p, i32, i32p]
    lib.pfm_lfr_frames.argtypes = [i32]
    lib.pfm_last_error.argtypes = []
    lib.pfm_last_error.restype = ctypes.c_char_p
    lib.pfm_destroy.argtypes = [vp]
    lib.pfm_destroy.restype = None
    lib.pfm_profile.argtypes = [vp, i32]
    lib.pfm_profile_read.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    lib.pfm_op_gemm.argtypes = [vp, i32, vp, vp, f32p, f32p, f32p, i32, i32, i32, i32]
    lib.pfm_op_ln_gemm.argtypes = [vp, f32p, f32p, f32p, ctypes.c_float, vp, f32p, f32p, vp, i32, i32, i32]
    lib.pfm_op_attention.argtypes = [vp, i32, vp, vp, vp, i32p, f32p, i32, i32, i32, i32, ctypes.c_float]
    lib.pfm_op_layernorm.argtypes = [vp, f32p, f32p, f32p, f32p, i32, i32, ctypes.c_float]
    lib.pfm_op_fsmn.argtypes = [vp, f32p, i32p, f32p, f32p, f32p, i32, i32, i32, i32, i32]
    lib.pfm_op_cif.argtypes = [vp, f32p, f32p, f32p, f32p, i32p, i32p, i32, i32, i32, i32]
    lib.pfm_op_ctc_beam.argtypes = [vp, f32p, i32, f32p, i32, i32p, i32p, i32, i32, i32, ctypes.c_float,
                                    ctypes.c_float, i32, i32, i32, i32, i32, i32p, i32, i32p, f32p]
    lib.pfm_op_layernorm_bf16.argtypes = [vp, vp, f32p, f32p, f32p, i32, i32, ctypes.c_float]
    lib.pfm_op_fsmn_bf16.argtypes = [vp, vp, i32p, f32p, vp, i32, i32, i32, i32, i32]
    lib.pfm_op_ffn.argtypes = [vp, f32p, i32, f32p, f32p, ctypes.c_float, f32p, f32p, f32p, f32p, f32p, f32p, f32p,
                               vp]
    lib.pfm_op_ffn_op.argtypes = [vp, vp, vp, f32p, f32p, f32p, i32, f32p, f32p, ctypes.c_float, f32p, f32p, f32p,
                                  f32p, f32p, f32p, f32p, vp]
    lib.pfm_op_ffn_op_qkv.argtypes = [vp, vp, vp, f32p, f32p, f32p, i32, f32p, f32p, ctypes.c_float, f32p, f32p, f32p,
                                      f32p, f32p, f32p, f32p, f32p, f32p, vp]
    lib.pfm_op_ffn_dec.argtypes = [vp, f32p, i32, f32p, f32p, ctypes.c_float, f32p, f32p, f32p, f32p, f32p, f32p,
                                   f32p, f32p, vp, vp, f32p, f32p]
    lib.pfm_streams_create.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_int32), i32, i32, i32, ctypes.POINTER(vp)]
    lib.pfm_streams_reset.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int32), i32]
    lib.pfm_stream_step.argtypes = [vp, vp, i32, ctypes.POINTER(ctypes.c_int32), f32p, i32,
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), i32p, i32, i32p,
                                    f32p, f32p]
    lib.pfm_stream_step_beam.argtypes = [vp, vp, i32, ctypes.POINTER(ctypes.c_int32), f32p, i32,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), i32,
                                         ctypes.c_float, ctypes.c_float, i32, i32, i32, i32, i32, i32p, i32, i32p,
                                         f32p, i32p]
    lib.pfm_fbank_raw.argtypes = [vp, vp, f32p, i32p, i32, i32, f32p, i32]
    lib.pfm_lfr_gather.argtypes = [vp, f32p, i32p, i32, i32, f32p, f32p]
    lib.pfm_config_punc.argtypes = [ctypes.POINTER(PfmConfig)]
    lib.pfm_config_punc.restype = None
    lib.pfm_run_punc.argtypes = [vp, vp, i32, i32p, i32p, i32, i32, i32p, f32p]
    lib.pfm_vad_config_default.argtypes = [ctypes.POINTER(PfmVadConfig)]
    lib.pfm_vad_config_default.restype = None
    lib.pfm_vad_create.argtypes = [ctypes.POINTER(PfmVadConfig), i32, ctypes.POINTER(vp)]
    lib.pfm_vad_set_weight.argtypes = [vp, ctypes.c_char_p, vp, i32, ctypes.POINTER(ctypes.c_int64), i32]
    lib.pfm_vad_missing_weights.argtypes = [vp]
    lib.pfm_vad_reset.argtypes = [vp, vp]
    lib.pfm_vad_run.argtypes = [vp, vp, f32p, i32, f32p, f32p]
    lib.pfm_vad_fbank_raw.argtypes = [vp, vp, f32p, i32p, i32, i32, f32p, i32]
    lib.pfm_vad_frame_energy.argtypes = [vp, vp, f32p, i32, i32, i32, f32p]
    lib.pfm_run_punc_host.argtypes = [vp, vp, i32, vp, i32, vp]
    lib.pfm_vad_opts_default.argtypes = [ctypes.POINTER(PfmVadOpts)]
    lib.pfm_vad_opts_default.restype = None
    lib.pfm_vad_detector_create.argtypes = [ctypes.POINTER(PfmVadOpts), ctypes.POINTER(vp)]
    lib.pfm_vad_detector_push.argtypes = [vp, vp, i32, vp, i32, i32, i32, vp, i32, ctypes.POINTER(ctypes.c_int32)]
    lib.pfm_vad_detector_destroy.argtypes = [vp]
    lib.pfm_vad_detector_destroy.restype = None
    lib.pfm_vad_destroy.argtypes = [vp]
    lib.pfm_vad_destroy.restype = None
    lib.pfm_streams_destroy.argtypes = [vp]
    lib.pfm_streams_destroy.restype = None
    for name in ABI_SYMBOLS:
        getattr(lib, name)
    if path is None:
        _lib = lib
    return lib


def check(rc: int, what: str = "pfm call"):
    if rc != 0:
        msg = load_library().pfm_last_error().decode(errors="replace")
        raise PfmError(f"{what} failed ({rc}): {msg}")


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _stream_ptr(torch, device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class PfmEngine:
    """One pfm_handle on one HIP device: weights + workspace, stream-ordered calls."""

    def __init__(self, cfg, device: int = 0):   # ParaformerConfig | SenseVoiceConfig
        import torch
        if not torch.cuda.is_available():
            raise PfmError("PfmEngine needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
        self.torch = torch
        self.cfg = cfg
        self.device = int(device)
        self.fast_only = False   # set by load_flat_device(fast_only=True): bf16-rounded matrices, no EXACT mode
        self.wire_xw = None      # the PFM_FAST_XW the bf16 wire split was made for (fast runs need the same bits)
        self.lib = load_library()
        c = PfmConfig.from_config(cfg)
        h = ctypes.c_void_p()
        check(self.lib.pfm_create(ctypes.byref(c), self.device, ctypes.byref(h)), "pfm_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.pfm_destroy(h)
            except Exception:
                pass
            self.h = None

    # ---- weights
    def set_weight(self, name: str, arr) -> None:
        a = np.ascontiguousarray(arr.detach().cpu().numpy() if hasattr(arr, "detach") else arr, dtype=np.float32)
        shape = (ctypes.c_int64 * a.ndim)(*a.shape)
        check(self.lib.pfm_set_weight(self.h, name.encode(), a.ctypes.data_as(ctypes.c_void_p), PFM_F32, shape,
                                      a.ndim), f"pfm_set_weight({name})")

    def load_state_dict(self, sd: Dict[str, "np.ndarray"], strict: bool = True) -> None:
        for k, v in sd.items():
            self.set_weight(k, v)
        miss = self.lib.pfm_missing_weights(self.h)
        if strict and miss:
            raise PfmError(f"{miss} required weights missing after load_state_dict")

    def load_flat_device(self, flat, layout, strict: bool = True, fast_only: bool = False,
                         wire_xw: Optional[int] = None) -> None:
        """Weights from ONE flat f32 device tensor on this engine's GPU, packed in `layout` order
        ([(key, shape, ...)], weights.param_layout) — e.g. the buffer a data-parallel rank received by
        RCCL broadcast (distributed.broadcast_state_dict(keep_on_device=True)). pfm_set_weight_device per
        key: device-to-device copies, nothing round-trips through the host. fast_only: the matrices were sent as
        bf16 (broadcast_state_dict(wire="bf16")), so EXACT mode is refused on this engine. wire_xw: the PFM_FAST_XW
        bits that wire split was made for (broadcast_state_dict(with_xw=True)); fast runs under other bits are refused,
        since the library would build split planes from weights that reached this rank bf16-rounded."""
        torch = self.torch
        self.fast_only = bool(fast_only)
        if fast_only:
            from .distributed import fast_xw_bits
            self.wire_xw = fast_xw_bits() if wire_xw is None else int(wire_xw)
        if flat.device.type != "cuda" or flat.device.index != self.device or flat.dtype != torch.float32:
            raise PfmError(f"load_flat_device: need an f32 tensor on cuda:{self.device}, got {flat.dtype} on {flat.device}")
        flat = flat.contiguous()
        stream = torch.cuda.current_stream(flat.device).cuda_stream
        off = 0
        for k, shp, *_ in layout:
            n = int(np.prod(shp))
            if off + n > flat.numel():
                raise PfmError(f"load_flat_device: buffer of {flat.numel()} floats ends inside {k}")
            shape = (ctypes.c_int64 * len(shp))(*shp)
            check(self.lib.pfm_set_weight_device(self.h, k.encode(), ctypes.c_void_p(flat.data_ptr() + 4 * off),
                                                 PFM_F32, shape, len(shp), ctypes.c_void_p(stream)),
                  f"pfm_set_weight_device({k})")
            off += n
        miss = self.lib.pfm_missing_weights(self.h)
        if strict and miss:
            raise PfmError(f"{miss} required weights missing after load_flat_device")

    @property
    def missing_weights(self) -> int:
        return self.lib.pfm_missing_weights(self.h)

    def reserve(self, B: int, T: int) -> None:
        check(self.lib.pfm_reserve(self.h, int(B), int(T)), "pfm_reserve")

    # ---- live per-kernel-class timing
    def profile(self, enable: bool) -> None:
        check(self.lib.pfm_profile(self.h, 1 if enable else 0), "pfm_profile")

    def profile_read(self, kclass: int) -> dict:
        ms, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        check(self.lib.pfm_profile_read(self.h, int(kclass), ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by),
                                        ctypes.byref(n)), "pfm_profile_read")
        return dict(ms=ms.value, flops=fl.value, bytes=by.value, launches=n.value)

    def _mode(self, mode) -> int:
        m = MODES[mode] if isinstance(mode, str) else int(mode)
        if m == MODE_EXACT and self.fast_only:
            raise PfmError("EXACT mode needs the f32 weights; this engine holds bf16-rounded matrices "
                           "(broadcast_state_dict(wire='bf16') -> load_flat_device(fast_only=True))")
        if self.fast_only and self.wire_xw is not None:
            from .distributed import fast_xw_bits
            if fast_xw_bits() != self.wire_xw:   # the library re-reads PFM_FAST_XW on every call
                raise PfmError(f"PFM_FAST_XW is {fast_xw_bits()} but this engine's weights came over the bf16 wire "
                               f"split for {self.wire_xw}: its split-plane rows would be built from bf16-rounded "
                               "weights (set PFM_FAST_XW back or reload the weights in f32)")
        return m

    # ---- inference
    def run(self, feats, lens, mode="exact", L_cap: Optional[int] = None, want_enc=False, want_alphas=False):
        """feats [B,T,in] f32 cuda, lens [B] int32 cuda -> dict of cuda tensors."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        if feats.device != dev or feats.dtype != torch.float32 or not feats.is_contiguous():
            feats = feats.to(device=dev, dtype=torch.float32).contiguous()
        lens = lens.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        B, T, I = feats.shape
        if I != self.cfg.input_size:
            raise PfmError(f"feature dim {I} != input_size {self.cfg.input_size}")
        if lens.numel() != B:
            raise PfmError("lens must have one entry per utterance")
        L_cap = T + 1 if L_cap is None else int(L_cap)
        tokens = torch.empty((B, max(L_cap, 1)), dtype=torch.int32, device=dev)
        ntok = torch.empty((B,), dtype=torch.int32, device=dev)
        enc = torch.empty((B, T, self.cfg.d_model), dtype=torch.float32, device=dev) if want_enc else None
        alphas = torch.empty((B, T + 1), dtype=torch.float32, device=dev) if want_alphas else None
        peaks = torch.empty((B, T + 1), dtype=torch.float32, device=dev) if want_alphas else None
        m = self._mode(mode)
        check(self.lib.pfm_run(self.h, _stream_ptr(torch, dev), m, _ptr(feats), _ptr(lens), B, T, _ptr(tokens),
                               L_cap, _ptr(ntok), _ptr(enc), _ptr(alphas), _ptr(peaks)), "pfm_run")
        return dict(tokens=tokens, ntok=ntok, enc=enc, alphas=alphas, peaks=peaks)

    def run_beam(self, feats, lens, mode="exact", beam=2, ctc_weight=0.5, penalty=0.0, nbest=1, end_detect=True,
                 L_cap: Optional[int] = None, want_alphas: bool = False):
        """Joint decoder + CTC prefix beam search (pfm_run_beam; Paraformer with a CTC head):
        feats [B,T,in], lens [B] -> dict(tokens [B,nbest,L_cap] int32, ntok [B,nbest] (-1 = none), scores, and with
        want_alphas the CIF alphas / peaks [B,T+1] of the same encoder pass)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        feats = feats.to(device=dev, dtype=torch.float32).contiguous()
        lens = lens.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        B, T, I = feats.shape
        if I != self.cfg.input_size or lens.numel() != B:
            raise PfmError("run_beam: feats [B, T, input_size] and lens [B] expected")
        L_cap = T + 1 if L_cap is None else int(L_cap)
        tokens = torch.empty((B, nbest, max(L_cap, 1)), dtype=torch.int32, device=dev)
        ntok = torch.empty((B, nbest), dtype=torch.int32, device=dev)
        scores = torch.empty((B, nbest), dtype=torch.float32, device=dev)
        alphas = torch.empty((B, T + 1), dtype=torch.float32, device=dev) if want_alphas else None
        peaks = torch.empty((B, T + 1), dtype=torch.float32, device=dev) if want_alphas else None
        m = self._mode(mode)
        c = self.cfg
        check(self.lib.pfm_run_beam(self.h, _stream_ptr(torch, dev), m, _ptr(feats), _ptr(lens), B, T, int(beam),
                                    float(ctc_weight), float(penalty), int(nbest), 1 if end_detect else 0,
                                    int(c.sos), int(c.eos), int(c.blank_id), _ptr(tokens), L_cap, _ptr(ntok),
                                    _ptr(scores), _ptr(alphas), _ptr(peaks)), "pfm_run_beam")
        return dict(tokens=tokens, ntok=ntok, scores=scores, alphas=alphas, peaks=peaks)

    def run_punc(self, ids, lens, mode="exact", want_logits=False):
        """CT-Transformer: word ids [B,T] int32 cuda, lens [B] -> dict(punc [B,T] int32 (-1 beyond lens),
        logits [B,T,classes] on request)."""
        torch = self.torch
        if not isinstance(self.cfg, CTTransformerConfig):
            raise PfmError("run_punc needs a CT-Transformer engine")
        dev = torch.device("cuda", self.device)
        ids = ids.to(device=dev, dtype=torch.int32).contiguous()
        if ids.dim() != 2:
            raise PfmError("ids must be [B, T]")
        lens = lens.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        B, T = ids.shape
        if lens.numel() != B:
            raise PfmError("lens must have one entry per sequence")
        punc = torch.empty((B, T), dtype=torch.int32, device=dev)
        logits = torch.empty((B, T, self.cfg.n_punc), dtype=torch.float32, device=dev) if want_logits else None
        m = self._mode(mode)
        check(self.lib.pfm_run_punc(self.h, _stream_ptr(torch, dev), m, _ptr(ids), _ptr(lens), B, T, _ptr(punc),
                                    _ptr(logits)), "pfm_run_punc")
        return dict(punc=punc, logits=logits)

    def run_punc_host(self, ids: np.ndarray, mode="exact") -> np.ndarray:
        """One word-id sequence (host int32 [n]) -> host labels [n] (pfm_run_punc_host: one C call, pinned staging)."""
        if not isinstance(self.cfg, CTTransformerConfig):
            raise PfmError("run_punc_host needs a CT-Transformer engine")
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.int32).reshape(-1))
        out = np.empty_like(a)
        if a.size == 0:
            return out
        dev = self.torch.device("cuda", self.device)
        check(self.lib.pfm_run_punc_host(self.h, _stream_ptr(self.torch, dev), self._mode(mode), a.ctypes.data,
                                         int(a.size), out.ctypes.data), "pfm_run_punc_host")
        return out

    def run_ctc(self, feats, lens, query, mode="exact", ban_token: int = -1, L_cap: Optional[int] = None,
                want_enc=False, want_frames=False):
        """SenseVoice: feats [B,T,in] f32 cuda, lens [B] int32 cuda, query 4 ints -> dict of cuda tensors
        (tokens [B, L_cap] collapsed CTC ids, ntok [B]; enc [B,T+4,D], frame_ids [B,T+4] on request)."""
        torch = self.torch
        if not isinstance(self.cfg, SenseVoiceConfig):
            raise PfmError("run_ctc needs a SenseVoice engine")
        dev = torch.device("cuda", self.device)
        if feats.device != dev or feats.dtype != torch.float32 or not feats.is_contiguous():
            feats = feats.to(device=dev, dtype=torch.float32).contiguous()
        lens = lens.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        B, T, I = feats.shape
        if I != self.cfg.input_size:
            raise PfmError(f"feature dim {I} != input_size {self.cfg.input_size}")
        if lens.numel() != B:
            raise PfmError("lens must have one entry per utterance")
        q = [int(x) for x in query]
        if len(q) != 4:
            raise PfmError("query must hold 4 embedding ids [language, event, emotion, textnorm]")
        L_cap = T + 4 if L_cap is None else int(L_cap)
        tokens = torch.empty((B, max(L_cap, 1)), dtype=torch.int32, device=dev)
        ntok = torch.empty((B,), dtype=torch.int32, device=dev)
        enc = torch.empty((B, T + 4, self.cfg.d_model), dtype=torch.float32, device=dev) if want_enc else None
        frames = torch.empty((B, T + 4), dtype=torch.int32, device=dev) if want_frames else None
        qa = (ctypes.c_int32 * 4)(*q)
        m = self._mode(mode)
        check(self.lib.pfm_run_ctc(self.h, _stream_ptr(torch, dev), m, _ptr(feats), _ptr(lens), B, T, qa,
                                   int(ban_token), _ptr(tokens), L_cap, _ptr(ntok), _ptr(enc), _ptr(frames)),
              "pfm_run_ctc")
        return dict(tokens=tokens, ntok=ntok, enc=enc, frame_ids=frames)

    def ctc_align(self, enc, olens, targets, blank: int = 0):
        """SenseVoice timestamps' forced alignment (pfm_ctc_align): enc [B, T+4, D] f32 cuda (run_ctc's enc),
        olens [B] (lens + 4), targets: one list of token ids per utterance (token_int[4:]) -> align [B, T] int32
        cuda (label id per speech frame, -1 beyond the utterance)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        enc = enc.to(device=dev, dtype=torch.float32).contiguous()
        B, Tq, _ = enc.shape
        olens = olens.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        Lmax = max([len(t) for t in targets] + [0])
        tg = torch.zeros((B, max(Lmax, 1)), dtype=torch.int32)
        for i, t in enumerate(targets):
            if len(t):
                tg[i, : len(t)] = torch.as_tensor(list(t), dtype=torch.int32)
        tl = torch.as_tensor([len(t) for t in targets], dtype=torch.int32)
        tg, tl = tg.to(dev), tl.to(dev)
        align = torch.empty((B, max(Tq - 4, 1)), dtype=torch.int32, device=dev)
        check(self.lib.pfm_ctc_align(self.h, _stream_ptr(torch, dev), _ptr(enc), B, Tq, _ptr(olens), _ptr(tg), Lmax,
                                     _ptr(tl), int(blank), _ptr(align)), "pfm_ctc_align")
        return align

    def fbank(self, wav, nsamp, cmvn=None):
        """wav [B,S] f32 cuda in [-1,1), nsamp [B] int32 -> (feats [B,T,560], T_out [B])."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        wav = wav.to(device=dev, dtype=torch.float32).contiguous()
        nsamp = nsamp.reshape(-1).to(device=dev, dtype=torch.int32).contiguous()
        B, S = wav.shape
        T_cap = max(1, self.lib.pfm_lfr_frames(int(S)))
        feats = torch.empty((B, T_cap, 560), dtype=torch.float32, device=dev)
        t_out = torch.empty((B,), dtype=torch.int32, device=dev)
        cm = None
        if cmvn is not None:
            cm = torch.as_tensor(np.asarray(cmvn, dtype=np.float32)).to(dev).contiguous()
        check(self.lib.pfm_fbank(self.h, _stream_ptr(torch, dev), _ptr(wav), _ptr(nsamp), B, S, _ptr(cm), _ptr(feats),
                                 T_cap, _ptr(t_out)), "pfm_fbank")
        return feats, t_out

    def fbank_raw(self, wav, nsamp_host):
        """wav [B,S] f32 cuda, nsamp_host: B host ints -> raw fbank frames [B, N_cap, 80] (pfm_fbank_raw)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        wav = wav.to(device=dev, dtype=torch.float32).contiguous()
        B, S = wav.shape
        ns = torch.tensor([int(x) for x in nsamp_host], dtype=torch.int32).to(dev)
        N_cap = max(1, 1 + (S - 400) // 160 if S >= 400 else 1)
        fb = torch.empty((B, N_cap, 80), dtype=torch.float32, device=dev)
        check(self.lib.pfm_fbank_raw(self.h, _stream_ptr(torch, dev), _ptr(wav), _ptr(ns), B, S, _ptr(fb), N_cap),
              "pfm_fbank_raw")
        return fb

    def lfr_gather(self, frames, idx, m, cmvn=None):
        """frames [F,80] f32 cuda, idx [rows, m] host int array -> [rows, m*80] (pfm_lfr_gather)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        idx_h = np.ascontiguousarray(np.asarray(idx, dtype=np.int32).reshape(-1, m))
        rows = idx_h.shape[0]
        out = torch.empty((rows, m * 80), dtype=torch.float32, device=dev)
        if rows:
            if int(idx_h.min()) < 0 or int(idx_h.max()) >= frames.shape[0]:
                raise PfmError("lfr_gather: frame index out of range")
            frames = frames.contiguous()
            idx = torch.from_numpy(idx_h).to(dev)
            check(self.lib.pfm_lfr_gather(_stream_ptr(torch, dev), _ptr(frames), _ptr(idx), rows, m, _ptr(cmvn),
                                          _ptr(out)), "pfm_lfr_gather")
        return out


# ---- single-op helpers (kernel-level parity tests) ------------------------------------------
class PfmStreams:
    """A pfm_streams object: `slots` streaming-Paraformer streams with their chunk caches in HBM
    (ParaformerStreaming.init_cache, paraformer_streaming/model.py:435-466, one per slot)."""

    def __init__(self, engine: PfmEngine, slots: int, chunk_size=(0, 10, 5), encoder_chunk_look_back: int = 0,
                 decoder_chunk_look_back: int = 0, mode="exact"):
        self.engine, self.lib, self.torch = engine, engine.lib, engine.torch
        self.slots = int(slots)
        self.chunk_size = [int(x) for x in chunk_size]
        self.mode = MODES[mode] if isinstance(mode, str) else int(mode)
        cs = (ctypes.c_int32 * 3)(*self.chunk_size)
        h = ctypes.c_void_p()
        check(self.lib.pfm_streams_create(engine.h, self.slots, cs, int(encoder_chunk_look_back),
                                          int(decoder_chunk_look_back), self.mode, ctypes.byref(h)),
              "pfm_streams_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.pfm_streams_destroy(h)
            except Exception:
                pass
            self.h = None

    def reset(self, slot_ids) -> None:
        ids = [int(x) for x in slot_ids]
        arr = (ctypes.c_int32 * max(len(ids), 1))(*ids)
        dev = self.torch.device("cuda", self.engine.device)
        check(self.lib.pfm_streams_reset(self.h, _stream_ptr(self.torch, dev), arr, len(ids)), "pfm_streams_reset")

    def step(self, slot_ids, feats, nfeat, is_final, L_cap: Optional[int] = None, want_enc=False, want_alphas=False):
        """One chunk for len(slot_ids) streams. feats [n, Tn, input_size] f32 cuda (or None when every
        stream is on its tail chunk), nfeat / is_final: n host ints -> dict of cuda tensors."""
        torch = self.torch
        dev = torch.device("cuda", self.engine.device)
        ids = [int(x) for x in slot_ids]
        n = len(ids)
        nf = [int(x) for x in nfeat]
        fin = [1 if x else 0 for x in is_final]
        if len(nf) != n or len(fin) != n:
            raise PfmError("slot_ids, nfeat and is_final must have one entry per stream")
        Tn = 0
        if feats is not None:
            if feats.device != dev or feats.dtype != torch.float32 or not feats.is_contiguous():
                feats = feats.to(device=dev, dtype=torch.float32).contiguous()
            if feats.dim() != 3 or feats.shape[0] != n or feats.shape[2] != self.engine.cfg.input_size:
                raise PfmError(f"feats must be [n, Tn, {self.engine.cfg.input_size}]")
            Tn = feats.shape[1]
        C0 = self.chunk_size[0] + self.chunk_size[2]
        Tw = C0 + max(nf)
        L_cap = Tw + 2 if L_cap is None else int(L_cap)
        tokens = torch.empty((n, max(L_cap, 1)), dtype=torch.int32, device=dev)
        ntok = torch.empty((n,), dtype=torch.int32, device=dev)
        enc = torch.empty((n, Tw, self.engine.cfg.d_model), dtype=torch.float32, device=dev) if want_enc else None
        alphas = torch.empty((n, Tw), dtype=torch.float32, device=dev) if want_alphas else None
        I32 = ctypes.c_int32 * n
        check(self.lib.pfm_stream_step(self.h, _stream_ptr(torch, dev), n, I32(*ids), _ptr(feats), Tn, I32(*nf),
                                       I32(*fin), _ptr(tokens), L_cap, _ptr(ntok), _ptr(enc), _ptr(alphas)),
              "pfm_stream_step")
        return dict(tokens=tokens, ntok=ntok, enc=enc, alphas=alphas)

    def _args(self, slot_ids, feats, nfeat, is_final):
        torch = self.torch
        dev = torch.device("cuda", self.engine.device)
        ids = [int(x) for x in slot_ids]
        n = len(ids)
        nf = [int(x) for x in nfeat]
        fin = [1 if x else 0 for x in is_final]
        if len(nf) != n or len(fin) != n:
            raise PfmError("slot_ids, nfeat and is_final must have one entry per stream")
        Tn = 0
        if feats is not None:
            if feats.device != dev or feats.dtype != torch.float32 or not feats.is_contiguous():
                feats = feats.to(device=dev, dtype=torch.float32).contiguous()
            if feats.dim() != 3 or feats.shape[0] != n or feats.shape[2] != self.engine.cfg.input_size:
                raise PfmError(f"feats must be [n, Tn, {self.engine.cfg.input_size}]")
            Tn = feats.shape[1]
        return dev, ids, n, nf, fin, feats, Tn

    def step_beam(self, slot_ids, feats, nfeat, is_final, beam=2, ctc_weight=0.5, penalty=0.0, nbest=1,
                  end_detect=True, L_cap: Optional[int] = None):
        """One chunk with the joint decoder + CTC prefix beam search per stream (pfm_stream_step_beam,
        paraformer_streaming/model.py:510-521; the model needs its CTC head) -> dict(tokens [n, nbest, L_cap],
        ntok [n, nbest] (-1 = no hypothesis: no CIF fire this chunk), scores [n, nbest], nfire [n])."""
        torch = self.torch
        dev, ids, n, nf, fin, feats, Tn = self._args(slot_ids, feats, nfeat, is_final)
        C0 = self.chunk_size[0] + self.chunk_size[2]
        Tw = C0 + max(nf)
        L_cap = Tw + 2 if L_cap is None else int(L_cap)
        tokens = torch.empty((n, nbest, max(L_cap, 1)), dtype=torch.int32, device=dev)
        ntok = torch.empty((n, nbest), dtype=torch.int32, device=dev)
        scores = torch.empty((n, nbest), dtype=torch.float32, device=dev)
        nfire = torch.empty((n,), dtype=torch.int32, device=dev)
        c = self.engine.cfg
        I32 = ctypes.c_int32 * n
        check(self.lib.pfm_stream_step_beam(self.h, _stream_ptr(torch, dev), n, I32(*ids), _ptr(feats), Tn,
                                            I32(*nf), I32(*fin), int(beam), float(ctc_weight), float(penalty),
                                            int(nbest), 1 if end_detect else 0, int(c.sos), int(c.eos),
                                            int(c.blank_id), _ptr(tokens), L_cap, _ptr(ntok), _ptr(scores),
                                            _ptr(nfire)), "pfm_stream_step_beam")
        return dict(tokens=tokens, ntok=ntok, scores=scores, nfire=nfire)


def op_ln_gemm(X, g, b, eps, W, bias=None, res=None, relu=False, out_bf16=False):
    """bf16(LN(X) g + b) . W^T (+ bias, relu, res): X [M, 512] f32, W [N, 512] bf16 (pfm_op_ln_gemm)."""
    import torch
    lib = load_library()
    M, K = X.shape
    N = W.shape[0]
    if K != 512 or W.shape[1] != 512 or W.dtype != torch.bfloat16:
        raise PfmError("op_ln_gemm: X [M, 512] f32 and W [N, 512] bf16 expected")
    C = torch.empty((M, N), dtype=torch.bfloat16 if out_bf16 else torch.float32, device=X.device)
    act = (1 if relu else 0) | (2 if out_bf16 else 0)
    check(lib.pfm_op_ln_gemm(_stream_ptr(torch, X.device), _ptr(X.contiguous()), _ptr(g), _ptr(b), float(eps),
                             _ptr(W.contiguous()), _ptr(bias), _ptr(res), _ptr(C), M, N, act), "pfm_op_ln_gemm")
    return C


def op_gemm(A, W, bias=None, res=None, relu=False, out_bf16=False):
    """W [N, K], or [2, N, K] bf16 planes (w = w0 + w1: the split-weight GEMM of PFM_FAST_XW)."""
    import torch
    lib = load_library()
    dt = PFM_BF16 if A.dtype == torch.bfloat16 else PFM_F32
    M, K = A.shape
    N = W.shape[-2]
    C = torch.empty((M, N), dtype=torch.bfloat16 if out_bf16 else torch.float32, device=A.device)
    act = (1 if relu else 0) | (2 if out_bf16 else 0) | (4 if W.dim() == 3 else 0)
    check(lib.pfm_op_gemm(_stream_ptr(torch, A.device), dt, _ptr(A.contiguous()), _ptr(W.contiguous()), _ptr(bias),
                          _ptr(res), _ptr(C), M, N, K, act), "pfm_op_gemm")
    return C


def op_ffn(x, g2, b2n, eps, W1, b1, W2, b2, gn=None, bn=None):
    """Fused encoder FFN sub-layer (pfm_op_ffn): x [M,512] f32 -> (x + W2 relu(W1 LN2(x) + b1) + b2,
    LN_next(that) as bf16 or None)."""
    import torch
    lib = load_library()
    M = x.shape[0]
    xo = torch.empty_like(x)
    xn = torch.empty((M, 512), dtype=torch.bfloat16, device=x.device) if gn is not None else None
    check(lib.pfm_op_ffn(_stream_ptr(torch, x.device), _ptr(x.contiguous()), M, _ptr(g2), _ptr(b2n),
                         ctypes.c_float(eps), _ptr(W1.contiguous()), _ptr(b1), _ptr(W2.contiguous()), _ptr(b2),
                         _ptr(xo), _ptr(gn), _ptr(bn), _ptr(xn)), "pfm_op_ffn")
    return xo, xn


def op_ffn_op(o, f, Wo, bo, x, g2, b2n, eps, W1, b1, W2, b2, gn=None, bn=None):
    """Fused encoder sub-layer tail (pfm_op_ffn_op): o, f bf16 [M,512], x f32 [M,512] or None ->
    (x2 = x1 + W2 relu(W1 LN2(x1) + b1) + b2 with x1 = o Wo^T + bo + f (+ x), LN_next(x2) bf16 or None)."""
    import torch
    lib = load_library()
    M = o.shape[0]
    xo = torch.empty((M, 512), dtype=torch.float32, device=o.device)
    xn = torch.empty((M, 512), dtype=torch.bfloat16, device=o.device) if gn is not None else None
    check(lib.pfm_op_ffn_op(_stream_ptr(torch, o.device), _ptr(o.contiguous()), _ptr(f.contiguous()),
                            _ptr(Wo.contiguous()), _ptr(bo), _ptr(x.contiguous() if x is not None else None), M,
                            _ptr(g2), _ptr(b2n), ctypes.c_float(eps), _ptr(W1.contiguous()), _ptr(b1),
                            _ptr(W2.contiguous()), _ptr(b2), _ptr(xo), _ptr(gn), _ptr(bn), _ptr(xn)), "pfm_op_ffn_op")
    return xo, xn


def op_ffn_op_qkv(o, f, Wo, bo, x, g2, b2n, eps, W1, b1, W2, b2, gn, bn, Wq, bq):
    """op_ffn_op plus the next layer's QKV projection in the same launch (pfm_op_ffn_op_qkv, 128-row kernel MODE 4):
    -> (x2 f32 [M,512], qkv = LN_next(x2) Wq^T + bq bf16 [M,1536])."""
    import torch
    lib = load_library()
    M = o.shape[0]
    xo = torch.empty((M, 512), dtype=torch.float32, device=o.device)
    qkv = torch.empty((M, 1536), dtype=torch.bfloat16, device=o.device)
    check(lib.pfm_op_ffn_op_qkv(_stream_ptr(torch, o.device), _ptr(o.contiguous()), _ptr(f.contiguous()),
                                _ptr(Wo.contiguous()), _ptr(bo), _ptr(x.contiguous() if x is not None else None), M,
                                _ptr(g2), _ptr(b2n), ctypes.c_float(eps), _ptr(W1.contiguous()), _ptr(b1),
                                _ptr(W2.contiguous()), _ptr(b2), _ptr(xo), _ptr(gn), _ptr(bn), _ptr(Wq.contiguous()),
                                _ptr(bq), _ptr(qkv)), "pfm_op_ffn_op_qkv")
    return xo, qkv


def op_ffn_dec(x, g1, b1n, eps, W1, b1, W2, gF, bF, gn, bn, o=None, Wo=None, bo=None):
    """Fused decoder FFN (pfm_op_ffn_dec): x f32 [M,512] -> (xo, LN_next(y) bf16) with y = W2 LN_F(relu(W1 LN1(x1)
    + b1)); x1 = x (+ o Wo^T + bo when o is given, then xo = x1), else xo = y."""
    import torch
    lib = load_library()
    M = x.shape[0]
    xo = torch.empty_like(x)
    xn = torch.empty((M, 512), dtype=torch.bfloat16, device=x.device)
    check(lib.pfm_op_ffn_dec(_stream_ptr(torch, x.device), _ptr(x.contiguous()), M, _ptr(g1), _ptr(b1n),
                             ctypes.c_float(eps), _ptr(W1.contiguous()), _ptr(b1), _ptr(W2.contiguous()), _ptr(gF),
                             _ptr(bF), _ptr(xo), _ptr(gn), _ptr(bn), _ptr(xn),
                             _ptr(o.contiguous() if o is not None else None),
                             _ptr(Wo.contiguous() if Wo is not None else None), _ptr(bo)), "pfm_op_ffn_dec")
    return xo, xn


def op_attention(q, k, v, klen, B, Tq, Tk, heads, scale):
    import torch
    lib = load_library()
    dt = PFM_BF16 if q.dtype == torch.bfloat16 else PFM_F32
    out = torch.empty((B * Tq, heads * 128), dtype=torch.float32, device=q.device)
    check(lib.pfm_op_attention(_stream_ptr(torch, q.device), dt, _ptr(q), _ptr(k), _ptr(v),
                               _ptr(klen.to(torch.int32)), _ptr(out), B, Tq, Tk, heads, float(scale)),
          "pfm_op_attention")
    return out


def op_layernorm(x, g, b, eps):
    import torch
    lib = load_library()
    M, D = x.shape
    out = torch.empty_like(x)
    check(lib.pfm_op_layernorm(_stream_ptr(torch, x.device), _ptr(x), _ptr(g), _ptr(b), _ptr(out), M, D, float(eps)),
          "pfm_op_layernorm")
    return out


def op_fsmn(v, lens, w, B, T, left, res=None):
    import torch
    lib = load_library()
    D, K = w.shape[0], w.shape[-1]
    out = torch.empty((B * T, D), dtype=torch.float32, device=v.device)
    check(lib.pfm_op_fsmn(_stream_ptr(torch, v.device), _ptr(v), _ptr(lens.to(torch.int32)),
                          _ptr(w.reshape(D, K).t().contiguous()), _ptr(res), _ptr(out), B, T, D, K, left),
          "pfm_op_fsmn")
    return out


def op_layernorm_bf16(x, g, b, eps):
    """LayerNorm of bf16 rows -> f32 (fast-mode FFN-hidden kernel)."""
    import torch
    lib = load_library()
    M, D = x.shape
    out = torch.empty((M, D), dtype=torch.float32, device=x.device)
    check(lib.pfm_op_layernorm_bf16(_stream_ptr(torch, x.device), _ptr(x.contiguous()), _ptr(g), _ptr(b), _ptr(out),
                                    M, D, ctypes.c_float(eps)), "pfm_op_layernorm_bf16")
    return out


def op_fsmn_bf16(v, lens, w, B, T, left):
    """bf16 v [B*T, D] -> bf16 FSMN memory (fast-mode encoder kernel)."""
    import torch
    lib = load_library()
    D, K = w.shape[0], w.shape[-1]
    out = torch.empty((B * T, D), dtype=torch.bfloat16, device=v.device)
    check(lib.pfm_op_fsmn_bf16(_stream_ptr(torch, v.device), _ptr(v.contiguous()), _ptr(lens.to(torch.int32)),
                               _ptr(w.reshape(D, K).t().contiguous()), _ptr(out), B, T, D, K, left),
          "pfm_op_fsmn_bf16")
    return out


def op_cif(alphas, hidden, L_cap):
    import torch
    lib = load_library()
    B, T1, D = hidden.shape
    emb = torch.empty((B, L_cap, D), dtype=torch.float32, device=hidden.device)
    peaks = torch.empty((B, T1), dtype=torch.float32, device=hidden.device)
    nf = torch.empty((B,), dtype=torch.int32, device=hidden.device)
    nt = torch.empty((B,), dtype=torch.int32, device=hidden.device)
    check(lib.pfm_op_cif(_stream_ptr(torch, hidden.device), _ptr(alphas), _ptr(hidden), _ptr(emb), _ptr(peaks),
                         _ptr(nf), _ptr(nt), B, T1 - 1, D, L_cap), "pfm_op_cif")
    return emb, peaks, nf, nt


def op_ctc_collapse(ids, olen, blank=0, L_cap=None):
    """Greedy CTC collapse of int32 frame ids [B, T] (first olen[b] valid) -> (tokens [B, L_cap], ntok [B])."""
    import torch
    lib = load_library()
    ids = ids.to(torch.int32).contiguous()
    B, T = ids.shape
    L_cap = T if L_cap is None else int(L_cap)
    tokens = torch.empty((B, max(L_cap, 1)), dtype=torch.int32, device=ids.device)
    ntok = torch.empty((B,), dtype=torch.int32, device=ids.device)
    check(lib.pfm_op_ctc_collapse(_stream_ptr(torch, ids.device), _ptr(ids), T, _ptr(olen.to(torch.int32).contiguous()),
                                  B, int(blank), _ptr(tokens), L_cap, _ptr(ntok)), "pfm_op_ctc_collapse")
    return tokens, ntok


def op_ctc_beam(am, x, lens, ntok, beam, ctc_weight, penalty=0.0, nbest=1, sos=1, eos=2, blank=0, end_detect=True,
                L_cap=None):
    """Joint decoder + CTC prefix beam search alone (pfm_op_ctc_beam) on device log-probs am [B, L, V] and
    x [B, T, V] -> (tokens [B, nbest, L_cap], ntok [B, nbest] (-1 = none), scores [B, nbest])."""
    import torch
    lib = load_library()
    am = am.float().contiguous()
    x = x.float().contiguous()
    B, L, V = am.shape
    T = x.shape[1]
    L_cap = L + 1 if L_cap is None else int(L_cap)
    tokens = torch.zeros((B, nbest, max(L_cap, 1)), dtype=torch.int32, device=am.device)
    nt = torch.empty((B, nbest), dtype=torch.int32, device=am.device)
    sc = torch.empty((B, nbest), dtype=torch.float32, device=am.device)
    check(lib.pfm_op_ctc_beam(_stream_ptr(torch, am.device), _ptr(am), L, _ptr(x), T,
                              _ptr(lens.to(torch.int32).contiguous()), _ptr(ntok.to(torch.int32).contiguous()), B, V,
                              int(beam), float(ctc_weight), float(penalty), int(nbest), 1 if end_detect else 0,
                              int(sos), int(eos), int(blank), _ptr(tokens), L_cap, _ptr(nt), _ptr(sc)),
          "pfm_op_ctc_beam")
    return tokens, nt, sc


class PfmVad:
    """A pfm_vad object: the FSMN-VAD encoder of one stream (memory caches in HBM) on one device."""

    def __init__(self, cfg, device: int = 0):   # FsmnVADConfig
        import torch
        if not torch.cuda.is_available():
            raise PfmError("PfmVad needs a ROCm GPU; there is no CPU fallback")
        self.torch, self.cfg, self.device = torch, cfg, int(device)
        self.lib = load_library()
        c = PfmVadConfig(cfg.input_dim, cfg.input_affine_dim, cfg.fsmn_layers, cfg.linear_dim, cfg.proj_dim,
                         cfg.lorder, cfg.output_affine_dim, cfg.output_dim)
        h = ctypes.c_void_p()
        check(self.lib.pfm_vad_create(ctypes.byref(c), self.device, ctypes.byref(h)), "pfm_vad_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.pfm_vad_destroy(h)
            except Exception:
                pass
            self.h = None

    @property
    def missing_weights(self) -> int:
        return int(self.lib.pfm_vad_missing_weights(self.h))

    def load_state_dict(self, sd):
        for k, v in sd.items():
            a = v.detach().cpu().float().numpy() if hasattr(v, "detach") else np.asarray(v, np.float32)
            a = np.ascontiguousarray(a, dtype=np.float32)
            shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
            check(self.lib.pfm_vad_set_weight(self.h, k.encode(), a.ctypes.data, PFM_F32, shape, a.ndim),
                  f"pfm_vad_set_weight({k})")

    def reset(self):
        dev = self.torch.device("cuda", self.device)
        check(self.lib.pfm_vad_reset(self.h, _stream_ptr(self.torch, dev)), "pfm_vad_reset")

    def frame_energy(self, wav, frame_len: int = 400, frame_shift: int = 160) -> np.ndarray:
        """ComputeDecibel's per-frame energies of a host waveform chunk (pfm_vad_frame_energy: numpy's float32 pairwise
        sum of the squared samples, bit for bit) -> host f32 [frames]."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        w = np.ascontiguousarray(np.asarray(wav, np.float32).reshape(-1))
        n = w.shape[0]
        nf = (n - frame_len) // frame_shift + 1 if n >= frame_len else 0
        if nf <= 0:
            return np.zeros((0,), np.float32)
        wd = torch.from_numpy(w).to(dev)
        e = torch.empty((nf,), dtype=torch.float32, device=dev)
        check(self.lib.pfm_vad_frame_energy(self.h, _stream_ptr(torch, dev), _ptr(wd), n, frame_len, frame_shift, _ptr(e)),
              "pfm_vad_frame_energy")
        return e.cpu().numpy()

    def fbank_raw(self, wav, nsamp_host):
        """Raw fbank frames [B, N_cap, 80] of the VAD's online frontend (pfm_vad_fbank_raw)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        wav = wav.to(device=dev, dtype=torch.float32).contiguous()
        B, S = wav.shape
        ns = torch.tensor([int(x) for x in nsamp_host], dtype=torch.int32).to(dev)
        N_cap = max(1, 1 + (S - 400) // 160 if S >= 400 else 1)
        fb = torch.empty((B, N_cap, 80), dtype=torch.float32, device=dev)
        check(self.lib.pfm_vad_fbank_raw(self.h, _stream_ptr(torch, dev), _ptr(wav), _ptr(ns), B, S, _ptr(fb), N_cap),
              "pfm_vad_fbank_raw")
        return fb

    lfr_gather = PfmEngine.lfr_gather

    def run(self, feats, want_probs=False):
        """feats [T, input_dim] f32 cuda -> p_sil [T] cuda (and probs [T, output_dim] on request)."""
        torch = self.torch
        dev = torch.device("cuda", self.device)
        feats = feats.to(device=dev, dtype=torch.float32).contiguous()
        if feats.dim() != 2 or feats.shape[1] != self.cfg.input_dim:
            raise PfmError(f"feats must be [T, {self.cfg.input_dim}]")
        T = feats.shape[0]
        p = torch.empty((T,), dtype=torch.float32, device=dev)
        probs = torch.empty((T, self.cfg.output_dim), dtype=torch.float32, device=dev) if want_probs else None
        check(self.lib.pfm_vad_run(self.h, _stream_ptr(torch, dev), _ptr(feats), T, _ptr(p), _ptr(probs)),
              "pfm_vad_run")
        return (p, probs) if want_probs else p


class PfmVadDetector:
    """pfm_vad_detector: the VAD decision state machine of one stream, native host code (no GPU)."""

    def __init__(self, opts: Dict):
        self.lib = load_library()
        o = PfmVadOpts()
        for name, _ in PfmVadOpts._fields_:
            v = opts[name]
            setattr(o, name, float(v) if isinstance(getattr(o, name), float) else int(v))
        h = ctypes.c_void_p()
        check(self.lib.pfm_vad_detector_create(ctypes.byref(o), ctypes.byref(h)), "pfm_vad_detector_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.pfm_vad_detector_destroy(h)
            except Exception:
                pass
            self.h = None

    def push(self, decibel, p_sil, is_final: bool, streaming: bool):
        """One forward() call: the call's frame decibels and posteriors -> the segments it outputs."""
        db = np.ascontiguousarray(decibel, dtype=np.float64)
        ps = np.ascontiguousarray(p_sil, dtype=np.float32)
        self.frames = getattr(self, "frames", 0) + int(ps.size)
        cap = self.frames + 16   # every segment covers >= 1 frame: never more segments than frames
        segs = np.zeros((cap, 2), np.int32)
        n = ctypes.c_int32(0)
        check(self.lib.pfm_vad_detector_push(self.h, db.ctypes.data if db.size else None, int(db.size),
                                             ps.ctypes.data if ps.size else None, int(ps.size), int(is_final),
                                             int(streaming), segs.ctypes.data, cap, ctypes.byref(n)),
              "pfm_vad_detector_push")
        return segs[: n.value].tolist()
