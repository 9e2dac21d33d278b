"""`Paraformer` model class with the reference's plugin contract, backed by libpfm_hip.so.

Contract (funasr/auto/auto_model.py:260-288, funasr/models/paraformer/model.py:443-596):
  * constructed as cls(**model_conf, encoder_conf=..., decoder_conf=..., predictor_conf=...,
    input_size=560, vocab_size=V, **AutoModel kwargs);
  * an nn.Module with >= 1 parameter (AutoModel reads next(model.parameters()).device);
  * state_dict() / load_state_dict() speak the reference state_dict keys and shapes, so
    load_pretrained_model (funasr/train_utils/load_pretrained_model.py:14-47) and this
    package's loader both work unchanged;
  * inference(data_in, data_lengths=None, key=None, tokenizer=None, frontend=None, **kwargs)
    -> (results, meta) with results [{"key", "text"}] or [{"key", "token_int"}] when
    tokenizer is None; meta has load_data / extract_feat / batch_data_time.
All compute runs in the HIP library; there is no CPU/PyTorch fallback.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .config import ParaformerConfig
from .register import tables
from .runtime import PfmEngine, PfmError
from .writer import model_writer
from .text import sentence_postprocess
from .timestamp import ts_prediction_lfr6_standard
from .weights import param_layout


def _as_hip_frontend(frontend):
    """Accept the reference's WavFrontend (plugin route: reference AutoModel builds it) by taking
    its CMVN over into the HIP frontend; the fbank itself always runs in k_fbank.hip."""
    from .frontend import WavFrontend
    if isinstance(frontend, WavFrontend):
        return frontend
    fe = WavFrontend(cmvn_file=None)
    cm = getattr(frontend, "cmvn", None)
    if cm is not None:
        fe.cmvn = np.asarray(cm.detach().cpu().numpy() if hasattr(cm, "detach") else cm, dtype=np.float32)
    return fe


class HipModel(torch.nn.Module):
    """Shared plugin contract of the HIP-backed model classes: reference state_dict keys and shapes,
    a device anchor parameter, one PfmEngine (C-ABI handle) per device. Subclasses set `self.cfg`."""

    family = "model"

    def _init_common(self, kwargs):
        self.mode = kwargs.get("mode", "exact")
        # device anchor: AutoModel and callers read next(model.parameters()).device
        self._anchor = torch.nn.Parameter(torch.zeros(1), requires_grad=False)
        self._host_sd: Dict[str, np.ndarray] = {}
        self._engine: Optional[PfmEngine] = None
        self._engine_dev: Optional[int] = None

    # ---------------- weights (reference key names) ----------------
    def state_dict(self, *args, **kwargs):
        out = {}
        for k, shape, _ in param_layout(self.cfg):
            v = self._host_sd.get(k)
            out[k] = torch.from_numpy(v) if v is not None else torch.zeros(shape)
        return out

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        want = {k: s for k, s, _ in param_layout(self.cfg)}
        missing = [k for k in want if k not in state_dict]
        unexpected = [k for k in state_dict if k not in want]
        if "ctc.ctc_lo.weight" in unexpected and getattr(self.cfg, "ctc_weight", None) == 0.0:
            # the reference builds ctc.ctc_lo whenever model_conf.ctc_weight > 0 (its constructor default is 0.5,
            # paraformer/model.py:51, 95-100); a config that leaves ctc_weight out would drop the head here
            msg = (f"{type(self).__name__}: the checkpoint carries a CTC head (ctc.ctc_lo) but the model was built "
                   "with ctc_weight 0.0; set model_conf.ctc_weight > 0 (the reference default is 0.5) to keep it")
            if strict:
                raise RuntimeError(msg)
            import warnings
            warnings.warn(msg)
        if strict and (missing or unexpected):
            raise RuntimeError(f"{type(self).__name__}.load_state_dict: missing {missing[:5]} "
                               f"unexpected {unexpected[:5]}")
        for k, v in state_dict.items():
            if k not in want:
                continue
            a = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32)
            if tuple(a.shape) != tuple(want[k]):
                raise RuntimeError(f"{k}: shape {a.shape} != {want[k]}")
            self._host_sd[k] = np.ascontiguousarray(a, dtype=np.float32)
            if self._engine is not None:
                self._engine.set_weight(k, self._host_sd[k])
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    # ---------------- device / engine ----------------
    def _device_index(self) -> int:
        d = self._anchor.device
        if d.type != "cuda":
            if not torch.cuda.is_available():
                raise PfmError(f"{type(self).__name__} (HIP) needs a ROCm GPU; there is no CPU path in this build")
            return torch.cuda.current_device()
        return d.index if d.index is not None else torch.cuda.current_device()

    def engine(self) -> PfmEngine:
        dev = self._device_index()
        if self._engine is None or self._engine_dev != dev:
            eng = PfmEngine(self.cfg, dev)
            if self._host_sd:
                eng.load_state_dict(self._host_sd, strict=False)
            self._engine, self._engine_dev = eng, dev
        if self._engine.missing_weights:
            raise PfmError(f"{self._engine.missing_weights} {type(self).__name__} weights not loaded "
                           "(load_state_dict / init_param)")
        return self._engine

    # ---------------- shared input handling (model.py:452-493 / sense_voice/model.py:819-846) -------------
    def _speech(self, eng, data_in, data_lengths, frontend, kwargs, meta):
        """fbank tensor or waveforms -> (feats [B,T,560] on the device, lens [B])."""
        if isinstance(data_in, torch.Tensor) and kwargs.get("data_type", "sound") == "fbank":
            speech = data_in if data_in.dim() == 3 else data_in[None]
            if data_lengths is None:
                lens = torch.full((speech.shape[0],), speech.shape[1], dtype=torch.int32)
            else:
                lens = torch.as_tensor(data_lengths).reshape(-1)
            return speech, lens
        if frontend is None:
            raise ValueError("waveform input needs a frontend (frontend_conf)")
        frontend = _as_hip_frontend(frontend)
        items = data_in if isinstance(data_in, (list, tuple)) else [data_in]
        t1 = time.perf_counter()
        speech, lens, _ = frontend(eng, items)
        torch.cuda.synchronize(speech.device)
        t2 = time.perf_counter()
        meta["load_data"] = "0.000"
        meta["extract_feat"] = f"{t2 - t1:0.3f}"
        meta["batch_data_time"] = float(lens.sum().item()) * frontend.frame_shift * frontend.lfr_n / 1000
        return speech, lens

    @staticmethod
    def _keys(key, b):
        if key is None:
            key = [f"utt{i}" for i in range(b)]
        if isinstance(key[0], (list, tuple)):
            key = key[0]
        if len(key) < b:
            key = key * b
        return key


@tables.register("model_classes", "Paraformer")
class Paraformer(HipModel):
    family = "paraformer"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.cfg = ParaformerConfig.from_kwargs(**kwargs)
        self.blank_id, self.sos, self.eos = self.cfg.blank_id, self.cfg.sos, self.cfg.eos
        self._init_common(kwargs)

    def _greedy_hyps(self, toks, ntok):
        """[B, L_cap] per-position argmax ids + counts -> per utterance a one-entry n-best list of token ids with
        blank / sos / eos dropped (model.py:541-565)."""
        toks, ntok = np.asarray(toks), np.asarray(ntok).reshape(-1)
        n = np.where(ntok <= toks.shape[1], ntok, 0)   # a count past L_cap: the row was not decoded (empty result)
        keep = np.arange(toks.shape[1])[None, :] < n[:, None]
        for sp in (self.eos, self.sos, self.blank_id):
            keep &= toks != sp
        return [[toks[i][keep[i]].tolist()] for i in range(toks.shape[0])]

    def results_from_token_matrix(self, toks, ntok, key, tokenizer=None, **kwargs):
        """Greedy results from a (gathered) host token matrix, exactly as inference() builds them."""
        if tokenizer is not None and hasattr(tokenizer, "postprocessed_texts_matrix"):
            texts = tokenizer.postprocessed_texts_matrix(toks, ntok, (self.eos, self.sos, self.blank_id))
            key = self._keys(key, len(texts))
            return [{"key": key[i], "text": t} for i, t in enumerate(texts)]
        hyps = self._greedy_hyps(toks, ntok)
        key = self._keys(key, len(hyps))
        if tokenizer is not None and hasattr(tokenizer, "postprocessed_texts"):
            return [{"key": key[i], "text": t} for i, t in
                    enumerate(tokenizer.postprocessed_texts([hl[0] for hl in hyps]))]
        out = []
        for i, hl in enumerate(hyps):
            ids = hl[0]
            if tokenizer is None:
                out.append({"key": key[i], "token_int": ids})
                continue
            toks_i = tokenizer.ids2tokens(ids)
            if hasattr(tokenizer, "bpemodel"):
                text = tokenizer.tokens2text(toks_i)
            else:
                text, _ = sentence_postprocess(toks_i)
            out.append({"key": key[i], "text": text})
        return out

    # ---------------- inference (paraformer/model.py:443-596) ----------------
    @torch.no_grad()
    def inference(self, data_in, data_lengths=None, key: List[str] = None, tokenizer=None, frontend=None,
                  **kwargs):
        # paraformer/model.py:443-458: beam search when decoding_ctc_weight > 1e-5 and the model has a CTC head
        # (otherwise the reference's is_use_ctc is False and it decodes greedily); LM fusion needs an LM scorer the
        # reference does not build either (init_beam_search: "ngram is not supported now")
        if kwargs.get("lm_weight", 0.0) > 1e-5 and kwargs.get("lm_file") is not None:
            raise NotImplementedError("LM shallow fusion (lm_file) is not on the HIP Paraformer path")
        use_ctc = kwargs.get("decoding_ctc_weight", 0.0) > 1e-5 and self.cfg.ctc_weight > 0.0
        if kwargs.get("decoding_ctc_weight", 0.0) > 1e-5 and not use_ctc:
            import warnings   # the reference decodes greedily too when self.ctc is None (model.py:443-458)
            warnings.warn("decoding_ctc_weight > 0 on a Paraformer without a CTC head (ctc_weight 0.0): greedy "
                          "decoding, as the reference does when the model has no ctc module")
        eng = self.engine()
        mode = kwargs.get("mode", self.mode)
        meta = {}
        speech, lens = self._speech(eng, data_in, data_lengths, frontend, kwargs, meta)
        pred_ts = bool(kwargs.get("pred_timestamp", False))
        if use_ctc:   # joint decoder + CTC prefix beam search on the device (pfm_run_beam)
            nbest = int(kwargs.get("nbest", 1))
            # the kernel's n-best list holds up to 16 ended hypotheses (sorted(ended_hyps)[:nbest], model.py:553)
            if not 1 <= nbest <= 16:
                raise PfmError(f"nbest {nbest}: the HIP beam search keeps at most 16 ended hypotheses")
            r = eng.run_beam(speech, lens, mode=mode, beam=int(kwargs.get("beam_size", 2)),
                             ctc_weight=float(kwargs["decoding_ctc_weight"]), penalty=float(kwargs.get("penalty", 0.0)),
                             nbest=nbest, end_detect=float(kwargs.get("maxlenratio", 0.0)) == 0.0,
                             want_alphas=pred_ts)   # with timestamps: the CIF outputs of the same encoder pass
            btok, bn = r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy()
            hyps = [[btok[i, k, :bn[i, k]].tolist() for k in range(nbest) if bn[i, k] >= 0]
                    for i in range(btok.shape[0])]
        else:
            r = eng.run(speech, lens, mode=mode, want_alphas=pred_ts)
            if not pred_ts and kwargs.get("output_dir") is None:
                # greedy text / token_int results are a function of the device token matrix alone: a data-parallel
                # caller may gather the matrices across ranks as tensors and build the results afterwards
                meta["token_matrix"] = (r["tokens"], r["ntok"])
            toks = r["tokens"].cpu().numpy()           # one device->host copy for the whole batch
            ntok = r["ntok"].cpu().numpy()
            if (tokenizer is not None and not pred_ts and kwargs.get("output_dir") is None and
                    hasattr(tokenizer, "postprocessed_texts_matrix")):
                # text results only: detokenised from the matrix itself (no per-utterance id lists)
                texts = tokenizer.postprocessed_texts_matrix(toks, ntok, (self.eos, self.sos, self.blank_id))
                key = self._keys(key, len(texts))
                meta["owner"] = list(range(len(texts)))
                return [{"key": key[i], "text": t} for i, t in enumerate(texts)], meta
            hyps = self._greedy_hyps(toks, ntok)
        if pred_ts:   # CIF outputs for ts_prediction_lfr6_standard (paraformer/model.py:572-582)
            peaks_h, alphas_h = r["peaks"].cpu(), r["alphas"].cpu()
        b = len(hyps)
        key = self._keys(key, b)
        results = []
        owner = []   # batch index of each result (n-best gives several per utterance, an unfinished search none)
        writer = model_writer(self, kwargs)   # output_dir: {n}best_recog/{token,text} (model.py:548-552, 588-591)
        # the texts of a character tokenizer in one vectorised pass (CharTokenizer.postprocessed_texts)
        fast_txt = None
        if tokenizer is not None and not pred_ts and hasattr(tokenizer, "postprocessed_texts"):
            fast_txt = iter(tokenizer.postprocessed_texts([ids for i in range(b) for ids in hyps[i]]))
        for i in range(b):
            for nb, ids in enumerate(hyps[i]):   # n-best hypotheses of utterance i, best first (model.py:553)
                owner.append(i)
                if fast_txt is not None:
                    text = next(fast_txt)
                    results.append({"key": key[i], "text": text})
                    if writer is not None:
                        writer[f"{nb + 1}best_recog"]["token"][key[i]] = " ".join(tokenizer.ids2tokens(ids))
                        writer[f"{nb + 1}best_recog"]["text"][key[i]] = text
                    continue
                if tokenizer is not None:
                    # model.py:567-586: text = tokens2text(ids2tokens(ids)); sentence_postprocess replaces it
                    # only for tokenizers without a `bpemodel` (a SentencepiecesTokenizer keeps tokens2text)
                    toks_i = tokenizer.ids2tokens(ids)
                    bpe = hasattr(tokenizer, "bpemodel")
                    # (without a bpemodel sentence_postprocess replaces the tokens2text result: not computed then)
                    text = tokenizer.tokens2text(toks_i) if bpe else None
                    if pred_ts:
                        if bpe:   # model.py:580-582 reads time_stamp_postprocessed, which only the non-bpe branch binds
                            raise UnboundLocalError("pred_timestamp with a bpemodel tokenizer: the reference leaves "
                                                    "time_stamp_postprocessed unbound (paraformer/model.py:580-582)")
                        # the reference passes the CIF peaks as `us_alphas` and the alphas as `us_peaks`
                        _, ts = ts_prediction_lfr6_standard(peaks_h[i], alphas_h[i], list(toks_i),
                                                            vad_offset=kwargs.get("begin_time", 0), upsample_rate=1)
                        text, ts_pp, _ = sentence_postprocess(toks_i, ts)
                        results.append({"key": key[i], "text": text, "timestamp": ts_pp})
                    else:
                        if not bpe:
                            text, _ = sentence_postprocess(toks_i)
                        results.append({"key": key[i], "text": text})
                    if writer is not None:
                        writer[f"{nb + 1}best_recog"]["token"][key[i]] = " ".join(toks_i)
                        writer[f"{nb + 1}best_recog"]["text"][key[i]] = text
                else:
                    results.append({"key": key[i], "token_int": ids})
        meta["owner"] = owner
        return results, meta
