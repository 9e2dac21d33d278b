"""`ParaformerStreaming` model class with the reference's plugin contract, backed by libpfm_hip.so.

Contract (funasr/models/paraformer_streaming/model.py:435-656):
  * registered as tables.model_classes["ParaformerStreaming"]; constructed like Paraformer with
    encoder "SANMEncoderChunkOpt" and the causal decoder FSMN (decoder_conf sanm_shfit 5);
  * inference(data_in, data_lengths=None, key=None, tokenizer=None, frontend=None, cache={}, **kwargs)
    with kwargs is_final, chunk_size ([0, 10, 5]), encoder_chunk_look_back, decoder_chunk_look_back:
    the caller's `cache` dict carries the stream between calls exactly as the reference's does
    (init_cache on first use and after is_final, prev_samples, 600 ms sample chunks, the tail chunk);
    results [{"key", "text"}] (text = sentence_postprocess of this call's tokens), or
    [{"key", "token_int"}] with tokenizer None.
  * decoding_ctc_weight > 0 on a model with a CTC head (model_conf ctc_weight > 0) runs the joint decoder + CTC
    prefix beam search per chunk (model.py:510-521, 567-575; pfm_stream_step_beam), beam_size / nbest / penalty /
    maxlenratio as the reference's kwargs; the chunk's tokens are those of every n-best hypothesis in order;
  * `inference_streams(...)` advances many streams by one call each in a single batched pass — the
    serving entry point (the reference is batch 1, model.py:598).
The per-stream state lives in HBM inside a pfm_streams object (one slot per live cache dict); the
chunk encoder, CIF, decoder, argmax (pfm_stream_step) and the online frontend (pfm_fbank_raw +
pfm_lfr_gather) run in the HIP library. There is no CPU path.
"""
from __future__ import annotations

import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .config import ParaformerStreamingConfig
from .frontend import WavFrontendOnline
from .model import HipModel
from .register import tables
from .runtime import PfmError, PfmStreams
from .text import sentence_postprocess
from .writer import model_writer

CHUNK_SAMPLES_PER_FRAME = 960   # model.py:582: chunk_size[1] * 960 samples (60 ms per LFR frame)


class _Slot:
    """Lease of one pfm_streams slot, held in the caller's cache dict; returned to the pool when the
    cache dict (and so this lease) is dropped."""

    def __init__(self, pool: "_SlotPool", idx: int):
        self.idx = idx
        self._fin = weakref.finalize(self, pool._release, idx)


class _SlotPool:
    def __init__(self, streams: PfmStreams):
        self.streams = streams
        self.free = list(range(streams.slots))[::-1]

    def _release(self, idx):
        self.free.append(idx)

    def acquire(self) -> _Slot:
        if not self.free:
            raise PfmError(f"all {self.streams.slots} stream slots are in use (raise max_streams)")
        idx = self.free.pop()
        self.streams.reset([idx])
        return _Slot(self, idx)


@tables.register("model_classes", "ParaformerStreaming")
class ParaformerStreaming(HipModel):
    family = "paraformer_streaming"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.cfg = ParaformerStreamingConfig.from_kwargs(**kwargs)
        self.blank_id, self.sos, self.eos = self.cfg.blank_id, self.cfg.sos, self.cfg.eos
        self.max_streams = int(kwargs.get("max_streams", 64))
        self._pools: Dict[tuple, _SlotPool] = {}
        self._init_common(kwargs)

    # ---------------- caches (init_cache, model.py:435-466) ----------------
    def _pool(self, chunk_size, elb, dlb, mode) -> _SlotPool:
        eng = self.engine()
        k = (tuple(int(x) for x in chunk_size), int(elb), int(dlb), mode, eng.device)
        if k not in self._pools:
            self._pools[k] = _SlotPool(PfmStreams(eng, self.max_streams, k[0], elb, dlb, mode))
        return self._pools[k]

    def init_cache(self, cache: dict, **kwargs) -> dict:
        chunk_size = list(kwargs.get("chunk_size", [0, 10, 5]))
        elb = int(kwargs.get("encoder_chunk_look_back", 0))
        dlb = int(kwargs.get("decoder_chunk_look_back", 0))
        mode = kwargs.get("mode", self.mode)
        pool = self._pool(chunk_size, elb, dlb, mode)
        slot = cache.get("slot")
        if slot is not None and cache.get("pool") is pool:
            pool.streams.reset([slot.idx])          # re-init after is_final keeps the lease
        else:
            slot = pool.acquire()
        cache.clear()
        cache.update(pool=pool, slot=slot, chunk_size=chunk_size, frontend={},
                     prev_samples=np.zeros((0,), np.float32), tail_chunk=False)
        return cache

    @staticmethod
    def _audio(data_in) -> np.ndarray:
        x = data_in[0] if isinstance(data_in, (list, tuple)) else data_in
        if isinstance(x, str):
            from .frontend import read_wav
            return read_wav(x)
        if hasattr(x, "detach"):
            x = x.detach().cpu().numpy()
        return np.asarray(x, dtype=np.float32).reshape(-1)

    # ---------------- batched stream advance ----------------
    @torch.no_grad()
    def inference_streams(self, calls: Sequence[Tuple[object, dict, bool]], tokenizer=None, frontend=None,
                          **kwargs) -> List[list]:
        """calls: (audio samples, cache dict, is_final) per stream -> per stream the tokens of this call
        (token strings with a tokenizer, else ids). Each stream is cut into 600 ms chunks as in
        inference() (model.py:591-642); chunk j of every stream runs in the same pfm_stream_step."""
        if kwargs.get("lm_weight", 0.0) > 1e-5 and kwargs.get("lm_file") is not None:
            raise NotImplementedError("LM shallow fusion (lm_file) is not on the HIP streaming path")
        # model.py:567-575: the joint decoder + CTC prefix beam search when decoding_ctc_weight > 1e-5 and the
        # model has a CTC head (model_conf ctc_weight > 0); the released model has none and decodes greedily
        beam = None
        if kwargs.get("decoding_ctc_weight", 0.0) > 1e-5:
            if self.cfg.ctc_weight > 0.0:
                nbest = int(kwargs.get("nbest", 1))
                if not 1 <= nbest <= 16:
                    raise PfmError(f"nbest {nbest}: the HIP beam search keeps at most 16 ended hypotheses")
                beam = dict(beam=int(kwargs.get("beam_size", 2)), ctc_weight=float(kwargs["decoding_ctc_weight"]),
                            penalty=float(kwargs.get("penalty", 0.0)), nbest=nbest,
                            end_detect=float(kwargs.get("maxlenratio", 0.0)) == 0.0)
            else:
                import warnings
                warnings.warn("decoding_ctc_weight > 0 on a ParaformerStreaming without a CTC head (ctc_weight 0.0): "
                              "greedy decoding, as the reference does when the model has no ctc module")
        fe = frontend if isinstance(frontend, WavFrontendOnline) else self._default_frontend(frontend)
        eng = self.engine()
        plans = []
        for audio, cache, is_final in calls:
            if len(cache) == 0 or "slot" not in cache:
                self.init_cache(cache, **kwargs)
            cs = cache["chunk_size"]
            stride = int(cs[1] * CHUNK_SAMPLES_PER_FRAME)
            a = np.concatenate([cache["prev_samples"], self._audio(audio)])
            n = int(len(a) // stride + int(is_final))
            m = int(len(a) % stride * (1 - int(is_final)))
            plans.append((a, n, m, stride, cache, bool(is_final)))
        out: List[list] = [[] for _ in calls]
        dev = torch.device("cuda", eng.device)
        for j in range(max((p[1] for p in plans), default=0)):
            act = [k for k, p in enumerate(plans) if j < p[1]]
            by_pool: Dict[int, List[int]] = {}
            for k in act:
                by_pool.setdefault(id(plans[k][4]["pool"]), []).append(k)
            for ks in by_pool.values():
                pool = plans[ks[0]][4]["pool"]
                fe_items, fe_ks, rows = [], [], {}
                for k in ks:
                    a, n, _, stride, cache, fin = plans[k]
                    seg = a[j * stride:(j + 1) * stride]
                    last = fin and j == n - 1
                    if last and len(seg) < CHUNK_SAMPLES_PER_FRAME:
                        cache["tail_chunk"] = True       # model.py:601-607: encoder over the overlap only
                        rows[k] = None
                    else:
                        fe_items.append((seg, last, cache["frontend"]))
                        fe_ks.append(k)
                for k, f in zip(fe_ks, fe.step(eng, fe_items) if fe_items else []):
                    rows[k] = f
                run = [k for k in ks if rows[k] is None or rows[k].shape[0] > 0]
                if not run:
                    continue
                nf = [0 if rows[k] is None else int(rows[k].shape[0]) for k in run]
                Tn = max(nf)
                feats = None
                if Tn:
                    feats = torch.zeros((len(run), Tn, self.cfg.input_size), dtype=torch.float32, device=dev)
                    for i, k in enumerate(run):
                        if nf[i]:
                            feats[i, : nf[i]] = rows[k]
                fins = [plans[k][5] and j == plans[k][1] - 1 for k in run]
                slots = [plans[k][4]["slot"].idx for k in run]
                if beam is None:
                    r = pool.streams.step(slots, feats, nf, fins)
                    toks = r["tokens"].cpu().numpy()
                    ntok = r["ntok"].cpu().numpy()
                    hyps = [[[t for t in toks[i, : int(ntok[i])].tolist() if t not in (self.eos, self.sos, self.blank_id)]]
                            for i in range(len(run))]
                else:   # model.py:530-552: the tokens of every n-best hypothesis, concatenated
                    r = pool.streams.step_beam(slots, feats, nf, fins, **beam)
                    toks = r["tokens"].cpu().numpy()
                    ntok = r["ntok"].cpu().numpy()
                    hyps = [[toks[i, q, : int(ntok[i, q])].tolist() for q in range(toks.shape[1]) if ntok[i, q] >= 0]
                            for i in range(len(run))]
                for i, k in enumerate(run):
                    for ids in hyps[i]:
                        out[k].extend(tokenizer.ids2tokens(ids) if tokenizer is not None else ids)
        for a, n, m, stride, cache, fin in plans:
            cache["prev_samples"] = a[:-m] if m else a[:0]    # model.py:646 (keeps audio[:-m], as the reference)
            if fin:
                self.init_cache(cache, chunk_size=cache["chunk_size"], **{k: v for k, v in kwargs.items()
                                                                           if k != "chunk_size"})
        return out

    def _default_frontend(self, frontend):
        fe = WavFrontendOnline(cmvn_file=None)
        cm = getattr(frontend, "cmvn", None)
        if cm is not None:
            fe.cmvn = np.asarray(cm.detach().cpu().numpy() if hasattr(cm, "detach") else cm, dtype=np.float32)
        if not hasattr(self, "_fe_cache"):
            self._fe_cache = {}
        key = id(frontend)
        if key not in self._fe_cache:
            self._fe_cache[key] = fe
        return self._fe_cache[key]

    # ---------------- inference (model.py:556-656) ----------------
    @torch.no_grad()
    def inference(self, data_in, data_lengths=None, key: List[str] = None, tokenizer=None, frontend=None,
                  cache: Optional[dict] = None, **kwargs):
        if cache is None:
            cache = {}
        is_final = bool(kwargs.pop("is_final", False))
        if isinstance(data_in, (list, tuple)) and len(data_in) != 1:
            raise AssertionError("batch_size must be set 1")   # model.py:587 (use inference_streams to batch)
        if isinstance(data_in, str):
            is_final = True                                      # a file input is a whole stream (load_utils)
        tokens = self.inference_streams([(data_in, cache, is_final)], tokenizer=tokenizer, frontend=frontend,
                                        **kwargs)[0]
        key = self._keys(key, 1)
        if tokenizer is None:
            return [{"key": key[0], "token_int": tokens}], {}
        text, _ = sentence_postprocess(tokens)
        if kwargs.get("output_dir"):   # paraformer_streaming/model.py:649-654
            writer = model_writer(self, kwargs)
            writer["1best_recog"]["token"][key[0]] = " ".join(tokens)
            writer["1best_recog"]["text"][key[0]] = text
        return [{"key": key[0], "text": text}], {}
