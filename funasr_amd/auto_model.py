"""AutoModel with the reference's generate()/inference() contract over the HIP Paraformer path.

Mirrors funasr/auto/auto_model.py:
  prepare_data_iterator   :40-108   input forms -> (keys, items)
  AutoModel.__init__      :113, build_model :176-293  (local model dir: config.yaml + model.pt +
                                     tokens.json + am.mvn merge, download_model_from_hub.py:60-79)
  generate / inference    :301-376  batch loop, batch_size, fbank single-tensor batch (:339-341),
                                     speed stats, results in input order
Differences (by design): device defaults to the GPU and there is no CPU path; hub names are
not fetched (no network); VAD/punctuation/speaker pipelines are not built.
Multi-GPU: when torch.distributed is initialised with world > 1, inference() deals the
utterances over ranks longest-first (funasr_amd.distributed.length_sorted_shards) and all-gathers
the results back into input order.
"""
from __future__ import annotations

import json
import os
import random
import string
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import model as _model  # noqa: F401  (registers "Paraformer")
from . import sense_voice as _sense_voice  # noqa: F401  (registers "SenseVoiceSmall")
from . import streaming as _streaming  # noqa: F401  (registers "ParaformerStreaming")
from . import punc as _punc  # noqa: F401  (registers "CTTransformer")
from . import vad as _vad  # noqa: F401  (registers "FsmnVADStreaming")
from .frontend import WavFrontend, WavFrontendOnline
from .register import tables
from .text import CharTokenizer, SentencepiecesTokenizer

_TOKENIZERS = {"CharTokenizer": CharTokenizer, "SentencepiecesTokenizer": SentencepiecesTokenizer}


def build_tokenizer(name, conf):
    """tokenizer name + tokenizer_conf -> (tokenizer, vocab_size) (auto_model.py:192-248: vocab from the
    token list, else get_vocab_size()). Without a name the conf decides: bpemodel -> sentencepiece,
    token_list -> CharTokenizer."""
    conf = dict(conf or {})
    if name is None:
        name = "SentencepiecesTokenizer" if conf.get("bpemodel") else (
            "CharTokenizer" if conf.get("token_list") is not None else None)
    if name is None:
        return None, -1
    if not isinstance(name, str) or name not in _TOKENIZERS:
        raise ValueError(f"tokenizer {name!r} is not available (have {sorted(_TOKENIZERS)})")
    tok = _TOKENIZERS[name](**conf)
    vocab = tok.get_num_vocabulary_size() if hasattr(tok, "get_num_vocabulary_size") else tok.get_vocab_size()
    return tok, vocab

_CHARS = string.ascii_letters + string.digits
_LIST_EXT = (".scp", ".txt", ".json", ".jsonl", ".text")


def _load_audio(item) -> np.ndarray:
    if isinstance(item, str):
        from .frontend import read_wav
        return read_wav(item)
    if hasattr(item, "detach"):
        item = item.detach().cpu().numpy()
    return np.asarray(item, dtype=np.float32).reshape(-1)


def _rand_key() -> str:
    return "rand_key_" + "".join(random.choice(_CHARS) for _ in range(13))


def prepare_data_iterator(data_in, input_len=None, data_type=None, key=None) -> Tuple[List[str], List[Any]]:
    """Normalise generate() input into parallel (key_list, data_list)."""
    if isinstance(data_in, str) and data_in.startswith(("http://", "https://")):
        raise ValueError("URL inputs need network access, which this build does not have")
    if isinstance(data_in, str) and os.path.exists(data_in):
        ext = os.path.splitext(data_in)[1].lower()
        if ext in _LIST_EXT:
            keys, items = [], []
            with open(data_in, encoding="utf-8") as f:
                for line in f:
                    if not line.strip():
                        continue
                    if data_in.endswith(".jsonl"):
                        d = json.loads(line.strip())["source"]
                        items.append(d)
                        keys.append(d["key"] if isinstance(d, dict) and "key" in d else _rand_key())
                    else:
                        parts = line.strip().split(maxsplit=1)
                        items.append(parts[1] if len(parts) > 1 else parts[0])
                        keys.append(parts[0] if len(parts) > 1 else _rand_key())
            return keys, items
        k = key if key is not None else os.path.splitext(os.path.basename(data_in))[0]
        return [k], [data_in]
    if isinstance(data_in, (list, tuple)):
        keys = []
        for d in data_in:
            if isinstance(d, str) and os.path.exists(d):
                keys.append(os.path.splitext(os.path.basename(d))[0])
            else:
                keys.append(key if key is not None else _rand_key())
        return keys, list(data_in)
    return [key if key is not None else _rand_key()], [data_in]


def _read_model_dir(path: str, kwargs: Dict[str, Any]) -> Dict[str, Any]:
    """Local model dir: config.yaml (safe YAML) + model.pt + tokens.json + am.mvn."""
    import yaml
    cfg_path = os.path.join(path, "config.yaml")
    conf: Dict[str, Any] = {}
    if os.path.exists(cfg_path):
        with open(cfg_path, encoding="utf-8") as f:
            conf = yaml.safe_load(f) or {}
    out = dict(conf)
    for k, v in kwargs.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = {**out[k], **v}
        else:
            out[k] = v
    out["model"] = conf.get("model", "Paraformer")
    if os.path.exists(os.path.join(path, "model.pt")) and "init_param" not in kwargs:
        out["init_param"] = os.path.join(path, "model.pt")
    tok = os.path.join(path, "tokens.json")
    if os.path.exists(tok):
        out.setdefault("tokenizer_conf", {})
        out["tokenizer_conf"] = {**out.get("tokenizer_conf", {}), "token_list": tok}
    bpe = out.get("tokenizer_conf", {}).get("bpemodel") if isinstance(out.get("tokenizer_conf"), dict) else None
    if bpe and not os.path.isabs(bpe) and os.path.exists(os.path.join(path, os.path.basename(bpe))):
        out["tokenizer_conf"] = {**out["tokenizer_conf"], "bpemodel": os.path.join(path, os.path.basename(bpe))}
    mvn = os.path.join(path, "am.mvn")
    if os.path.exists(mvn):
        out["frontend_conf"] = {**out.get("frontend_conf", {}), "cmvn_file": mvn}
    return out


def load_pretrained_state(path: str) -> Dict[str, torch.Tensor]:
    """model.pt -> state_dict, unwrapping 'state_dict' / 'model_state_dict' / 'model'
    (load_pretrained_model.py:44-47). weights_only=True: nothing in the file executes."""
    src = torch.load(path, map_location="cpu", weights_only=True)
    for k in ("state_dict", "model_state_dict", "model"):
        if isinstance(src, dict) and k in src and isinstance(src[k], dict):
            src = src[k]
            break
    return src


def merge_vad(vad_result, max_length=15000, min_length=0):
    """utils/vad_utils.py merge_vad (SenseVoice `merge_vad=True`): join consecutive VAD segments up to
    max_length ms."""
    if len(vad_result) <= 1:
        return vad_result
    steps = sorted(set([t[0] for t in vad_result] + [t[1] for t in vad_result]))
    if not steps:
        return []
    out, bg = [], 0
    for i in range(len(steps) - 1):
        t = steps[i]
        if steps[i + 1] - bg < max_length:
            continue
        if t - bg > min_length:
            out.append([bg, t])
        bg = t
    out.append([bg, steps[-1]])
    return out


def _dp_world(kwargs) -> Tuple[int, int]:
    """(world, rank) of the data-parallel group a generate() call runs over: the initialised default process group,
    unless the call passes dp=False. Under data parallelism generate() / inference() are COLLECTIVE calls: every
    rank must make them, with the same number of inputs (a rank-0-only call would wait for the others forever)."""
    if kwargs.get("dp", True) and torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_world_size(), torch.distributed.get_rank()
    return 1, 0


def _merge_rank_dirs(model, out_dir: str, rank_dirs: List[str], keys: List[str], kwargs) -> None:
    """Data-parallel output_dir: every rank wrote its share into its own directory (as the reference's multi-GPU
    recipe writes one output dir per job, examples/aishell/paraformer/run.sh:136-170); rank 0 appends their lines to
    the model's writer under out_dir in input order (key order of `keys`) and removes the rank directories."""
    import shutil
    from .writer import model_writer
    order = {}
    for i, k in enumerate(keys):
        order.setdefault(str(k), i)
    files: Dict[Tuple[str, ...], list] = {}
    for rd in rank_dirs:
        for root, _, names in os.walk(rd):
            for n in names:
                rel = tuple(os.path.relpath(os.path.join(root, n), rd).split(os.sep))
                with open(os.path.join(root, n), encoding="utf-8") as f:
                    for line in f:
                        k, _, v = line.rstrip("\n").partition(" ")
                        files.setdefault(rel, []).append((k, v))
    writer = model_writer(model, {**kwargs, "output_dir": out_dir})
    for rel in sorted(files):
        w = writer
        for part in rel:
            w = w[part]
        for k, v in sorted(files[rel], key=lambda kv: order.get(kv[0], len(order))):
            w[k] = v
    for rd in rank_dirs:
        shutil.rmtree(rd, ignore_errors=True)


class AutoModel:
    """funasr.auto.auto_model.AutoModel on the HIP path: model / vad_model / punc_model are built from
    registered names or local model dirs (auto_model.py:110-170); generate() runs inference_with_vad when
    a VAD model is present (:300-306)."""

    def __init__(self, **kwargs):
        if kwargs.get("spk_model"):
            raise NotImplementedError("speaker diarisation (spk_model) is out of scope (SURVEY §7)")
        self.model, self.kwargs = self.build_model(**kwargs)
        self.vad_model, self.vad_kwargs = self._sub_model(kwargs, "vad")
        self.punc_model, self.punc_kwargs = self._sub_model(kwargs, "punc")

    def _sub_model(self, kwargs, kind):
        name = kwargs.get(f"{kind}_model")
        if name is None:
            return None, {}
        sub = dict(kwargs.get(f"{kind}_kwargs") or {})
        sub["model"] = name
        sub["device"] = self.kwargs["device"]
        sub.setdefault("mode", kwargs.get("mode", "exact"))
        return self.build_model(**sub)

    @staticmethod
    def build_model(**kwargs):
        name = kwargs.get("model", "Paraformer")
        if isinstance(name, str) and os.path.isdir(name):
            kwargs = _read_model_dir(name, kwargs)
            name = kwargs["model"]
        if name not in tables.model_classes:
            raise ValueError(f"model {name!r} is not registered (available: {sorted(tables.model_classes)}); "
                             "hub names cannot be downloaded offline — pass a local model dir")
        device = kwargs.get("device", "cuda")
        if not torch.cuda.is_available() or str(device).startswith("cpu") or kwargs.get("ngpu", 1) == 0:
            raise RuntimeError("the HIP Paraformer path needs a ROCm GPU (device='cuda[:i]'); there is no CPU path")
        kwargs["device"] = device
        torch.manual_seed(kwargs.get("seed", 0))
        tok_name = kwargs.get("tokenizer") if isinstance(kwargs.get("tokenizer"), str) else None
        tokenizer, vocab = build_tokenizer(tok_name, kwargs.get("tokenizer_conf"))
        kwargs["tokenizer"] = tokenizer
        fconf = kwargs.get("frontend_conf") or {}
        online = kwargs.get("frontend") == "WavFrontendOnline" or name in ("ParaformerStreaming", "FsmnVADStreaming")
        kwargs["frontend"] = (WavFrontendOnline if online else WavFrontend)(**fconf)
        if tokenizer is None:
            vocab = kwargs.get("vocab_size", -1)
        model_conf = kwargs.get("model_conf") or {}
        mk = {**model_conf, **{k: v for k, v in kwargs.items() if k not in ("model_conf",)}}
        mk["vocab_size"] = vocab
        mk["input_size"] = kwargs["frontend"].output_size()
        model = tables.model_classes[name](**mk)
        if kwargs.get("init_param"):
            model.load_state_dict(load_pretrained_state(kwargs["init_param"]), strict=True)
        elif kwargs.get("synthetic_seed") is not None:
            from .weights import make_weights
            model.load_state_dict(make_weights(model.cfg, int(kwargs["synthetic_seed"])), strict=True)
        model.to(device)
        model.eval()
        return model, kwargs

    def __call__(self, *args, **cfg):
        kwargs = dict(self.kwargs)
        kwargs.update(cfg)
        return self.model(*args, kwargs)

    def generate(self, input, input_len=None, **cfg):
        if self.vad_model is None:
            return self.inference(input, input_len=input_len, **cfg)
        return self.inference_with_vad(input, input_len=input_len, **cfg)

    def inference_with_vad(self, input, input_len=None, **cfg):
        """auto_model.py:378-673 without the speaker branch: VAD segments per input -> segments sorted by
        duration and packed into batches of <= batch_size_s seconds of audio (segments longer than
        batch_size_threshold_s go alone) -> ASR -> original order restored -> texts joined with " ",
        timestamps shifted by the segment start, other fields summed -> punctuation of the joined text."""
        kwargs = dict(self.kwargs)
        kwargs.update(cfg)
        vad_kw = dict(self.vad_kwargs)
        vad_kw.update(cfg)
        keys, items = prepare_data_iterator(input, input_len=input_len, data_type=kwargs.get("data_type"))
        world, rank = _dp_world(kwargs)
        if world > 1:   # data parallel over whole inputs: each rank runs VAD -> ASR -> punctuation on its own share
            from .distributed import agree_item_count, gather_results, shard_items
            if agree_item_count(len(items)) > 1:
                mine = shard_items(items, world, rank)
                sub = {**cfg, "dp": False}
                out_dir = kwargs.get("output_dir")
                if out_dir is not None:   # the ASR writer of each rank writes into a directory of its own
                    saved, self.model.writer = getattr(self.model, "writer", None), None
                    sub["output_dir"] = os.path.join(out_dir, f".dp_rank{rank}")
                local = self._vad_pipeline([items[i] for i in mine], None, sub, {**kwargs, **sub}, vad_kw)
                if out_dir is not None:
                    if getattr(self.model, "writer", None) is not None:
                        self.model.writer.close()
                    self.model.writer = saved
                    torch.distributed.barrier()
                    if rank == 0:
                        _merge_rank_dirs(self.model, out_dir,
                                         [os.path.join(out_dir, f".dp_rank{r}") for r in range(world)], keys, kwargs)
                    torch.distributed.barrier()
                pairs = gather_results([(mine[j], r) for j, r in local])
                return [r for _, r in sorted(pairs, key=lambda p: p[0])]
        return [r for _, r in self._vad_pipeline(input, input_len, cfg, kwargs, vad_kw)]

    def _vad_pipeline(self, input, input_len, cfg, kwargs, vad_kw):
        """(input index, result) pairs of inference_with_vad on this process (inputs whose text is empty give none,
        as in the reference)."""
        vad_kw = {**vad_kw, "dp": cfg.get("dp", vad_kw.get("dp", True))}
        res = self.inference(input, input_len=input_len, model=self.vad_model, kwargs=vad_kw)
        if cfg.get("merge_vad", False):
            for r in res:
                r["value"] = merge_vad(r["value"], kwargs.get("merge_length_s", 15) * 1000)
        batch_ms = max(int(kwargs.get("batch_size_s", 300)) * 1000, 1)
        thres_ms = int(kwargs.get("batch_size_threshold_s", 60)) * 1000
        _, items = prepare_data_iterator(input, input_len=input_len, data_type=kwargs.get("data_type"))
        asr_kw = dict(kwargs)
        asr_kw.pop("batch_size_s", None)
        asr_kw["dp"] = False   # the segment batches of one input stay on this rank
        out = []
        for i, r in enumerate(res):
            key, segs = r["key"], r["value"]
            speech = _load_audio(items[i])
            n = len(segs)
            order = sorted(range(n), key=lambda j: segs[j][1] - segs[j][0])
            if n == 0:
                out.append((i, {"key": key, "text": "", "timestamp": []}))
                continue
            bsz = max(batch_ms, segs[order[0]][1] - segs[order[0]][0])
            results_sorted, beg, end, max_len = [], 0, 1, 0
            for j in range(n):
                slen = segs[order[j]][1] - segs[order[j]][0]
                if j < n - 1 and slen < thres_ms and max(max_len, slen) * (j + 1 - beg) < bsz:
                    max_len = max(max_len, slen)
                    end += 1
                    continue
                batch = []
                for jj in order[beg:end]:   # slice_padding_audio_samples (vad_utils.py:21-32)
                    b0 = int(segs[jj][0] * 16)
                    b1 = min(int(segs[jj][1] * 16), len(speech))
                    batch.append(speech[b0:b1])
                asr_kw["batch_size"] = len(batch)
                results_sorted.extend(self.inference(batch, input_len=None, model=self.model, kwargs=asr_kw))
                beg, end, max_len = end, end + 1, slen
            if len(results_sorted) != n:
                out.append((i, {"key": key, "text": "", "timestamp": []}))
                continue
            restored = [None] * n
            for j in range(n):
                restored[order[j]] = results_sorted[j]
            result: Dict[str, Any] = {}
            for j in range(n):
                for k, v in restored[j].items():
                    if k.startswith("timestamp"):
                        result.setdefault(k, [])
                        for t in v:
                            t[0] += segs[j][0]
                            t[1] += segs[j][0]
                        result[k].extend(v)
                    elif "text" in k:
                        result[k] = v if k not in result else result[k] + " " + v
                    else:
                        result[k] = v if k not in result else result[k] + v
            if not len(result["text"].strip()):
                continue
            if self.punc_model is not None:
                punc_kw = dict(self.punc_kwargs)
                punc_kw.update(cfg)
                punc_kw["dp"] = False   # one text of this rank's input: no collective
                pres = self.inference(result["text"], model=self.punc_model, kwargs=punc_kw)
                if kwargs.get("return_raw_text", False):
                    result["raw_text"] = result["text"]
                result["text"] = pres[0]["text"]
            result["key"] = key
            out.append((i, result))
        return out

    def inference(self, input, input_len=None, model=None, kwargs=None, key=None, **cfg):
        kwargs = dict(self.kwargs if kwargs is None else kwargs)
        kwargs.update(cfg)
        model = self.model if model is None else model
        model.eval()
        batch_size = int(kwargs.get("batch_size", 1))
        keys, items = prepare_data_iterator(input, input_len=input_len, data_type=kwargs.get("data_type"), key=key)
        world, rank = _dp_world(kwargs)
        dp = False
        if world > 1:   # every rank takes the same branch: the decision is made on rank 0's input count
            from .distributed import agree_item_count
            dp = agree_item_count(len(items)) > 1
        mine = list(range(len(items)))
        out_dir, saved_writer = kwargs.get("output_dir"), None
        if dp:   # longest-first round-robin: balanced padded work per rank, decided on rank 0
            from .distributed import shard_items
            mine = shard_items(items, world, rank)
            kb = [keys]   # rank 0's keys on every rank (generated keys are random per process)
            torch.distributed.broadcast_object_list(kb, src=0)
            keys = kb[0]
            if out_dir is not None:   # each rank writes its share into a directory of its own (merged below)
                saved_writer = getattr(model, "writer", None)
                model.writer = None
                kwargs["output_dir"] = os.path.join(out_dir, f".dp_rank{rank}")
        results = []
        mats, mat_index = [], []   # greedy token matrices (device) of this rank's batches, for the tensor gather
        speech_s, wall_s = 0.0, 0.0
        for beg in range(0, len(mine), batch_size):
            idx = mine[beg:beg + batch_size]
            batch = {"data_in": [items[i] for i in idx], "key": [keys[i] for i in idx]}
            if len(idx) == 1 and kwargs.get("data_type") == "fbank":
                batch["data_in"] = items[idx[0]]
                batch["data_lengths"] = input_len
            t1 = time.perf_counter()
            with torch.no_grad():
                res = model.inference(**batch, **{k: v for k, v in kwargs.items() if k not in ("key",)})
            t2 = time.perf_counter()
            out, meta = (res[0], res[1]) if isinstance(res, (list, tuple)) and len(res) > 1 else (res, {})
            if dp and "token_matrix" in meta and hasattr(model, "results_from_token_matrix"):
                mats.append(meta["token_matrix"])
                mat_index.extend(idx)
            if dp:   # (input index, result) per result; n-best models give several per input (meta "owner")
                owner = meta.get("owner")
                if owner is None:
                    if len(out) != len(idx):
                        raise RuntimeError(f"data-parallel inference: {len(out)} results for {len(idx)} inputs")
                    owner = list(range(len(idx)))
                results.extend((idx[o], r) for o, r in zip(owner, out))
            else:
                results.extend(out)
            bt = meta.get("batch_data_time", -1)
            speech_s += bt if bt > 0 else 0.0
            wall_s += t2 - t1
        self.last_speed = {"rtf": (wall_s / speech_s) if speech_s > 0 else None, "forward_s": wall_s}
        self.last_gather = None   # data-parallel runs: "tensor" (token matrices over RCCL / gloo) or "objects"
        if dp and out_dir is not None:
            if getattr(model, "writer", None) is not None:
                model.writer.close()
            model.writer = saved_writer
            torch.distributed.barrier()   # every rank's files are complete
            if rank == 0:
                _merge_rank_dirs(model, out_dir, [os.path.join(out_dir, f".dp_rank{r}") for r in range(world)], keys,
                                 kwargs)
            torch.distributed.barrier()
        if dp:
            from .distributed import gather_results, gather_token_matrices
            # every rank must take the same gather: tensors only when all of them decoded greedy token matrices
            flag = torch.tensor([1 if len(mats) and len(mat_index) == len(mine) else 0], dtype=torch.int64)
            if torch.distributed.get_backend() == "nccl":
                flag = flag.cuda()
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            if int(flag.item()) == 1:   # [n, L] int32 token matrices over RCCL; results built from them on every rank
                self.last_gather = "tensor"
                toks, ntok, index = gather_token_matrices(mats, mat_index)
                if sorted(index.tolist()) != list(range(len(items))):
                    raise RuntimeError("data-parallel inference: the gathered token matrices do not cover the inputs")
                order = np.argsort(index, kind="stable")
                return model.results_from_token_matrix(toks[order], ntok[order], [keys[i] for i in index[order]],
                                                       **{k: v for k, v in kwargs.items() if k != "key"})
            # (input index, result) pairs from every rank -> input order (stable: n-best order kept)
            self.last_gather = "objects"
            pairs = gather_results(results)
            if any(not 0 <= i < len(items) for i, _ in pairs):
                raise RuntimeError("data-parallel inference: gathered a result for an unknown input index")
            results = [r for _, r in sorted(pairs, key=lambda p: p[0])]
        return results
