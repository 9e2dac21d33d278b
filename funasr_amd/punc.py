"""`CTTransformer` punctuation model with the reference's plugin contract, backed by libpfm_hip.so.

Contract (funasr/models/ct_transformer/model.py:35-420):
  * registered as tables.model_classes["CTTransformer"]; constructed as cls(encoder="SANMEncoder",
    encoder_conf=..., vocab_size=V, punc_list=[...], embed_unit, att_unit, sentence_end_id, **kwargs);
  * state_dict keys/shapes of the reference (embed, encoder.*, decoder);
  * inference(data_in=[text], key=[k], tokenizer=CharTokenizer, **kwargs) -> ([{"key", "text",
    "punc_array"}], meta): text split into words, 20-word mini-sentences, each run through the model
    with the words carried over since the last sentence end, punctuation inserted (model.py:240-412).
The model forward — embedding gather, x sqrt(d) + PE, the SAN-M blocks, after_norm, the punctuation
head and its argmax — runs in the HIP library (pfm_run_punc); the text bookkeeping below is host code,
as in the reference.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import numpy as np
import torch

from .config import CTTransformerConfig
from .model import HipModel
from .register import tables

CACHE_POP_TRIGGER_LIMIT = 200   # model.py:257


def split_words(text: str) -> List[str]:
    """ct_transformer/utils.py:23-83 without a jieba dictionary: every non-ASCII character is a word,
    runs of ASCII characters inside a whitespace-separated segment are one word."""
    words: List[str] = []
    for seg in text.split():
        cur = ""
        for ch in seg:
            if len(ch.encode()) == 1:
                cur += ch
            else:
                if cur:
                    words.append(cur)
                    cur = ""
                words.append(ch)
        if cur:
            words.append(cur)
    return words


def split_to_mini_sentence(words: Sequence, word_limit: int = 20) -> List[list]:
    """ct_transformer/utils.py:9-20: consecutive pieces of word_limit words (the last one shorter)."""
    if word_limit <= 1:
        raise ValueError("word_limit must be > 1")
    words = list(words)
    if len(words) <= word_limit:
        return [words]
    return [words[i:i + word_limit] for i in range(0, len(words), word_limit)]


def _ascii_start(w: str) -> bool:
    return len(w[0].encode()) == 1


def punc_inference(text: str, tokenizer, forward: Callable[[np.ndarray], np.ndarray], punc_list: List[str],
                   sentence_end_id: int, split_size: int = 20) -> Tuple[str, List[int]]:
    """The text loop of CTTransformer.inference (model.py:244-390). `forward(ids int32 [n]) -> punctuation
    id per word [n]` is the model. Returns (punctuated text, punc_array)."""
    words = split_words(text)
    ids = list(tokenizer.encode(words))
    mini = split_to_mini_sentence(words, split_size)
    mini_ids = split_to_mini_sentence(ids, split_size)
    cache_words: List[str] = []
    cache_ids: List[int] = []
    out_text = ""
    out_punc: List[int] = []
    punc_array: List[int] = []
    text_out = ""
    is_end = lambda p: punc_list[p] in ("。", "？")   # noqa: E731
    for si in range(len(mini)):
        sent = cache_words + list(mini[si])
        sent_ids = np.asarray(cache_ids + list(mini_ids[si]), dtype=np.int32)
        punc = [int(x) for x in forward(sent_ids)]
        if len(punc) != len(sent):
            raise RuntimeError("punctuation model returned a wrong number of labels")
        if si < len(mini) - 1:
            # the last sentence end (period / question mark) closes this piece; the rest is carried
            end, last_comma = -1, -1
            for i in range(len(punc) - 2, 1, -1):
                if is_end(punc[i]):
                    end = i
                    break
                if last_comma < 0 and punc_list[punc[i]] == "，":
                    last_comma = i
            if end < 0 and len(sent) > CACHE_POP_TRIGGER_LIMIT and last_comma >= 0:
                end = last_comma   # too long without a sentence end: cut at the last comma
                punc[end] = sentence_end_id
            cache_words, cache_ids = sent[end + 1:], [int(x) for x in sent_ids[end + 1:]]
            sent, punc = sent[:end + 1], punc[:end + 1]
        out_punc += punc
        pieces = []
        for i in range(len(sent)):
            if (i == 0 or is_end(punc[i - 1])) and _ascii_start(sent[i]):
                sent[i] = sent[i].capitalize()
            if i == 0 and _ascii_start(sent[i]):
                sent[i] = " " + sent[i]
            if i > 0 and _ascii_start(sent[i]) and _ascii_start(sent[i - 1]):
                sent[i] = " " + sent[i]
            pieces.append(sent[i])
            p = punc_list[punc[i]]
            if p != "_":
                if _ascii_start(sent[i]):
                    p = {"，": ",", "。": ".", "？": "?"}.get(p, p)
                pieces.append(p)
        out_text += "".join(pieces)
        text_out = out_text
        if si == len(mini) - 1:   # close the text with a sentence end (model.py:346-381)
            last = out_text[-1]
            if last in ("，", "、"):
                text_out = out_text[:-1] + "。"
            elif last == ",":
                text_out = out_text[:-1] + "."
            elif last not in ("。", "？") and len(last.encode()) != 1:
                text_out = out_text + "。"
                if punc:
                    punc[-1] = 2
            elif last not in (".", "?") and len(last.encode()) == 1:
                text_out = out_text + "."
                if punc:
                    punc[-1] = 2
        punc_array += punc
    return text_out, punc_array


@tables.register("model_classes", "CTTransformer")
class CTTransformer(HipModel):
    family = "ct_transformer"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.cfg = CTTransformerConfig.from_kwargs(**kwargs)
        self.punc_list = list(self.cfg.punc_list)
        self.sentence_end_id = self.cfg.sentence_end_id
        if kwargs.get("jieba_usr_dict"):
            raise NotImplementedError("word-level (jieba) punctuation models are not on the HIP path")
        self._init_common(kwargs)

    def punc_forward(self, ids: np.ndarray) -> np.ndarray:
        """One mini-sentence: word ids [n] -> argmax punctuation id per word (pfm_run_punc)."""
        # the text loop is latency-bound (one call per mini-sentence): host ids in, host labels out, one C call
        return self.engine().run_punc_host(ids, mode=self.mode)

    @torch.no_grad()
    def inference(self, data_in, data_lengths=None, key: List[str] = None, tokenizer=None, frontend=None,
                  **kwargs):
        items = data_in if isinstance(data_in, (list, tuple)) else [data_in]
        if len(items) != 1:
            raise AssertionError("batch_size must be 1")   # model.py:240
        text = items[0]
        if isinstance(text, bytes):
            text = text.decode("utf-8")
        if tokenizer is None:
            raise ValueError("CTTransformer.inference needs the CharTokenizer of the model's token list")
        mode = kwargs.get("mode", self.mode)
        prev, self.mode = self.mode, mode
        try:
            out, punc_array = punc_inference(text, tokenizer, self.punc_forward, self.punc_list,
                                             self.sentence_end_id, int(kwargs.get("split_size", 20)))
        finally:
            self.mode = prev
        key = self._keys(key, 1)
        return [{"key": key[0], "text": out, "punc_array": torch.tensor(punc_array, dtype=torch.int64)}], {}
