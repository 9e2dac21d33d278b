"""Host-side detokenisation: CharTokenizer + sentence post-processing.

Restates the reference's L0 host stage:
  CharTokenizer.ids2tokens / tokens2text   funasr/tokenizer/abs_tokenizer.py:79-82,
                                           funasr/tokenizer/char_tokenizer.py:76-78
  sentence_postprocess (no timestamps)     funasr/utils/postprocess_utils.py:144-249
  abbreviation joining (abbr_dispose)      funasr/utils/postprocess_utils.py:56-141
Pinned by tests/golden/postprocess.json (outputs of the reference functions).
"""
from __future__ import annotations

import json
import os
from functools import lru_cache
from typing import Optional, Iterable, List, Sequence, Union

_SPECIAL = frozenset(("<s>", "</s>", "<unk>", "<OOV>"))


def load_token_list(token_list: Union[str, Sequence[str], None]) -> List[str]:
    """token_list as a list, a tokens.json path (list) or a tokens.txt path (one per line)."""
    if token_list is None:
        return []
    if isinstance(token_list, (list, tuple)):
        return list(token_list)
    p = str(token_list)
    with open(p, encoding="utf-8") as f:
        if p.endswith(".json"):
            return list(json.load(f))
        return [line.rstrip("\n").split()[0] if line.strip() else "" for line in f]


class CharTokenizer:
    """ids <-> tokens <-> text for character vocabularies (tokenizer_conf.token_list)."""

    def __init__(self, token_list=None, space_symbol: str = "<space>", unk_symbol: str = "<unk>", **kwargs):
        self.token_list = load_token_list(token_list)
        self.token2id = {t: i for i, t in enumerate(self.token_list)}
        self.space_symbol = space_symbol
        self.unk_symbol = unk_symbol
        self.unk_id = self.token2id.get(unk_symbol, -1)

    def get_num_vocabulary_size(self) -> int:
        return len(self.token_list)

    def ids2tokens(self, ids: Iterable[int]) -> List[str]:
        return [self.token_list[int(i)] for i in ids]

    def tokens2text(self, tokens: Iterable[str]) -> str:
        tokens = tokens if isinstance(tokens, list) else list(tokens)
        if self.space_symbol not in tokens:
            return "".join(tokens)
        return "".join(" " if t == self.space_symbol else t for t in tokens)

    def text2tokens(self, line: str) -> List[str]:
        return [c for c in line if c != " "]

    def tokens2ids(self, tokens: Iterable[str]) -> List[int]:
        return [self.token2id.get(t, self.unk_id) for t in tokens]

    def decode(self, ids: Iterable[int]) -> str:
        return self.tokens2text(self.ids2tokens(ids))

    def postprocessed_texts(self, rows: Sequence[Sequence[int]]) -> List[str]:
        """sentence_postprocess(ids2tokens(ids))[0] for every id row, with the common case vectorised: a row whose
        tokens (specials dropped) are all Chinese / digit-led / "@" without spaces comes out as their concatenation
        (sentence_postprocess's all-Chinese branch), every other row takes sentence_postprocess itself."""
        import numpy as np
        tab = getattr(self, "_pp_tab", None)
        if tab is None:
            spec = np.array([t in _SPECIAL for t in self.token_list], bool)
            simple = np.array([(t in _SPECIAL) or (_zh_word(t) and " " not in t) for t in self.token_list], bool)
            # one-character tokens as a '<U1' table: a row of them joins as one '<U{k}' view of its gathered codes
            single = np.array([len(t) == 1 for t in self.token_list], bool)
            u1 = np.array([t if len(t) == 1 else " " for t in self.token_list], dtype="<U1")
            tab = self._pp_tab = (spec, simple, single, u1)
        spec, simple, single, u1 = tab
        out = []
        tl = self.token_list
        for ids in rows:
            a = np.asarray(ids, dtype=np.int64)
            if a.size and bool(simple[a].all()):
                kept = a[~spec[a]]
                if kept.size:   # an all-special row is not "all Chinese" (len(mid) == 0): the general path
                    if bool(single[kept].all()):
                        out.append(np.ascontiguousarray(u1[kept]).view(f"<U{kept.size}")[0].strip())
                    else:
                        out.append("".join([tl[i] for i in kept.tolist()]).strip())
                    continue
            out.append(sentence_postprocess(self.ids2tokens(ids))[0])
        return out

    def postprocessed_texts_matrix(self, toks, ntok, drop: Sequence[int] = ()) -> List[str]:
        """postprocessed_texts of the rows toks[i, :ntok[i]] with the ids in `drop` removed (a count past the row width:
        an empty row), straight from the [B, L] host token matrix: the masks, table lookups and the gather of every
        simple one-character row's codes run over the whole matrix at once, each such row is then one '<U{k}' view of
        its slice; other rows take postprocessed_texts."""
        import numpy as np
        toks = np.asarray(toks)
        ntok = np.asarray(ntok).reshape(-1)
        B, L = toks.shape
        self.postprocessed_texts([])   # builds the tables
        spec, simple, single, u1 = self._pp_tab
        n = np.where(ntok <= L, ntok, 0)
        keep = np.arange(L)[None, :] < n[:, None]
        for d in drop:
            keep &= toks != d
        ids = np.where(keep, toks, 0)
        ok = (simple[ids] | ~keep).all(1)
        kept = keep & ~spec[ids]
        ok &= (single[ids] | ~kept).all(1)
        cnt = kept.sum(1)
        ok &= cnt > 0
        codes = u1[toks[kept & ok[:, None]]]   # row-major: the fast rows' codes back to back
        out: List[str] = []
        o = 0
        for i in range(B):
            if ok[i]:
                c = int(cnt[i])
                out.append(codes[o:o + c].view(f"<U{c}")[0].strip())
                o += c
            else:
                out.append(self.postprocessed_texts([toks[i][keep[i]].tolist()])[0])
        return out

    def encode(self, text, **kwargs) -> List[int]:
        """text (a string, or a list of words as the punctuation model passes) -> ids
        (abs_tokenizer.py:65-69; unknown tokens -> unk id)."""
        return self.tokens2ids(self.text2tokens(text))


class SentencepiecesTokenizer:
    """BPE tokenizer over a sentencepiece model file (the SenseVoice tokenizer,
    funasr/tokenizer/sentencepiece_tokenizer.py:12-60): decode = SentencePieceProcessor.DecodeIds."""

    def __init__(self, bpemodel, **kwargs):
        import sentencepiece as spm
        self.bpemodel = str(bpemodel)
        self.sp = spm.SentencePieceProcessor()
        if not self.sp.load(self.bpemodel):
            raise ValueError(f"cannot load sentencepiece model {self.bpemodel}")

    def text2tokens(self, line: str) -> List[str]:
        return self.sp.EncodeAsPieces(line)

    def tokens2text(self, tokens: Iterable[str]) -> str:
        return self.sp.DecodePieces(list(tokens))

    def encode(self, line: str, **kwargs) -> List[int]:
        return self.sp.EncodeAsIds(line)

    def decode(self, line: List[int], **kwargs) -> str:
        return self.sp.DecodeIds([int(i) for i in line])

    def get_vocab_size(self) -> int:
        return self.sp.GetPieceSize()

    def ids2tokens(self, *args, **kwargs):
        return self.decode(*args, **kwargs)

    def tokens2ids(self, *args, **kwargs):
        return self.encode(*args, **kwargs)


def _strip_specials(w: str) -> str:
    w = w.replace(" ", "")
    for s in ("</s>", "<s>", "<unk>", "<OOV>"):
        w = w.replace(s, "")
    return w


def _is_zh(w: str) -> bool:
    # same (string-range) test as the reference's isChinese: CJK block, a digit-led string, or "@"
    return ("一" <= w <= "鿿") or ("0" <= w <= "9") or w == "@"


# Per-token properties, memoised: a vocabulary has at most a few ten thousand distinct tokens, and the greedy results of
# a 64-utterance batch walk ~15k of them through these tests (uncached they cost ~20 ms per batch of host time).
@lru_cache(maxsize=1 << 16)
def _zh_word(w: str) -> bool:
    return _is_zh(_strip_specials(w))


@lru_cache(maxsize=1 << 16)
def _alpha_word(w: str) -> int:
    """_all_alpha of one stripped word: 1 alphabetic (or "'") and not Chinese, 0 otherwise."""
    w = _strip_specials(w)
    if not w.isalpha() and w != "'":
        return 0
    return 0 if (w.isalpha() and _is_zh(w)) else 1


def _all_zh(words) -> bool:
    if isinstance(words, str):   # the reference calls isAllChinese on single words too (a str is its characters)
        return len(words) > 0 and all(_zh_word(c) for c in words)
    return len(words) > 0 and all(_zh_word(w) for w in words)


def _all_alpha(words) -> bool:
    if isinstance(words, str):
        return len(words) > 0 and all(_alpha_word(c) for c in words)
    return len(words) > 0 and all(_alpha_word(w) for w in words)


@lru_cache(maxsize=1 << 16)
def _single_letter(w: str) -> bool:
    return len(w) == 1 and w.encode("utf-8").isalpha()


def _join_abbreviations(words: List[str]) -> List[str]:
    """Runs 'a', ' ', 'b', ' ', 'c' of single ASCII letters become one upper-case word 'ABC'."""
    out: List[str] = []
    n, i = len(words), 0
    while i < n:
        if _single_letter(words[i]) and i + 2 < n and words[i + 1] == " " and _single_letter(words[i + 2]):
            j = i + 2
            while j + 2 < n and words[j + 1] == " " and _single_letter(words[j + 2]):
                j += 2
            out.append("".join(words[k].upper() for k in range(i, j + 1) if words[k] != " "))
            i = j + 1
        else:
            out.append(words[i])
            i += 1
    return out


def _abbreviations_with_spans(words: List[str], spans: List[List[int]]):
    """Abbreviation merge carrying token time spans (postprocess_utils.py:56-141): a run of single
    ASCII letters separated by ' ' becomes one upper-case word spanning first start -> last end;
    other non-space words keep their own span (indexed by their position among non-space words)."""
    n = len(words)
    starts, ends = [], []
    last = -1
    for i in range(n):                                   # pass 1: runs (reference detection order)
        if i <= last:
            continue
        if _single_letter(words[i]) and i + 2 < n and words[i + 1] == " " and _single_letter(words[i + 2]):
            starts.append(i)
            j = i + 2
            ends.append(j)
            while True:
                j += 1
                if j < n and words[j] == " ":
                    j += 1
                    if j < n and _single_letter(words[j]):
                        ends[-1] = j
                        last = j
                    else:
                        break
                else:
                    break
    before = []                                          # non-space words before position i
    cnt = 0
    for w in words:
        before.append(cnt)
        if w != " ":
            cnt += 1
    out, out_spans = [], []
    last = -1
    begin = end = None
    i = 0
    while i < n:
        if i <= last:
            i += 1
            continue
        if i in starts:
            begin = spans[before[i]][0]
            word = words[i].upper()
            i += 1
            while i < n:
                if i in ends:
                    word += words[i].upper()
                    last = i
                    break
                if words[i].encode("utf-8").isalpha():
                    word += words[i].upper()
                i += 1
            out.append(word)
            if i < n and before[i] < len(spans):
                end = spans[before[i]][1]
                out_spans.append([begin, end])
        else:
            out.append(words[i])
            if before[i] < len(spans) and words[i] != " ":
                begin, end = spans[before[i]]
                out_spans.append([begin, end])
        i += 1
    return out, out_spans


def sentence_postprocess(words: Sequence[Union[str, bytes]], time_stamp: Optional[List[List[int]]] = None):
    """Token list -> (sentence, word list); with `time_stamp` (one [start, end] per token) ->
    (sentence, word spans, word list), words then joined by spaces (postprocess_utils.py:144-251).
    Chinese chars joined, BPE '@@' pieces merged, alphabetic words space-separated, single-letter
    runs joined as upper-case abbreviations."""
    mid = [w if isinstance(w, str) else w.decode("utf-8") for w in words]
    mid = [w for w in mid if w not in _SPECIAL]
    ts = time_stamp is not None
    out: List[str] = []
    spans: List[List[int]] = []
    all_zh = _all_zh(mid)
    if all_zh:
        out = [w.replace(" ", "") for w in mid] if any(" " in w for w in mid) else mid
        if ts:
            spans = time_stamp
    elif _all_alpha(mid):
        piece, open_span = "", True
        begin = end = None
        for i, w in enumerate(mid):
            if ts and open_span:
                begin, end = time_stamp[i][0], time_stamp[i][1]
            if "@@" in w:
                piece += w.replace("@@", "")
                if ts:
                    open_span, end = False, time_stamp[i][1]
            else:
                out += [piece + w, " "]
                piece = ""
                if ts:
                    open_span, end = True, time_stamp[i][1]
                    spans.append([begin, end])
                    begin = end
    else:
        piece, after_alpha, open_span = "", False, True
        begin = end = -1
        for i, w in enumerate(mid):
            if ts and open_span:
                begin, end = time_stamp[i][0], time_stamp[i][1]
            if _all_zh(w):
                if after_alpha:
                    out.pop()
                out.append(w)
                after_alpha = False
                if ts:
                    open_span = True
                    spans.append([begin, end])
                    begin = end
            elif "@@" in w:
                piece += w.replace("@@", "")
                after_alpha = False
                if ts:
                    open_span, end = False, time_stamp[i][1]
            elif _all_alpha(w):
                out += [piece + w, " "]
                piece = ""
                after_alpha = True
                if ts:
                    open_span, end = True, time_stamp[i][1]
                    spans.append([begin, end])
                    begin = end
            else:
                out.append(w)
    if ts:
        out, spans = _abbreviations_with_spans(out, spans)
        real = [w for w in out if w != " "]
        return " ".join(real).strip(), spans, real
    if not all_zh:   # an all-Chinese list holds no single ASCII letter: the abbreviation pass would be the identity
        out = _join_abbreviations(out)
    real = [w for w in out if w != " "]
    return "".join(out).strip(), real
