"""`SenseVoiceSmall` model class with the reference's plugin contract, backed by libpfm_hip.so.

Contract (funasr/models/sense_voice/model.py:589-950):
  * registered as tables.model_classes["SenseVoiceSmall"]; constructed as
    cls(encoder="SenseVoiceEncoderSmall", encoder_conf=..., input_size=560, vocab_size=V, **kwargs);
  * state_dict keys/shapes of the reference (encoder.{encoders0,encoders,tp_encoders}.*,
    encoder.after_norm, encoder.tp_norm, ctc.ctc_lo, embed);
  * inference(data_in, data_lengths=None, key=None, tokenizer=None, frontend=None, **kwargs)
    -> (results, meta); kwargs language ("auto"|"zh"|"en"|"yue"|"ja"|"ko"|"nospeech"), use_itn,
    text_norm ("withitn"|"woitn"), ban_emo_unk; results [{"key", "text"}] with
    text = tokenizer.decode(token_int) (model.py:896-945). With tokenizer None the result carries
    "token_int" instead (the reference would fail on tokenizer.decode);
  * output_timestamp=True adds "timestamp": [[start ms, end ms], ...] per word (model.py:917-945, post() at
    :949-965): the CTC forced alignment runs on the device (pfm_ctc_align), the frame grouping and word merge on
    the host. Each utterance uses its own frames (the reference's batch > 1 code indexes encoder_out_lens[0] and
    fails on ragged batches; at batch 1 the two agree), and an utterance with no token after the four query
    positions gets an empty list (the reference raises IndexError there).
All compute — query rows, 70 SAN-M layers, CTC head, argmax and the greedy CTC collapse — runs in
the HIP library (pfm_run_ctc); the host receives one [B, L] token matrix.
"""
from __future__ import annotations

from typing import List

import torch

from .config import SenseVoiceConfig
from .model import HipModel
from .register import tables
from .writer import model_writer


@tables.register("model_classes", "SenseVoiceSmall")
class SenseVoiceSmall(HipModel):
    family = "sensevoice"

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.cfg = SenseVoiceConfig.from_kwargs(**kwargs)
        self.blank_id = self.cfg.blank_id
        self.lid_dict = dict(self.cfg.lid_dict)
        self.textnorm_dict = dict(self.cfg.textnorm_dict)
        self.emo_dict = {"unk": 25009, "happy": 25001, "sad": 25002, "angry": 25003, "neutral": 25004}
        self._init_common(kwargs)

    def query_ids(self, language="auto", use_itn=False, text_norm=None) -> List[int]:
        """[language, event (1), emotion (2), textnorm] embedding rows (model.py:851-876)."""
        if text_norm is None:
            text_norm = "withitn" if use_itn else "woitn"
        if text_norm not in self.textnorm_dict:
            raise KeyError(text_norm)   # the reference indexes textnorm_dict directly
        return [self.lid_dict[language] if language in self.lid_dict else 0, 1, 2, self.textnorm_dict[text_norm]]

    @torch.no_grad()
    def inference(self, data_in, data_lengths=None, key: List[str] = None, tokenizer=None, frontend=None,
                  **kwargs):
        want_ts = bool(kwargs.get("output_timestamp", False))
        if want_ts and tokenizer is None:
            raise ValueError("output_timestamp needs the tokenizer (tokenizer.text2tokens, model.py:919)")
        eng = self.engine()
        mode = kwargs.get("mode", self.mode)
        meta = {}
        speech, lens = self._speech(eng, data_in, data_lengths, frontend, kwargs, meta)
        q = self.query_ids(kwargs.get("language", "auto"), kwargs.get("use_itn", False), kwargs.get("text_norm"))
        ban = self.emo_dict["unk"] if kwargs.get("ban_emo_unk", False) else -1
        if ban >= self.cfg.vocab_size:
            ban = -1
        r = eng.run_ctc(speech, lens, q, mode=mode, ban_token=ban, want_enc=want_ts)
        toks = r["tokens"].cpu().numpy()            # one device->host copy for the whole batch
        ntok = r["ntok"].cpu().numpy()
        b = toks.shape[0]
        key = self._keys(key, b)
        ids_all = [toks[i, : int(ntok[i])].tolist() for i in range(b)]
        align = None
        if want_ts:   # forced alignment of token_int[4:] on the device, one [B, T] readback
            olens = lens.reshape(-1).to(torch.int32) + 4
            align = eng.ctc_align(r["enc"], olens, [ids[4:] for ids in ids_all], self.blank_id).cpu().numpy()
            nfr = (olens - 4).cpu().numpy()
        results = []
        writer = model_writer(self, kwargs)   # output_dir: 1best_recog/text (sense_voice/model.py:899-915)
        for i in range(b):
            ids = ids_all[i]
            if tokenizer is None:
                results.append({"key": key[i], "token_int": ids})
                continue
            text = tokenizer.decode(ids)
            if writer is not None:
                writer["1best_recog"]["text"][key[i]] = text
            res = {"key": key[i], "text": text}
            if want_ts:
                n = int(nfr[i])
                groups = [] if len(ids) <= 4 else frame_groups(align[i, :n], n, tokenizer.text2tokens(text)[4:],
                                                               self.blank_id)
                res["timestamp"] = word_timestamps(groups)
            results.append(res)
        return results, meta


def frame_groups(align, n_frames: int, pieces, blank: int = 0) -> list:
    """model.py:929-944: consecutive frames of one label form a group; each non-blank group is
    [piece, start s, end s] with 60 ms frames centred at -30 ms. The end is capped at the last frame's time,
    computed as the reference does it: an int64 tensor divided by 1000, i.e. in float32."""
    import numpy as np
    cap = np.float32(n_frames * 60 - 30) / np.float32(1000)
    out, start, k = [], 0, 0
    labels = align.tolist()
    i = 0
    while i < len(labels):
        j = i
        while j < len(labels) and labels[j] == labels[i]:
            j += 1
        end = start + (j - i)
        if labels[i] != blank:
            right = (end * 60 - 30) / 1000
            out.append([pieces[k], max((start * 60 - 30) / 1000, 0), cap if cap < np.float32(right) else right])
            k += 1
        start, i = end, j
    return out


def word_timestamps(groups) -> list:
    """SenseVoiceSmall.post (model.py:949-965): pieces starting a word ("\u2581" prefix, one character, or a
    non-letter second character) open a [start ms, end ms] entry, the others extend the previous entry's end;
    a bare "\u2581" is dropped."""
    words = []
    for i, (piece, start, end) in enumerate(groups):
        if piece == "\u2581":
            continue
        if i == 0 or piece.startswith("\u2581") or len(piece) == 1 or not piece[1].isalpha():
            words.append([int(start * 1000), int(end * 1000)])
        else:
            words[-1][1] = int(end * 1000)
    return words
