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
    "token_int" instead (the reference would fail on tokenizer.decode).
All compute — query rows, 70 SAN-M layers, CTC head, argmax and the greedy CTC collapse — runs in
the HIP library (pfm_run_ctc); the host receives one [B, L] token matrix.
"""
from __future__ import annotations

from typing import List

import torch

from .config import SenseVoiceConfig
from .model import HipModel
from .register import tables


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
        if kwargs.get("output_timestamp", False):
            raise NotImplementedError("SenseVoice output_timestamp (ctc_forced_align) is not on the HIP path yet")
        eng = self.engine()
        mode = kwargs.get("mode", self.mode)
        meta = {}
        speech, lens = self._speech(eng, data_in, data_lengths, frontend, kwargs, meta)
        q = self.query_ids(kwargs.get("language", "auto"), kwargs.get("use_itn", False), kwargs.get("text_norm"))
        ban = self.emo_dict["unk"] if kwargs.get("ban_emo_unk", False) else -1
        if ban >= self.cfg.vocab_size:
            ban = -1
        r = eng.run_ctc(speech, lens, q, mode=mode, ban_token=ban)
        toks = r["tokens"].cpu().numpy()            # one device->host copy for the whole batch
        ntok = r["ntok"].cpu().numpy()
        b = toks.shape[0]
        key = self._keys(key, b)
        results = []
        for i in range(b):
            ids = toks[i, : int(ntok[i])].tolist()
            if tokenizer is not None:
                results.append({"key": key[i], "text": tokenizer.decode(ids)})
            else:
                results.append({"key": key[i], "token_int": ids})
        return results, meta
