"""Token timestamps from the CIF outputs of `pfm_run` (host post-processing, `pred_timestamp=True`).

Restates the reference's `cif_wo_hidden` (funasr/utils/timestamp_tools.py:11-29) and
`ts_prediction_lfr6_standard` (timestamp_tools.py:31-111) as called from
`Paraformer.inference` (funasr/models/paraformer/model.py:572-582). The fire search runs in
float32 torch-CPU arithmetic like the reference (`alphas.sum()`, the sequential integrate and the
`>= 1 - 1e-4` tests), so fire positions match bit for bit. Pinned by tests/golden/timestamps.json.

Note the reference call passes the CIF peaks as `us_alphas` and the alphas as `us_peaks`
(model.py:574-575); `Paraformer.inference` here does the same.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

FIRE_THRESHOLD = 1.0 - 1e-4


def cif_fire_values(weights: torch.Tensor, threshold: float) -> torch.Tensor:
    """Integrate-and-fire over one utterance without hidden states: value of the integrator at each
    frame before the threshold is subtracted (float32, sequential; timestamp_tools.py:11-29)."""
    w = weights.to(torch.float32).reshape(1, -1)
    acc = torch.zeros(1, dtype=torch.float32)
    thr = torch.ones(1, dtype=torch.float32) * threshold
    out = []
    for t in range(w.shape[1]):
        acc = acc + w[:, t]
        out.append(acc)
        acc = torch.where(acc >= threshold, acc - thr, acc)
    return torch.stack(out, 1)[0]


def ts_prediction_lfr6_standard(us_alphas: torch.Tensor, us_peaks: torch.Tensor, char_list: Sequence[str],
                                vad_offset: float = 0.0, force_time_shift: float = -1.5, sil_in_str: bool = True,
                                upsample_rate: int = 3) -> Tuple[str, List[List[int]]]:
    """(text with '<char> <start> <end>;' entries, [[start_ms, end_ms] per token])."""
    if not len(char_list):
        return "", []
    start_end_frames, max_token_frames = 5, 12
    time_rate = 10.0 * 6 / 1000 / upsample_rate
    a = us_alphas[0] if us_alphas.dim() == 2 else us_alphas
    p = us_peaks[0] if us_peaks.dim() == 2 else us_peaks
    a = a.detach().to("cpu", torch.float32).clone()
    p = p.detach().to("cpu", torch.float32)
    chars = list(char_list)
    if chars[-1] == "</s>":
        chars = chars[:-1]
    fire = torch.where(p >= FIRE_THRESHOLD)[0].numpy() + force_time_shift
    if len(fire) != len(chars) + 1:
        # renormalise the weights so they sum to #tokens + 1, then re-run the fire search
        a = a / (a.sum() / (len(chars) + 1))
        p = cif_fire_values(a, FIRE_THRESHOLD)
        fire = torch.where(p >= FIRE_THRESHOLD)[0].numpy() + force_time_shift
    n_frames = p.shape[0]
    spans: List[List[float]] = []
    labels: List[str] = []
    if fire[0] > start_end_frames:                      # leading silence
        spans.append([0.0, fire[0] * time_rate])
        labels.append("<sil>")
    for i in range(len(fire) - 1):
        labels.append(chars[i])
        if max_token_frames < 0 or fire[i + 1] - fire[i] <= max_token_frames:
            spans.append([fire[i] * time_rate, fire[i + 1] * time_rate])
        else:                                           # long gap: token then silence
            cut = fire[i] + max_token_frames
            spans.append([fire[i] * time_rate, cut * time_rate])
            spans.append([cut * time_rate, fire[i + 1] * time_rate])
            labels.append("<sil>")
    if n_frames - fire[-1] > start_end_frames:          # trailing silence
        mid = (n_frames + fire[-1]) * 0.5
        spans[-1][1] = mid * time_rate
        spans.append([mid * time_rate, n_frames * time_rate])
        labels.append("<sil>")
    elif spans:
        spans[-1][1] = n_frames * time_rate
    if vad_offset:
        for s in spans:
            s[0] += vad_offset / 1000.0
            s[1] += vad_offset / 1000.0
    text = ""
    for lab, s in zip(labels, spans):
        if not sil_in_str and lab == "<sil>":
            continue
        text += "{} {} {};".format(lab, str(s[0] + 0.0005)[:5], str(s[1] + 0.0005)[:5])
    ms = [[int(s[0] * 1000), int(s[1] * 1000)] for lab, s in zip(labels, spans) if lab != "<sil>"]
    return text, ms
