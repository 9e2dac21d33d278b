"""ORACLE — CPU restatement of Paraformer's joint decoder + CTC prefix beam search (TEST INFRASTRUCTURE).

Only `tests/` may import this module, as the checker; the product path runs `pfm_run_beam` (k_beam.hip).
Pinned by tests/test_oracle_golden.py against the reference's own beam_search() outputs
(tests/golden/beam_*.npz, make_golden.py save_beam).

  ctc_prefix_score   funasr/models/transformer/scorers/ctc_prefix_score.py:255-337 (CTCPrefixScore,
                     numpy float32: initial_state, __call__)
  beam_search        funasr/models/paraformer/search.py:35-451 (BeamSearchPara with the CTCPrefixScorer
                     of transformer/scorers/ctc.py:10-80 and LengthBonus, pre-beam "full" of int(1.5 beam)
                     candidates, stable sort-and-prune after each hypothesis, <eos> appended at the last
                     position, end detection of funasr/metrics/common.py:18-46)
  ctc_log_probs      funasr/models/ctc/ctc.py:173-185 (log_softmax(ctc_lo(x)))

Scores are float32 like the reference (torch f32 tensors, numpy f32 CTC states).
"""
from __future__ import annotations

from typing import List, NamedTuple

import numpy as np
import torch

LOGZERO = np.float32(-10000000000.0)


class Hyp(NamedTuple):
    yseq: List[int]
    score: np.float32
    ctc_prev: np.float32
    ctc_r: np.ndarray        # [T, 2] float32: r_t^n, r_t^b of the prefix


def ctc_initial_state(x: np.ndarray, blank: int) -> np.ndarray:
    """CTCPrefixScore.initial_state (ctc_prefix_score.py:272-285)."""
    T = x.shape[0]
    r = np.full((T, 2), LOGZERO, dtype=np.float32)
    r[0, 1] = x[0, blank]
    for i in range(1, T):
        r[i, 1] = r[i - 1, 1] + x[i, blank]
    return r


def ctc_prefix_score(x: np.ndarray, y: List[int], cs: np.ndarray, r_prev: np.ndarray, blank: int, eos: int):
    """CTCPrefixScore.__call__ (ctc_prefix_score.py:287-337): log prefix probabilities of y + c for c in cs and
    the new states [len(cs), T, 2]. Rows before output_length - 1 are never read (the reference leaves them
    uninitialised); they are zero here."""
    T = x.shape[0]
    ol = len(y) - 1
    r = np.zeros((T, 2, len(cs)), dtype=np.float32)
    xs = x[:, cs]
    if ol == 0:
        r[0, 0] = xs[0]
        r[0, 1] = LOGZERO
    else:
        r[ol - 1] = LOGZERO
    r_sum = np.logaddexp(r_prev[:, 0], r_prev[:, 1])
    last = y[-1]
    if ol > 0 and last in cs:
        log_phi = np.ndarray((T, len(cs)), dtype=np.float32)
        for i in range(len(cs)):
            log_phi[:, i] = r_sum if cs[i] != last else r_prev[:, 1]
    else:
        log_phi = r_sum
    start = max(ol, 1)
    log_psi = r[start - 1, 0].copy()
    for t in range(start, T):
        r[t, 0] = np.logaddexp(r[t - 1, 0], log_phi[t - 1]) + xs[t]
        r[t, 1] = np.logaddexp(r[t - 1, 0], r[t - 1, 1]) + x[t, blank]
        log_psi = np.logaddexp(log_psi, log_phi[t - 1] + xs[t])
    eos_pos = np.where(cs == eos)[0]
    if len(eos_pos) > 0:
        log_psi[eos_pos] = r_sum[-1]
    blank_pos = np.where(cs == blank)[0]
    if len(blank_pos) > 0:
        log_psi[blank_pos] = LOGZERO
    return log_psi.astype(np.float32), np.rollaxis(r, 2)


def _topk(v: np.ndarray, k: int) -> np.ndarray:
    """Indices of the k largest values, descending; equal values keep the lower index first."""
    return np.argsort(-v, kind="stable")[:k]


def end_detect(ended: List[Hyp], i: int, M: int = 3, D_end: float = np.log(1 * np.exp(-10))) -> bool:
    """funasr/metrics/common.py:18-46 (lengths count sos and eos)."""
    if len(ended) == 0:
        return False
    best = max(h.score for h in ended)
    count = 0
    for m in range(M):
        same = [h.score for h in ended if len(h.yseq) == i - m]
        if same and max(same) - best < D_end:
            count += 1
    return count == M


def beam_search(am_scores: np.ndarray, x: np.ndarray, beam: int, ctc_weight: float, penalty: float, sos: int,
                eos: int, blank: int = 0, end_detect_on: bool = True) -> List[Hyp]:
    """BeamSearchPara.forward over one utterance: am_scores [L, V] decoder log-probs, x [T, V] CTC log-probs.
    Returns the ended hypotheses, best first (stable for equal scores)."""
    L, V = am_scores.shape
    pre = int(1.5 * beam)
    do_pre = pre < V
    w = np.float32(ctc_weight)
    running = [Hyp([sos], np.float32(0.0), np.float32(0.0), ctc_initial_state(x, blank))]
    ended: List[Hyp] = []
    for i in range(L):
        ws0 = am_scores[i].astype(np.float32)
        if penalty != 0.0:
            ws0 = (ws0 + np.float32(penalty)).astype(np.float32)
        part = _topk(ws0, pre) if do_pre else np.arange(V)
        best: List[Hyp] = []
        for h in running:
            psi, rn = ctc_prefix_score(x, h.yseq, part, h.ctc_r, blank, eos)
            ts = (psi - h.ctc_prev).astype(np.float32)
            wsp = (ws0[part] + (w * ts).astype(np.float32)).astype(np.float32)
            wsp = (wsp + h.score).astype(np.float32)
            for j in _topk(wsp, beam):
                best.append(Hyp(h.yseq + [int(part[j])], wsp[j], psi[j], rn[j]))
            best = sorted(best, key=lambda z: z.score, reverse=True)[:beam]
        if i == L - 1:
            best = [h._replace(yseq=h.yseq + [eos]) for h in best]
        running = []
        for h in best:
            (ended if h.yseq[-1] == eos else running).append(h)
        if end_detect_on and end_detect(ended, i):
            break
        if not running:
            break
    return sorted(ended, key=lambda z: z.score, reverse=True)


@torch.no_grad()
def ctc_log_probs(enc: torch.Tensor, w, key: str = "ctc.ctc_lo") -> torch.Tensor:
    """ctc/ctc.py:173-185: log_softmax(ctc_lo(enc)) in f32."""
    W = w[f"{key}.weight"]
    b = w[f"{key}.bias"]
    W = W if isinstance(W, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(W))
    b = b if isinstance(b, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(b))
    return torch.log_softmax(torch.nn.functional.linear(enc, W, b), dim=-1)
