"""Fast-mode (bf16) parity statistics against a reference run's per-position top-k log-probs.

FAST mode cannot be token-exact against the f32 reference: random-weight models leave a median top-2 margin of
~0.1 nat, and bf16 operands move the logits by O(1e-2). What it must not do is move them far. The
statistic here is the REGRET of each decision: the reference's log-prob of its own best id minus the reference's
log-prob of the id the fast path chose (0 where they agree; the reference's top-k bounds it from below when the
chosen id is outside the stored top-k). A bf16 path's flips happen only at near-ties, so every regret is small and
the mean regret over all positions is tiny; a decoder or encoder bug that moves logits by a few tenths of a nat
produces flips at wider margins, to lower-ranked ids, and a mean regret many times larger
(tests/test_gpu_parity.py calibrates the bounds and checks that a 0.3-nat perturbation of the decoder fails them).

Paraformer positions come from the CIF: where the fast path's token count differs from the reference's, the
positions after the point where the fire patterns diverge are not comparable. Such utterances are compared up to
their first "break" (a chosen id outside the reference's top-k or a regret >= the margin bound). The break and the
positions behind it are not dropped silently: `trunc_positions` / `trunc_frac` count them, `break_max_regret` is
the largest regret AT a break (the first decision where a count-mismatched utterance left the reference; a lower
bound when the id is outside the top-k) and `max_regret_all` the largest regret over every position of the run,
breaks and misaligned tails included; each has its own bound from the emulation (bounds_from_emulation).
"""
from __future__ import annotations

import numpy as np


def regrets(chosen: np.ndarray, top_ids: np.ndarray, top_logp: np.ndarray):
    """chosen [P] ids, top_ids / top_logp [P, k] (best first) -> (regret [P], rank [P]; rank k = outside top-k)."""
    k = top_ids.shape[1]
    hit = top_ids == chosen[:, None]
    rank = np.where(hit.any(1), hit.argmax(1), k)
    lp = np.where(rank < k, top_logp[np.arange(len(chosen)), np.minimum(rank, k - 1)], top_logp[:, -1])
    return (top_logp[:, 0] - lp).astype(np.float64), rank


def paraformer_stats(tokens: np.ndarray, ntok: np.ndarray, g, margin: float) -> dict:
    """tokens [B, L_cap] per-position argmax ids of a run (special ids included), ntok [B]; g a headline golden
    (ntok, top_ids, top_logp per reference position in utterance order)."""
    off = np.concatenate([[0], np.cumsum(g["ntok"])]).astype(np.int64)
    k = g["top_ids"].shape[1]
    reg_all, rank_all = [], []
    equal_counts, prefix_frac = 0, []
    trunc, break_reg, all_max, total = 0, [], 0.0, 0
    for b in range(len(g["ntok"])):
        n_ref, n_got = int(g["ntok"][b]), int(ntok[b])
        n = min(n_ref, n_got)
        ids, lp = g["top_ids"][off[b]:off[b] + n], g["top_logp"][off[b]:off[b] + n]
        r, rk = regrets(tokens[b, :n].astype(np.int64), ids, lp)
        total += n
        if n:
            all_max = max(all_max, float(r.max()))
        if n_ref == n_got:
            equal_counts += 1
        else:   # count-mismatched: comparable up to the first break of the position alignment
            brk = np.nonzero((rk >= k) | (r >= margin))[0]
            cut = int(brk[0]) if len(brk) else n
            prefix_frac.append(cut / max(1, n_ref))
            trunc += n - cut
            if len(brk):
                break_reg.append(float(r[cut]))
            r, rk = r[:cut], rk[:cut]
        reg_all.append(r)
        rank_all.append(rk)
    reg, rank = np.concatenate(reg_all), np.concatenate(rank_all)
    return _summary(reg, rank, k) | dict(equal_counts=equal_counts / len(g["ntok"]),
                                         max_count_diff=int(np.abs(ntok - g["ntok"]).max()),
                                         mismatched=len(prefix_frac),
                                         mismatched_prefix=float(np.mean(prefix_frac)) if prefix_frac else 1.0,
                                         trunc_positions=int(trunc), trunc_frac=trunc / max(1, total),
                                         breaks=len(break_reg),
                                         break_max_regret=max(break_reg) if break_reg else 0.0,
                                         max_regret_all=all_max)


def frame_stats(frame_ids: np.ndarray, olens: np.ndarray, g) -> dict:
    """SenseVoice: per-frame CTC argmax [B, T+4] of a run against the golden's per-frame top-k (frames of
    utterance b are its first olens[b])."""
    k = g["top_ids"].shape[1]
    chosen = np.concatenate([frame_ids[b, : int(olens[b])] for b in range(len(olens))]).astype(np.int64)
    reg, rank = regrets(chosen, g["top_ids"], g["top_logp"])
    return _summary(reg, rank, k)


def _summary(reg, rank, k) -> dict:
    flips = reg > 0
    nf = int(flips.sum())
    return dict(positions=int(len(reg)), flips=nf, flip_frac=nf / max(1, len(reg)),
                mean_regret=float(reg.mean()) if len(reg) else 0.0,
                max_regret=float(reg.max()) if len(reg) else 0.0,
                second_best=float((rank[flips] == 1).mean()) if nf else 1.0,
                outside_topk=int((rank >= k).sum()))


def bounds_from_emulation(em: dict) -> dict:
    """Fast-mode bounds derived from the CPU emulation of the same rounding points (tools/fast_emul.py: the oracle with
    the fast path's bf16 roundings on the reference's inputs, tests/golden/fast_emul.json), NOT from the kernel's own
    output: the GPU must sit at the emulation's level -- flips within 3 points, mean regret within 1.5x (+0.001 nat),
    choices outside the reference top 5 within 2x (at least 0.2 % of the positions), the largest regret within
    0.15 nat, equal token counts within 5 points; the positions count-mismatched utterances lose at their alignment
    breaks within 2x (+2 points, about half an utterance at B = 24), and the regret at a break and over every position within 0.3 nat of the emulation's."""
    pos = max(1, em["positions"])
    b = dict(flip_frac=em["flip_frac"] + 0.03, mean_regret=1.5 * em["mean_regret"] + 0.001,
             outside_frac=max(2.0 * em["outside_topk"] / pos, 0.002), max_regret=em["max_regret"] + 0.15,
             equal_counts=em["equal_counts"] - 0.05)
    if "trunc_frac" in em:   # the positions count-mismatched utterances lose at their breaks, bounded too
        # a break is a decision too: bounded from the larger of the emulation's break and decision regrets
        b.update(trunc_frac=2.0 * em["trunc_frac"] + 0.02,
                 break_max_regret=max(em["break_max_regret"], em["max_regret"]) + 0.3,
                 max_regret_all=em["max_regret_all"] + 0.3)
    return b


def stream_stats(chunks, g, margin: float) -> dict:
    """Streaming: chunks = [(per-position argmax ids of a chunk (specials included), count)] in order; g a streaming
    golden with the reference's per-chunk decoder counts (ntok) and per-position top-k (top_ids / top_logp, chunks
    concatenated). Chunks whose counts differ are compared up to their first break, as paraformer_stats does."""
    off = np.concatenate([[0], np.cumsum(g["ntok"])]).astype(np.int64)
    k = g["top_ids"].shape[1]
    reg_all, rank_all, equal = [], [], 0
    for i, (ids, n_got) in enumerate(chunks):
        n_ref = int(g["ntok"][i])
        n = min(n_ref, int(n_got))
        r, rk = regrets(np.asarray(ids[:n], np.int64), g["top_ids"][off[i]:off[i] + n], g["top_logp"][off[i]:off[i] + n])
        if n_ref == int(n_got):
            equal += 1
        else:
            brk = np.nonzero((rk >= k) | (r >= margin))[0]
            cut = int(brk[0]) if len(brk) else n
            r, rk = r[:cut], rk[:cut]
        reg_all.append(r)
        rank_all.append(rk)
    reg, rank = np.concatenate(reg_all), np.concatenate(rank_all)
    return _summary(reg, rank, k) | dict(equal_counts=equal / max(1, len(chunks)))
