"""Timing of the beam-search kernel alone (pfm_op_ctc_beam) on synthetic log-probs: how the per-utterance search
scales with frames T, decoder positions L and beam (B utterances, one workgroup each)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from funasr_amd.runtime import op_ctc_beam


def run(B, L, T, V, beam, reps=2):
    g = torch.Generator(device="cuda").manual_seed(0)
    am = torch.log_softmax(torch.randn(B, L, V, device="cuda", generator=g) * 3, -1)
    x = torch.log_softmax(torch.randn(B, T, V, device="cuda", generator=g) * 3, -1)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    nt = torch.full((B,), L, dtype=torch.int32, device="cuda")
    op_ctc_beam(am, x, lens, nt, beam, 0.3, end_detect=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        op_ctc_beam(am, x, lens, nt, beam, 0.3, end_detect=False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


if __name__ == "__main__":
    V = 8404
    for B, L, T, beam in [(64, 230, 500, 10), (64, 230, 250, 10), (64, 115, 500, 10), (64, 230, 500, 5),
                          (16, 230, 500, 10), (128, 230, 500, 10)]:
        ms = run(B, L, T, V, beam)
        print(f"B={B} L={L} T={T} beam={beam}: {ms:.1f} ms  ({ms * 1e3 / L:.0f} us per position)", flush=True)
