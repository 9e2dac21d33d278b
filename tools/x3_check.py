"""EXACT mode with bf16x3 GEMMs (PFM_EXACT_TERMS=3) vs the reference goldens: per golden, token-count and
token mismatches, the reference top-2 margin at the flipped positions, encoder row rel-L2 (GPU box).
    PFM_EXACT_TERMS=3 python tools/x3_check.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_parity import GOLD, _margin_flips, _run  # noqa: E402
from funasr_amd.config import paraformer_large  # noqa: E402
from funasr_amd.runtime import PfmEngine  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

cfg = paraformer_large()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, seed=0))
for name in sorted(f[:-4] for f in os.listdir(GOLD) if f.startswith("para_large") and f.endswith(".npz")):
    g = np.load(f"{GOLD}/{name}.npz")
    r = _run(e, g, "exact")
    torch.cuda.synchronize()
    nt = r["ntok"].cpu().numpy()
    flips, worst, compared, frac = _margin_flips(r, g, cfg)
    enc = r["enc"].cpu().numpy()
    lens = g["lens"]
    rel = float("nan")
    if g["enc_rows"].shape[1] == 3:   # headline goldens: rows 0, n/2, n-1 of every utterance
        rows = np.stack([enc[b, [0, int(lens[b]) // 2, int(lens[b]) - 1]] for b in range(len(lens))])
        rel = np.linalg.norm(rows - g["enc_rows"]) / np.linalg.norm(g["enc_rows"])
    print(f"{name}: B={len(lens)} ntok mismatches {int((nt != g['ntok']).sum())}, token flips {flips}/{compared} "
          f"(largest reference margin {worst:.4f} nat), enc rows rel-L2 {rel:.2e}", flush=True)
