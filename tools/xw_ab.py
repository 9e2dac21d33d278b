"""Fast mode with PFM_FAST_XW variants (split-plane weights): parity statistics on the headline goldens
(tests/fast_parity.py) and the B=64 x 500 step time, in one process (the library rebuilds its planes / packs when
the knob changes).   python tools/xw_ab.py 0 1 2 4 7 [--rounds R] [--steps K]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from funasr_amd.config import paraformer_large  # noqa: E402
from funasr_amd.runtime import PfmEngine  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.fast_parity import paraformer_stats  # noqa: E402
from tests.golden.inputs import fbank_input  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    cfg = paraformer_large()
    e = PfmEngine(cfg, 0)
    e.load_state_dict(make_weights(cfg, seed=0))
    gold = {}
    for name in ("para_large_b24", "para_large_b64"):
        g = np.load(f"{GOLD}/{name}.npz")
        x, l = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
        gold[name] = (g, torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda())
    B, T = 64, 500
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1000)
    feats = torch.randn((B, T, cfg.input_size), generator=gen, device="cuda", dtype=torch.float32)
    lens = torch.full((B,), T, dtype=torch.int32, device="cuda")
    for v in args.variants:
        os.environ["PFM_FAST_XW"] = v
        for name, (g, x, l) in gold.items():
            r = e.run(x, l, mode="fast")
            s = paraformer_stats(r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy(), g, 0.5)
            print(f"XW={v} {name}", json.dumps({k: (round(val, 5) if isinstance(val, float) else val)
                                                 for k, val in s.items()}), flush=True)
    times = {v: [] for v in args.variants}
    for _ in range(args.rounds):
        for v in args.variants:
            os.environ["PFM_FAST_XW"] = v
            for _ in range(2):
                e.run(feats, lens, mode="fast")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                e.run(feats, lens, mode="fast")
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / args.steps * 1e3)
    for v in args.variants:
        print(f"XW={v} step ms {' '.join(f'{t:.2f}' for t in times[v])} (min {min(times[v]):.2f})", flush=True)


if __name__ == "__main__":
    main()
