"""Streaming (config C5) leg alone, for rocprofv3: S streams x C chunks of Paraformer-large streaming."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd.config import paraformer_streaming  # noqa: E402
from funasr_amd.runtime import PfmEngine, PfmStreams  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--streams", type=int, default=1)
ap.add_argument("--chunks", type=int, default=50)
ap.add_argument("--mode", default="fast")
a = ap.parse_args()
cfg = paraformer_streaming()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, 0))
S, C = a.streams, a.chunks
x = torch.randn((C, S, 10, cfg.input_size), device="cuda")
st = PfmStreams(e, S, (0, 10, 5), 4, 1, a.mode)
ids = list(range(S))
for rep in range(2):
    st.reset(ids)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(C):
        r = st.step(ids, x[c], [10] * S, [c == C - 1] * S)
        int(r["ntok"].sum())
    torch.cuda.synchronize()
    print(f"rep {rep}: {(time.perf_counter() - t0) / C * 1e3:.3f} ms/chunk", flush=True)
