"""Per-call latency of pfm_run_punc_host (released CT-Transformer dims, synthetic weights) at one word count:
python tools/punc_bench.py [n] [calls] [mode] -> mean microseconds per call; run under rocprofv3 --kernel-trace
--stats for the per-kernel split of one call."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from funasr_amd.config import ct_transformer
from funasr_amd.runtime import PfmEngine
from funasr_amd.weights import make_weights

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
mode = sys.argv[3] if len(sys.argv) > 3 else "fast"
cfg = ct_transformer()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, seed=0))
ids = np.random.default_rng(0).integers(3, cfg.vocab_size, n).astype(np.int32)
for _ in range(5):
    e.run_punc_host(ids, mode=mode)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(calls):
    e.run_punc_host(ids, mode=mode)
dt = time.perf_counter() - t0
print(f"n={n} mode={mode} graph={os.environ.get('PFM_PUNC_GRAPH', '1')}: {dt / calls * 1e6:.1f} us per call", flush=True)
