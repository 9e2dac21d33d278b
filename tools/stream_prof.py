"""S Paraformer-large streaming streams (default 1) (fast mode, chunk [0, 10, 5], look-back 4 / 1), 2 x 50 chunks (the second pass
replays the captured HIP graphs), for a rocprofv3 kernel trace of the per-chunk launch chain:
python tools/stream_prof.py [chunks] [streams] -> mean ms per chunk of the second pass."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from funasr_amd.config import paraformer_streaming
from funasr_amd.runtime import PfmEngine, PfmStreams
from funasr_amd.weights import make_weights

C = int(sys.argv[1]) if len(sys.argv) > 1 else 50
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1   # concurrent streams
cfg = paraformer_streaming()
eng = PfmEngine(cfg, 0)
eng.load_state_dict(make_weights(cfg, 0))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2000)
chunks = torch.randn((C, S, 10, cfg.input_size), generator=g, device=dev, dtype=torch.float32)
st = PfmStreams(eng, S, (0, 10, 5), 4, 1, "fast")
ids = list(range(S))
for rep in range(2):
    st.reset(ids)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(C):
        r = st.step(ids, chunks[c], [10] * S, [c == C - 1] * S)
        int(r["ntok"].sum().item())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
print(f"{dt / C * 1e3:.3f} ms per chunk", flush=True)
