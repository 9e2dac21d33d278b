"""One Paraformer-large streaming stream (fast mode, chunk [0, 10, 5], look-back 4 / 1), 2 x 50 chunks (the second pass
replays the captured HIP graphs), for a rocprofv3 kernel trace of the per-chunk launch chain:
python tools/stream_prof.py [chunks] -> mean ms per chunk of the second pass."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from funasr_amd.config import paraformer_streaming
from funasr_amd.runtime import PfmEngine, PfmStreams
from funasr_amd.weights import make_weights

C = int(sys.argv[1]) if len(sys.argv) > 1 else 50
cfg = paraformer_streaming()
eng = PfmEngine(cfg, 0)
eng.load_state_dict(make_weights(cfg, 0))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(2000)
chunks = torch.randn((C, 1, 10, cfg.input_size), generator=g, device=dev, dtype=torch.float32)
st = PfmStreams(eng, 1, (0, 10, 5), 4, 1, "fast")
for rep in range(2):
    st.reset([0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(C):
        r = st.step([0], chunks[c], [10], [c == C - 1])
        int(r["ntok"].sum().item())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
print(f"{dt / C * 1e3:.3f} ms per chunk", flush=True)
