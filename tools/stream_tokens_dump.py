"""Fast-mode streaming tokens of S streams x C chunks (seeded random features, Paraformer-large streaming
dims) written to a .npy file: run once per library (PFM_LIB=...) and compare the files to A/B a fusion."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd.config import paraformer_streaming  # noqa: E402
from funasr_amd.runtime import PfmEngine, PfmStreams  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402

out, S, C = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
cfg = paraformer_streaming()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, 0))
g = torch.Generator().manual_seed(5)
x = torch.randn((C, S, 10, cfg.input_size), generator=g).cuda()
st = PfmStreams(e, S, (0, 10, 5), 4, 1, "fast")
ids = list(range(S))
rows = []
for c in range(C):
    r = st.step(ids, x[c], [10] * S, [c == C - 1] * S)
    torch.cuda.synchronize()
    tk, nt = r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy()
    for s in range(S):
        rows.append([c, s, int(nt[s])] + tk[s, : nt[s]].tolist())
np.save(out, np.array([np.array(r) for r in rows], dtype=object), allow_pickle=True)
print("chunks", C, "streams", S, "tokens", sum(len(r) - 3 for r in rows))
