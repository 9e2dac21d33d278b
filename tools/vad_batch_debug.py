"""Tiny Paraformer over 3 VAD segments: alone vs one ragged batch (tokens, token counts, alphas sums)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd.config import paraformer_tiny  # noqa: E402
from funasr_amd.frontend import WavFrontend  # noqa: E402
from funasr_amd.runtime import PfmEngine  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.golden.inputs import vad_waveform  # noqa: E402

cfg = paraformer_tiny()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, 0))
fe = WavFrontend(cmvn_file=None)
fe.cmvn = np.load("tests/golden/lfr_cmvn.npz")["cmvn"]
wav = vad_waveform(51, 12.0, [(2.0, 4.0), (6.5, 7.7), (10.0, 12.0)])
segs = [[0, 2150], [3740, 6650], [7430, 10140]]
pieces = [wav[int(a * 16):int(b * 16)] for a, b in segs]
order = sorted(range(3), key=lambda j: segs[j][1] - segs[j][0])
batch = [pieces[j] for j in order]
f, l, _ = fe(e, batch)
r = e.run(f, l, mode="exact", want_alphas=True)
torch.cuda.synchronize()
for i, j in enumerate(order):
    f1, l1, _ = fe(e, [pieces[j]])
    r1 = e.run(f1, l1, mode="exact", want_alphas=True)
    torch.cuda.synchronize()
    n, n1 = int(r["ntok"][i]), int(r1["ntok"][0])
    T = int(l[i])
    df = float((f[i, :T] - f1[0, :T]).abs().max())
    a, a1 = r["alphas"][i].cpu().numpy(), r1["alphas"][0].cpu().numpy()
    print(j, "T", T, int(l1[0]), "feat diff", df, "ntok", n, n1, "alpha sum", a[:T + 1].sum(), a1[:T + 1].sum(),
          "tokens equal", r["tokens"][i, :n].tolist() == r1["tokens"][0, :n1].tolist())

# the oracle (torch-CPU restatement, pinned to the reference incl. ragged batches) on the same batch
from oracle.paraformer_ref import paraformer_infer  # noqa: E402
ref = paraformer_infer(f.cpu().numpy(), l.cpu().numpy(), make_weights(cfg, 0), cfg)
ra = ref["alphas"].numpy() if hasattr(ref["alphas"], "numpy") else np.asarray(ref["alphas"])
ga = r["alphas"].cpu().numpy()
for i, j in enumerate(order):
    T = int(l[i])
    n = int(r["ntok"][i])
    got = [t for t in r["tokens"][i, :n].tolist() if t not in (0, 1, 2)]
    print("oracle batched", j, "alpha max diff", float(np.abs(ga[i, :T + 1] - ra[i, :T + 1]).max()),
          "tokens equal", got == ref["tokens"][i])
print("oracle keys", list(ref.keys()))
