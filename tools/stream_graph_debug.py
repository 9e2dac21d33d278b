"""Per-chunk tokens of one stream through ParaformerStreaming.inference_streams with HIP graphs on vs off."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd.config import paraformer_streaming_tiny  # noqa: E402
from funasr_amd.runtime import PfmEngine, PfmStreams  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from funasr_amd.frontend import WavFrontendOnline  # noqa: E402
from tests.golden.inputs import waveform  # noqa: E402

cfg = paraformer_streaming_tiny()
e = PfmEngine(cfg, 0)
e.load_state_dict(make_weights(cfg, 0))
fe = WavFrontendOnline(cmvn_file=None)
w = waveform(seed=40, n=40000)
segs = [w[i * 9600:(i + 1) * 9600] for i in range(5)]
feats = []
cache = {}
for j, sgm in enumerate(segs):
    feats.append(fe.step(e, [(sgm, j == 4, cache)])[0].clone())
print("rows", [f.shape[0] for f in feats])


def run(flag):
    os.environ["PFM_STREAM_GRAPH"] = flag
    s = PfmStreams(e, 4, (0, 10, 5), 4, 1, "exact")
    out = []
    for rep in range(2):
        s.reset([0])
        for j, f in enumerate(feats):
            r = s.step([0], f[None].contiguous(), [f.shape[0]], [j == 4])
            torch.cuda.synchronize()
            n = int(r["ntok"][0])
            out.append((rep, j, n, r["tokens"][0, :n].tolist()))
    return out


a, b = run("0"), run("1")
for x, y in zip(a, b):
    print("OK " if x == y else "BAD", x, y if x != y else "")
