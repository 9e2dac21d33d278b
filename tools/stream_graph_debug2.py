"""test_inference_streams_batched_equals_single with per-step records, graphs on vs off."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd.config import paraformer_streaming_tiny  # noqa: E402
from funasr_amd import runtime  # noqa: E402
from funasr_amd.streaming import ParaformerStreaming  # noqa: E402
from funasr_amd.frontend import WavFrontendOnline  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.golden.inputs import waveform  # noqa: E402

cfg = paraformer_streaming_tiny()
mdl = ParaformerStreaming(**cfg.reference_kwargs())
mdl.load_state_dict(make_weights(cfg, 0))
mdl.to("cuda")
fe = WavFrontendOnline(cmvn_file=None)
kw = dict(chunk_size=[0, 10, 5], encoder_chunk_look_back=4, decoder_chunk_look_back=1)
wavs = [waveform(seed=40 + i, n=n) for i, n in enumerate([40000, 23456, 31000])]
calls = [[9600, 9600, 20800], [5000, 18456], [31000]]
rec = []
orig = runtime.PfmStreams.step


def step(self, ids, feats, nf, fin, **k):
    r = orig(self, ids, feats, nf, fin, **k)
    torch.cuda.synchronize()
    rec.append((list(ids), list(nf), list(fin), r["ntok"].tolist(),
                [r["tokens"][i, : int(r["ntok"][i])].tolist() for i in range(len(ids))]))
    return r


runtime.PfmStreams.step = step


def go(flag, batched, clear=True):
    os.environ["PFM_STREAM_GRAPH"] = flag
    if clear:
        mdl._pools.clear()
    rec.clear()
    if not batched:
        for w, cs in zip(wavs, calls):
            cache, pos = {}, 0
            for j, n in enumerate(cs):
                mdl.inference_streams([(w[pos:pos + n], cache, j == len(cs) - 1)], frontend=fe, **kw)
                pos += n
    else:
        caches = [{} for _ in wavs]
        pos = [0, 0, 0]
        for j in range(3):
            act = [k for k in range(3) if j < len(calls[k])]
            items = []
            for k in act:
                n = calls[k][j]
                items.append((wavs[k][pos[k]:pos[k] + n], caches[k], j == len(calls[k]) - 1))
                pos[k] += n
            mdl.inference_streams(items, frontend=fe, **kw)
    return list(rec)


def both(flag):
    os.environ["PFM_STREAM_GRAPH"] = flag
    mdl._pools.clear()
    out = []
    for batched in (False, True):
        print(f"---- flag {flag} batched {batched}", file=sys.stderr, flush=True)
        rec.clear()
        os.environ["PFM_STREAM_GRAPH"] = flag
        out += go(flag, batched, clear=False)
    return out


a, b = both("0"), both("1")
for x, y in zip(a, b):
    print("OK " if x == y else "BAD", x, "" if x == y else y, flush=True)
