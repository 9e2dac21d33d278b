"""cProfile of bench.py's generate leg (AutoModel.generate on the headline fbank batch with a tokenizer) on the GPU
box: python tools/generate_prof.py -> per-call wall and the top host functions."""
import cProfile, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from funasr_amd.auto_model import AutoModel
from funasr_amd.config import paraformer_large
from funasr_amd.weights import make_weights
from tests.golden.inputs import fbank_input, token_list

cfg = paraformer_large()
am = AutoModel(model="Paraformer", model_conf=dict(ctc_weight=0.0, predictor_bias=1), device="cuda", mode="fast",
               tokenizer_conf=dict(token_list=token_list(cfg.vocab_size)), **cfg.reference_kwargs())
am.model.load_state_dict(make_weights(cfg, 0))
x, l = fbank_input(seed=1, B=64, T=500)
feats, lens = torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda()
kw = dict(input=feats, input_len=lens, data_type="fbank", batch_size=64)
for _ in range(3):
    am.generate(**kw)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    am.generate(**kw)
torch.cuda.synchronize()
print(f"generate {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call", flush=True)
eng = am.model.engine()
t0 = time.perf_counter()
for _ in range(10):
    r = eng.run(feats, lens, mode="fast")
torch.cuda.synchronize()
print(f"engine.run {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per call", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    am.generate(**kw)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
