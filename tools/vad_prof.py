"""cProfile of the FSMN-VAD pass over the bench's 300 s long-audio waveform (GPU box):
python tools/vad_prof.py -> top host functions by cumulative time, and the pass's wall time."""
import cProfile, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from funasr_amd.auto_model import AutoModel
from funasr_amd.config import fsmn_vad
from funasr_amd.weights import vad_test_weights
from tests.golden.inputs import vad_waveform

S = 300
wav = vad_waveform(61, float(S), [(t + 7.0, t + 8.2) for t in range(0, S - 10, 11)])
vcfg = fsmn_vad()
am = AutoModel(model="FsmnVADStreaming", model_conf={}, frontend="WavFrontendOnline",
               frontend_conf=dict(lfr_m=5, lfr_n=1), device="cuda", **vcfg.reference_kwargs())
am.model.load_state_dict(vad_test_weights(vcfg, 0))
am.generate(input=wav[:16000 * 20])
torch.cuda.synchronize()
for _ in range(2):
    t0 = time.perf_counter(); r = am.generate(input=wav); torch.cuda.synchronize()
    print(f"VAD pass {S} s: {1e3 * (time.perf_counter() - t0):.1f} ms, {len(r[0]['value'])} segments", flush=True)
pr = cProfile.Profile(); pr.enable(); am.generate(input=wav); torch.cuda.synchronize(); pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
