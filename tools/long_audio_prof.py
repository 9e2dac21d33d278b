"""cProfile of bench.py's long-audio leg (AutoModel(model, vad_model, punc_model).generate over 300 s) on the
GPU box: python tools/long_audio_prof.py -> the leg's JSON and the top host functions by cumulative time."""
import cProfile, json, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse
import bench
from funasr_amd.config import paraformer_large
from funasr_amd.weights import make_weights

args = argparse.Namespace(long_audio_s=300, mode="fast", seed=0)
cfg = paraformer_large()
sd = make_weights(cfg, 0)
print(json.dumps(bench.long_audio_leg(args, sd, cfg)), flush=True)
pr = cProfile.Profile(); pr.enable(); print(json.dumps(bench.long_audio_leg(args, sd, cfg)), flush=True); pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
