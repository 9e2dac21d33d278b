"""Calibrate the fast-mode regret bounds (tests/fast_parity.py) on the headline goldens: exact, fast, and fast with
the decoder's (Paraformer) / CTC head's (SenseVoice) output bias perturbed by sigma * N(0, 1) nat.
python tools/fast_parity_calib.py [para|sv] ..."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from funasr_amd.config import paraformer_large, sense_voice_small  # noqa: E402
from funasr_amd.runtime import PfmEngine  # noqa: E402
from funasr_amd.weights import make_weights  # noqa: E402
from tests.fast_parity import frame_stats, paraformer_stats  # noqa: E402
from tests.golden.inputs import fbank_input  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def perturbed(w, key, sigma, seed=123):
    w = dict(w)
    rng = np.random.default_rng(seed)
    w[key] = (w[key] + sigma * rng.standard_normal(w[key].shape)).astype(np.float32)
    return w


def main():
    which = sys.argv[1:] or ["para", "sv"]
    out = {}
    if "para" in which:
        cfg = paraformer_large()
        w0 = make_weights(cfg, seed=0)
        e = PfmEngine(cfg, 0)
        for tag, w in (("base", w0), ("dec0.1", perturbed(w0, "decoder.output_layer.bias", 0.1)),
                       ("dec0.3", perturbed(w0, "decoder.output_layer.bias", 0.3))):
            e.load_state_dict(w)
            for name in ("para_large_b24", "para_large_b64"):
                g = np.load(f"{GOLD}/{name}.npz")
                x, l = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
                for mode in (("exact", "fast") if tag == "base" else ("fast",)):
                    r = e.run(torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda(), mode=mode)
                    s = paraformer_stats(r["tokens"].cpu().numpy(), r["ntok"].cpu().numpy(), g, 0.5)
                    out[f"{name} {mode} {tag}"] = s
                    print(f"{name} {mode:5s} {tag:7s}", json.dumps(s), flush=True)
    if "sv" in which:
        cfg = sense_voice_small()
        w0 = make_weights(cfg, seed=0)
        e = PfmEngine(cfg, 0)
        q = [cfg.lid_dict.get("auto", 0), 1, 2, cfg.textnorm_dict["woitn"]]
        for tag, w in (("base", w0), ("ctc0.1", perturbed(w0, "ctc.ctc_lo.bias", 0.1)),
                       ("ctc0.3", perturbed(w0, "ctc.ctc_lo.bias", 0.3))):
            e.load_state_dict(w)
            for name in ("sv_large_b24", "sv_large_b64"):
                g = np.load(f"{GOLD}/{name}.npz")
                x, l = fbank_input(int(g["seed"]), int(g["B"]), int(g["T"]), g["lens"])
                for mode in (("exact", "fast") if tag == "base" else ("fast",)):
                    r = e.run_ctc(torch.from_numpy(x).cuda(), torch.from_numpy(l).cuda(), q, mode=mode,
                                  want_frames=True)
                    s = frame_stats(r["frame_ids"].cpu().numpy(), g["enc_lens"], g)
                    nt = r["ntok"].cpu().numpy()
                    ref_nt = np.diff(g["tokens_off"])
                    s["tokens_equal"] = float(np.mean([
                        r["tokens"][b, : nt[b]].cpu().numpy().tolist() ==
                        g["tokens"][g["tokens_off"][b]:g["tokens_off"][b + 1]].tolist() for b in range(len(nt))]))
                    s["count_equal"] = float(np.mean(nt == ref_nt))
                    out[f"{name} {mode} {tag}"] = s
                    print(f"{name} {mode:5s} {tag:7s}", json.dumps(s), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "fast_parity_calib.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
