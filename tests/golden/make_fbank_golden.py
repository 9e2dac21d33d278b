"""Fbank goldens from the REFERENCE C++ (oracle/_ref/knf_fbank, built from the vendored
kaldi-native-fbank sources by oracle/Makefile) on seeded synthetic waveforms and on the
reference's own test wav (runtime/triton_gpu/client/test_wavs/mid.wav, stored as int16 input).
Build container only:  python tests/golden/make_fbank_golden.py"""
import os
import subprocess
import sys
import tempfile
import wave

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle.build_ref import build_ref  # noqa: E402
from tests.golden.inputs import waveform  # noqa: E402

MID = "/root/reference/runtime/triton_gpu/client/test_wavs/mid.wav"


def knf(wav_f32):
    exe = build_ref()
    with tempfile.TemporaryDirectory() as d:
        fi, fo = os.path.join(d, "in.f32"), os.path.join(d, "out.f32")
        (np.asarray(wav_f32, np.float32) * np.float32(32768.0)).tofile(fi)
        subprocess.run([exe, fi, fo], check=True)
        return np.fromfile(fo, dtype=np.float32).reshape(-1, 80)


def main():
    out = {}
    for i, n in enumerate([400, 401, 559, 560, 16000, 19680, 80000]):
        w = waveform(100 + i, n)
        out[f"syn{i}_n"] = np.array(n)
        out[f"syn{i}_seed"] = np.array(100 + i)
        out[f"syn{i}_fbank"] = knf(w)
    with wave.open(MID, "rb") as f:
        pcm = np.frombuffer(f.readframes(f.getnframes()), dtype="<i2").copy()
    out["mid_pcm"] = pcm
    out["mid_fbank"] = knf(pcm.astype(np.float32) / 32768.0)
    np.savez_compressed(os.path.join(HERE, "fbank_knf.npz"), **out)
    print({k: v.shape for k, v in out.items() if k.endswith("fbank")})


if __name__ == "__main__":
    main()
