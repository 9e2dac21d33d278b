"""Build oracle/_ref/knf_fbank (the reference's kaldi-native-fbank, compiled from its sources in
/root/reference by oracle/Makefile). Returns the binary path, or None when the reference tree is
absent (GPU box) — the committed golden fixtures then stand in for it."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "_ref", "knf_fbank")


def build_ref():
    if not os.path.isdir("/root/reference/runtime/onnxruntime/third_party/kaldi-native-fbank"):
        return None
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return BIN if os.path.exists(BIN) else None
