"""Attention kernel time vs key / query length (bf16 path, heads 4, d_k 128): the slope over Tk is the
per-key-tile cost, the intercept the prologue + epilogue. Arms are environment settings ("X=1" =
defaults). Usage: python tools/attn_scan.py [arm ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from funasr_amd import runtime as rt


def main():
    arms = sys.argv[1:] or ["X=1"]
    dev = torch.device("cuda", 0)
    H, DK = 4, 128
    for B, Tq, Tk in [(64, 500, 64), (64, 500, 128), (64, 500, 256), (64, 500, 512), (64, 500, 1024),
                      (64, 500, 2048), (64, 256, 512), (128, 256, 512), (32, 1000, 512), (16, 2000, 2000)]:
        torch.manual_seed(0)
        q = torch.randn(B * Tq, H * DK, device=dev).bfloat16()
        k = torch.randn(B * Tk, H * DK, device=dev).bfloat16()
        v = torch.randn(B * Tk, H * DK, device=dev).bfloat16()
        kl = torch.full((B,), Tk, dtype=torch.int32, device=dev)
        fl = 4.0 * B * Tq * Tk * DK * H
        line = f"B={B:4d} Tq={Tq:5d} Tk={Tk:5d} |"
        for a in arms:
            env = dict(kv.split("=") for kv in a.split())
            old = {x: os.environ.get(x) for x in env}
            os.environ.update(env)
            ts = []
            for _ in range(5):
                rt.op_attention(q, k, v, kl, B, Tq, Tk, H, DK ** -0.5)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    rt.op_attention(q, k, v, kl, B, Tq, Tk, H, DK ** -0.5)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            for x, o in old.items():
                if o is None:
                    os.environ.pop(x)
                else:
                    os.environ[x] = o
            ms = float(np.median(ts))
            line += f" {a}: {ms * 1e3:8.1f}us {fl / ms / 1e9:5.0f}TF |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
