"""In-process interleaved A/B of the bf16 attention kernel on the path's shapes (encoder self-attention
B=64 x 500 x 500, decoder cross-attention 64 x 231 x 500, heads 4, d_k 128). Arms are environment
settings read per launch ("X=1" = defaults). Median of rounds; TFLOP/s = 4*B*Tq*Tk*d_k*H / time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from funasr_amd import runtime as rt


def main():
    arms = sys.argv[1:] or ["X=1"]
    dev = torch.device("cuda", 0)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    H, DK = 4, 128
    for name, B, Tq, Tk in [("enc", 64, 500, 500), ("dec", 64, 231, 500)]:
        torch.manual_seed(0)
        q = torch.randn(B * Tq, H * DK, device=dev).bfloat16()
        k = torch.randn(B * Tk, H * DK, device=dev).bfloat16()
        v = torch.randn(B * Tk, H * DK, device=dev).bfloat16()
        kl = torch.full((B,), Tk, dtype=torch.int32, device=dev)
        fl = 4.0 * B * Tq * Tk * DK * H
        res = {a: [] for a in arms}
        for _ in range(5):
            for a in arms:
                env = dict(kv.split("=") for kv in a.split())
                old = {x: os.environ.get(x) for x in env}
                os.environ.update(env)
                rt.op_attention(q, k, v, kl, B, Tq, Tk, H, DK ** -0.5)
                e0, e1 = ev(), ev()
                e0.record()
                for _ in range(10):
                    rt.op_attention(q, k, v, kl, B, Tq, Tk, H, DK ** -0.5)
                e1.record()
                torch.cuda.synchronize()
                res[a].append(e0.elapsed_time(e1) / 10)
                for x, o in old.items():
                    if o is None:
                        os.environ.pop(x)
                    else:
                        os.environ[x] = o
        line = f"{name} B={B} Tq={Tq} Tk={Tk} |"
        for a in arms:
            ms = float(np.median(res[a]))
            line += f" {a}: {ms * 1e3:7.1f}us {fl / ms / 1e9:5.0f}TF |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
