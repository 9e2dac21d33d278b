"""In-process interleaved A/B: fused 512-wide GEMM + LayerNorm (pfm_op_gemm_layernorm) against the
unfused pair (pfm_op_gemm with residual, then pfm_op_layernorm) and the plain GEMM alone, on the
path's shapes. Median of rounds; prints us per call and the GEMM-equivalent TFLOP/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from funasr_amd import runtime as rt

SHAPES = [("enc out+res", 32000, 512, True), ("enc ffn2+res", 32000, 2048, True),
          ("dec w2", 14784, 2048, False), ("dec out+res", 14784, 512, True)]
if os.environ.get("SCAN_X6"):   # EXACT-mode (x6) K' = 6K shapes of one encoder group
    SHAPES = [("x6 out+res", 16000, 3072, True), ("x6 ffn2+res", 16000, 12288, True)]


def main():
    dev = torch.device("cuda", 0)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    N = 512
    for name, M, K, has_res in SHAPES:
        torch.manual_seed(0)
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=dev)
        R = torch.randn(M, N, device=dev) if has_res else None
        g = torch.ones(N, device=dev)
        z = torch.zeros(N, device=dev)
        variants = {
            "gemm": lambda: rt.op_gemm(A, W, b, R),
            "gemm+ln": lambda: rt.op_layernorm(rt.op_gemm(A, W, b, R), g, z, 1e-12),
            "fused": lambda: rt.op_gemm_layernorm(A, W, g, z, 1e-12, bias=b, res=R, want_x=has_res),
        }
        res = {k: [] for k in variants}
        for _ in range(5):
            for k, f in variants.items():
                f()
                a, e = ev(), ev()
                a.record()
                for _ in range(10):
                    f()
                e.record()
                torch.cuda.synchronize()
                res[k].append(a.elapsed_time(e) / 10)
        fl = 2.0 * M * N * K
        line = f"{name:14s} M={M:6d} K={K:5d} |"
        for k in variants:
            ms = float(np.median(res[k]))
            line += f" {k}: {ms * 1e3:7.1f}us {fl / ms / 1e9:5.0f}TF |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
