"""Fixed (prologue + epilogue) vs per-K-step cost of the bf16 GEMM: time M x N x K for a K sweep at the
path's M / N (one tile round for N=512). usage: python tools/gemm_kscan.py [M] [N] [cfg...]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from funasr_amd import runtime as rt


def tm(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 32000
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    cfgs = sys.argv[3:] or ["0"]
    dev = torch.device("cuda", 0)
    for cfg in cfgs:
        os.environ["PFM_GEMM_CFG"] = cfg
        for K in [64, 128, 256, 512, 1024, 2048]:
            A = torch.randn(M, K, device=dev).bfloat16()
            W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
            res = torch.randn(M, N, device=dev)
            t0 = tm(lambda: rt.op_gemm(A, W, out_bf16=True))
            t1 = tm(lambda: rt.op_gemm(A, W))
            t2 = tm(lambda: rt.op_gemm(A, W, res=res))
            fl = 2.0 * M * N * K
            print(f"cfg {cfg} M={M} N={N} K={K:5d}  bf16-out {t0:7.1f} us  f32-out {t1:7.1f} us  f32+res {t2:7.1f} us"
                  f"  ({fl / t1 / 1e6:6.1f} TF f32-out)", flush=True)


if __name__ == "__main__":
    main()
