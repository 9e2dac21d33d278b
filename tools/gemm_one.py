"""Run one bf16 GEMM shape through pfm_op_gemm repeatedly (for rocprofv3 --pmc passes).
usage: python tools/gemm_one.py M N K [iters] [relu] [bf16out]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from funasr_amd import runtime as rt


def main():
    M, N, K = (int(x) for x in sys.argv[1:4])
    it = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).bfloat16()
    W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    for _ in range(it):
        rt.op_gemm(A, W, out_bf16=N != 512)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
