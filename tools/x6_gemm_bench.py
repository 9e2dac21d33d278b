"""EXACT mode's split-bf16 x6 GEMM (pfm_op_gemm on f32 operands: six bf16 products, f32 accumulate) against
hipBLASLt (torch.matmul) on a plain bf16 GEMM of the same issued work (K' = 6 K), per projection shape of the
Paraformer-large path at B = 64 x 500 (M = 32000) and the decoder (M = 14784)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from funasr_amd import runtime as rt  # noqa: E402

SHAPES = [("qkv", 32000, 1536, 512), ("out", 32000, 512, 512), ("ffn1", 32000, 2048, 512),
          ("ffn2", 32000, 512, 2048), ("kv_grp", 32000, 4096, 512), ("dffn1", 14784, 2048, 512),
          ("dffn2", 14784, 512, 2048)]


def tm(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    dev = torch.device("cuda", 0)
    for name, M, N, K in SHAPES:
        torch.manual_seed(0)
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) / K ** 0.5
        fl6 = 2.0 * M * N * K * 6
        ms = tm(lambda: rt.op_gemm(A, W))
        A6 = torch.randn(M, 6 * K, device=dev).bfloat16()
        W6 = torch.randn(N, 6 * K, device=dev).bfloat16()
        ms_t = tm(lambda: torch.matmul(A6, W6.t()))
        print(f"{name:7s} M={M:6d} N={N:5d} K={K:5d}  x6 {ms*1e3:8.1f} us {fl6/ms/1e9:7.1f} TF issued   "
              f"hipBLASLt bf16 K'={6*K} {ms_t*1e3:8.1f} us {fl6/ms_t/1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
