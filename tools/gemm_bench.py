"""Per-shape GEMM throughput on the GPU: pfm kernels (via pfm_op_gemm) vs torch.matmul (hipBLASLt).
Shapes = the fast-mode Paraformer-large path at B=64, T=500 (M=32000) and decoder M=64*231."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from funasr_amd import runtime as rt

SHAPES = [("qkv", 32000, 1536, 512), ("out", 32000, 512, 512), ("ffn1", 32000, 2048, 512),
          ("ffn2", 32000, 512, 2048), ("conv", 32000, 512, 1536), ("kv_all", 32000, 16384, 512), ("kv_grp", 32000, 4096, 512),
          ("dffn1", 14784, 2048, 512), ("dffn2", 14784, 512, 2048), ("dq", 14784, 512, 512),
          ("vocab", 14784, 8404, 512), ("sq4k", 4096, 4096, 4096)]


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
    return a.elapsed_time(b) / it


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    dev = torch.device("cuda", 0)
    res = []
    for name, M, N, K in SHAPES:
        torch.manual_seed(0)
        ty = torch.bfloat16 if dt == "bf16" else torch.float32
        A = torch.randn(M, K, device=dev).to(ty)
        W = (torch.randn(N, K, device=dev) / K ** 0.5).to(ty)
        C = torch.empty(M, N, device=dev)
        fl = 2.0 * M * N * K
        ms = tm(lambda: rt.op_gemm(A, W, out_bf16=(dt == "bf16")))
        ms_t = tm(lambda: torch.matmul(A, W.t()))
        print(f"{name:7s} M={M:6d} N={N:6d} K={K:5d}  pfm {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF   "
              f"torch {ms_t*1e3:8.1f} us {fl/ms_t/1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
