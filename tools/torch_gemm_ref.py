"""Library GEMM reference timings (torch.matmul -> hipBLASLt on ROCm) for the bf16 shapes the fast path runs,
to size the headroom of k_gemm_bf16.hip. HIP events, warm runs. usage: python tools/torch_gemm_ref.py"""
import torch


def main():
    dev = torch.device("cuda")
    shapes = [(16000, 1536, 512), (32000, 1536, 512), (16000, 512, 512), (16000, 2048, 512), (32000, 16384, 512),
              (14750, 8404, 512), (16000, 512, 2048)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev).bfloat16()
        b = torch.randn(N, K, device=dev).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        for name, fn in (("mm", lambda: a @ b.T), ("addmm", lambda: torch.addmm(bias, a, b.T))):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            s.record()
            for _ in range(reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1000 / reps
            print(f"M={M:6d} N={N:6d} K={K:5d} {name:5s}: {us:8.1f} us  {2.0 * M * N * K / us / 1e6:7.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
