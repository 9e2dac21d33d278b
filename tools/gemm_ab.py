"""In-process interleaved A/B of bf16 GEMM tile configs (PFM_GEMM_CFG read per launch) on the path's
shapes; N=512 shapes carry an f32 residual like the out-proj / FFN2 epilogues. Median of rounds."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from funasr_amd import runtime as rt

SHAPES_ALL = [("qkv", 32000, 1536, 512), ("out+res", 32000, 512, 512), ("ffn1", 32000, 2048, 512),
          ("ffn2+res", 32000, 512, 2048), ("conv", 32000, 512, 1536), ("kv_all", 32000, 16384, 512),
          ("dffn1", 14784, 2048, 512), ("dffn2+res", 14784, 512, 2048), ("dq", 14784, 512, 512),
          ("vocab", 14784, 8404, 512), ("sq4k", 4096, 4096, 4096)]
SHAPES = [x for x in SHAPES_ALL if not os.environ.get("AB_SHAPES") or x[0] in os.environ["AB_SHAPES"].split(",")]
# tokens: "<cfg>" or "<cfg>:VAR=VAL" (extra env for that arm, e.g. 4:PFM_GEMM_ST16=0)
CFGS = (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4,5").split(",")


def arm_env(tok):
    cfg, _, extra = tok.partition(":")
    env = {"PFM_GEMM_CFG": cfg}
    if extra:
        k, _, v = extra.partition("=")
        env[k] = v
    return env


def main():
    dev = torch.device("cuda", 0)
    ev = lambda: torch.cuda.Event(enable_timing=True)
    for name, M, N, K in SHAPES:
        torch.manual_seed(0)
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        R = torch.randn(M, N, device=dev) if "res" in name else None
        b = torch.randn(N, device=dev)
        fl = 2.0 * M * N * K
        res = {c: [] for c in CFGS}
        for rnd in range(5):
            for c in CFGS:
                env = arm_env(c)
                os.environ.update(env)
                bf = R is None and N != 512            # QKV / FFN1 / KV: bf16 outputs on the path
                rt.op_gemm(A, W, b, R, out_bf16=bf)
                a, e = ev(), ev()
                a.record()
                for _ in range(10):
                    rt.op_gemm(A, W, b, R, out_bf16=bf)
                e.record()
                torch.cuda.synchronize()
                res[c].append(a.elapsed_time(e) / 10)
                for k in env:
                    if k != "PFM_GEMM_CFG":
                        os.environ.pop(k)
        line = f"{name:10s} M={M:6d} N={N:6d} K={K:5d} |"
        for c in CFGS:
            ms = float(np.median(res[c]))
            line += f" {c}: {ms*1e3:7.1f}us {fl/ms/1e9:6.0f}TF |"
        print(line, flush=True)


if __name__ == "__main__":
    main()
