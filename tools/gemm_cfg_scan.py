"""Per-shape time of every bf16 GEMM tile configuration (PFM_GEMM_CFG, read per C-ABI call):
python tools/gemm_cfg_scan.py [cfg ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd import runtime as rt  # noqa: E402
from tools.gemm_bench import tm  # noqa: E402

SHAPES = [("dq", 14784, 512, 512), ("dffn1", 14784, 2048, 512), ("dffn2", 14784, 512, 2048),
          ("out", 32000, 512, 512), ("qkv", 32000, 1536, 512),
          ("dq/2", 7392, 512, 512), ("dffn1/2", 7392, 2048, 512), ("dffn2/2", 7392, 512, 2048)]
# EXACT mode (split-bf16 x6) GEMMs of one encoder group: K' = 6K
X6_SHAPES = [("x6qkv", 16000, 1536, 3072), ("x6w1", 16000, 2048, 3072), ("x6out", 16000, 512, 3072),
             ("x6w2", 16000, 512, 12288), ("x6kv", 32000, 16384, 3072)]
if os.environ.get("SCAN_X6"):
    SHAPES = X6_SHAPES
if os.environ.get("SCAN_GROUP"):   # fast-mode GEMMs of one encoder group (two groups run concurrently)
    SHAPES = [("qkv/2", 16000, 1536, 512), ("kv", 32000, 16384, 512), ("qkv0/2", 16000, 1536, 576)]


def main():
    cfgs = [int(c) for c in sys.argv[1:]] or [0, 1, 2, 3, 4, 10, 11, 12, 15, 16, 17]
    dev = torch.device("cuda", 0)
    for name, M, N, K in SHAPES:
        torch.manual_seed(0)
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        fl = 2.0 * M * N * K
        row = []
        for c in cfgs:
            os.environ["PFM_GEMM_CFG"] = str(c)
            try:
                ms = tm(lambda: rt.op_gemm(A, W, out_bf16=True))
                row.append(f"c{c}:{ms * 1e3:6.1f}us/{fl / ms / 1e9:5.0f}TF")
            except Exception as e:  # noqa: BLE001
                row.append(f"c{c}:err")
        print(f"{name:6s} M={M} N={N} K={K}  " + "  ".join(row), flush=True)
    os.environ.pop("PFM_GEMM_CFG", None)


if __name__ == "__main__":
    main()
