"""Drive the fused encoder FFN kernel alone (pfm_op_ffn) for PMC / kernel-trace passes:
python tools/ffn_one.py [M] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from funasr_amd import runtime as rt  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, 512, generator=g, device=dev)
    W1 = torch.randn(2048, 512, generator=g, device=dev) / 512 ** 0.5
    W2 = torch.randn(512, 2048, generator=g, device=dev) / 2048 ** 0.5
    v = lambda n: torch.randn(n, generator=g, device=dev) * 0.1  # noqa: E731
    ones = torch.ones(512, device=dev)
    for _ in range(reps):
        rt.op_ffn(x, ones, v(512), 1e-12, W1, v(2048), W2, v(512), ones, v(512))
    torch.cuda.synchronize()
    print("ok", M, reps)


if __name__ == "__main__":
    main()
