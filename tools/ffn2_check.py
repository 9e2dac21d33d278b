"""Where does the 128-row fused FFN (k_ffn2.hip) differ from fp64? Per 32-column output block and per 32-row lane
group, the max abs error of x2 for the plain (MODE 0) and out-projection (MODE 1) entries:
python tools/ffn2_check.py [M ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PFM_FFN_KERNEL"] = "2"
from funasr_amd import runtime as rt  # noqa: E402


def ln64(x, g, b, eps=1e-12):
    x = x.double()
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * g.double() + b.double()


def ffn_ref(x1, g2, b2n, W1, b1, W2, b2):
    a = ln64(x1, g2, b2n).bfloat16().double()
    h = torch.relu(a @ W1.double().T + b1.double()).bfloat16().double()
    return x1 + h @ W2.double().T + b2.double()


def report(tag, got, want):
    err = (got.double().cpu() - want).abs()
    M = err.shape[0]
    blk = err.reshape(M, 16, 32).amax(-1)          # [M, 16 blocks]
    print(f"{tag}: max {err.max().item():.3e}; bad blocks (max > 0.05):",
          [(int(r), int(c)) for r, c in (blk > 0.05).nonzero()[:12].tolist()], "count", int((blk > 0.05).sum()))
    rows = (blk > 0.05).any(-1).nonzero().flatten().tolist()
    print(f"   bad rows {len(rows)}: {rows[:20]}")


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [64, 200, 4100]
    g = torch.Generator().manual_seed(0)
    dev = torch.device("cuda", 0)
    W1 = torch.randn(2048, 512, generator=g) / 512 ** 0.5
    W2 = torch.randn(512, 2048, generator=g) / 2048 ** 0.5
    Wo = torch.randn(512, 512, generator=g) / 512 ** 0.5
    v = lambda n, s=0.1: s * torch.randn(n, generator=g)  # noqa: E731
    g2, b2n, b1, b2, gn, bn, bo = 1 + v(512), v(512), v(2048), v(512), 1 + v(512), v(512), v(512)
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    for M in Ms:
        x = torch.randn(M, 512, generator=g) * 2
        y, _ = rt.op_ffn(d(x), d(g2), d(b2n), 1e-12, d(W1), d(b1), d(W2), d(b2), d(gn), d(bn))
        torch.cuda.synchronize()
        report(f"M={M} MODE0", y, ffn_ref(x.double(), g2, b2n, W1.bfloat16(), b1, W2.bfloat16(), b2))
        o = torch.randn(M, 512, generator=g).bfloat16()
        f = (0.5 * torch.randn(M, 512, generator=g)).bfloat16()
        x2, _ = rt.op_ffn_op(d(o), d(f), d(Wo), d(bo), d(x), d(g2), d(b2n), 1e-12, d(W1), d(b1), d(W2), d(b2), d(gn),
                             d(bn))
        torch.cuda.synchronize()
        x1 = o.double() @ Wo.bfloat16().double().T + bo.double() + f.double() + x.double()
        report(f"M={M} MODE1", x2, ffn_ref(x1, g2, b2n, W1.bfloat16(), b1, W2.bfloat16(), b2))


if __name__ == "__main__":
    main()
