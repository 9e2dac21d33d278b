"""Kernel-level numerics on the MI355X: each HIP op (through the C-ABI pfm_op_* entry points)
against a plain PyTorch reference of the same op (fp64 on CPU; tolerances stated per test)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from funasr_amd import runtime as rt  # noqa: E402
from oracle import paraformer_ref as ref  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rt.load_library()
    return torch.device("cuda", 0)


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize("M,N,K", [(300, 1536, 560), (128, 512, 512), (77, 8404, 512), (1000, 512, 2048),
                                   (5, 2048, 512), (129, 1024, 1536)])
def test_gemm_f32(dev, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    want = torch.relu(A.double() @ W.double().T + b.double()) + R.double()
    got = rt.op_gemm(A.to(dev), W.to(dev), b.to(dev), R.to(dev), relu=True)
    torch.cuda.synchronize()
    # exact f32 MFMA chain: error ~ K * 2^-24 relative to sum |a||w|
    assert rel(got, want) < 2e-6
    err = (got.double().cpu() - want).abs().max().item()
    assert err < 1e-4


@pytest.mark.parametrize("cfg", ["0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13", "14", "15", "16", "17"])
@pytest.mark.parametrize("M,N,K", [(300, 1536, 560), (77, 8404, 512), (1000, 512, 2048), (513, 1024, 1536),
                                   (256, 256, 64), (4000, 2048, 512), (2000, 768, 96), (600, 256, 32)])
@pytest.mark.parametrize("epi", ["none", "bias_res", "bias_res_nobatch", "bias_relu_res", "bias_relu_bf16"])
def test_gemm_bf16(dev, M, N, K, cfg, epi, monkeypatch):
    """Every bf16 tile configuration (PFM_GEMM_CFG, read per launch; 0 = automatic policy), including
    K-tile counts below the pipeline depth (K = 32, 64, 96), and the epilogue variants: bias + residual
    (batched or interleaved residual loads) and bias + relu + residual."""
    monkeypatch.setenv("PFM_GEMM_CFG", cfg)
    if epi == "bias_res_nobatch":    # residual loads interleaved with the stores
        monkeypatch.setenv("PFM_GEMM_RESBATCH", "0")
    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, K, generator=g).bfloat16()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, generator=g) if epi != "none" else None
    R = torch.randn(M, N, generator=g) if epi.startswith("bias_res") or epi == "bias_relu_res" else None
    want = A.double() @ W.double().T          # products of bf16 values are exact; f32 accumulate
    if b is not None:
        want = want + b.double()
    if epi in ("bias_relu_res", "bias_relu_bf16"):
        want = torch.relu(want)
    if R is not None:
        want = want + R.double()
    got = rt.op_gemm(A.to(dev), W.to(dev), None if b is None else b.to(dev), None if R is None else R.to(dev),
                     relu=epi in ("bias_relu_res", "bias_relu_bf16"), out_bf16=epi == "bias_relu_bf16")
    torch.cuda.synchronize()
    if epi == "bias_relu_bf16":   # f32 accumulate, one bf16 rounding of the output (rel 2^-9 per element)
        assert rel(got, want) < 4e-3
        assert torch.equal(got.cpu(), want.float().bfloat16()) or rel(got, want.float().bfloat16()) < 1e-3
    else:
        assert rel(got, want) < 1e-5


@pytest.mark.parametrize("M,N,K", [(1, 512, 512), (15, 1536, 512), (15, 512, 2048), (16, 2048, 512),
                                   (17, 1024, 1536), (33, 512, 512), (64, 520, 96), (7, 8, 32),
                                   (960, 512, 2048), (961, 1536, 512), (200, 48, 64)])
@pytest.mark.parametrize("epi", ["none", "bias_res", "bias_relu_bf16"])
def test_gemm_bf16_skinny(dev, M, N, K, epi, monkeypatch):
    """M <= 64 rows (and few-tile shapes above: M 200 / 960 / 961) take the weight-streaming kernel
    (k_gemm_skinny.hip); same epilogues and tolerance as the tiled kernels, and the tiled kernel's result
    up to f32 summation order."""
    g = torch.Generator().manual_seed(M * 31 + N)
    A = torch.randn(M, K, generator=g).bfloat16()
    W = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, generator=g) if epi != "none" else None
    R = torch.randn(M, N, generator=g) if epi == "bias_res" else None
    want = A.double() @ W.double().T
    if b is not None:
        want = want + b.double()
    if epi == "bias_relu_bf16":
        want = torch.relu(want)
    if R is not None:
        want = want + R.double()
    args = (A.to(dev), W.to(dev), None if b is None else b.to(dev), None if R is None else R.to(dev))
    kw = dict(relu=epi == "bias_relu_bf16", out_bf16=epi == "bias_relu_bf16")
    got = rt.op_gemm(*args, **kw)
    monkeypatch.setenv("PFM_GEMM_SKINNY", "0")
    tiled = rt.op_gemm(*args, **kw)
    torch.cuda.synchronize()
    if epi == "bias_relu_bf16":
        assert rel(got, want) < 4e-3
        assert rel(got, tiled) < 1e-2
    else:
        assert rel(got, want) < 1e-5
        assert rel(got, tiled) < 1e-5


@pytest.mark.parametrize("M,N", [(1, 1536), (15, 1536), (15, 2048), (16, 512), (33, 2048), (64, 512), (65, 1536),
                                 (200, 512)])
@pytest.mark.parametrize("epi", ["bias_bf16", "bias_relu", "bias_res"])
def test_ln_gemm(dev, M, N, epi):
    """LayerNorm folded into the skinny GEMM's A load (streaming LN1 -> QKV, LN2 -> w1, decoder LN -> w1 / q;
    pfm_op_ln_gemm): against fp64 on the kernel's own bf16 rounding of LN(x) (rel-L2 < 1e-5 for f32 outputs, one bf16
    output rounding otherwise), and equal to the separate LayerNorm + GEMM of the unfused path (M > 64 takes that path
    itself) up to bf16 operand rounding flips."""
    g = torch.Generator().manual_seed(7 * M + N)
    X = torch.randn(M, 512, generator=g) * 3 + 0.5
    gm, bt = 1 + 0.1 * torch.randn(512, generator=g), 0.1 * torch.randn(512, generator=g)
    W = (torch.randn(N, 512, generator=g) / 512 ** 0.5).bfloat16()
    b = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g) if epi == "bias_res" else None
    ln = _ln64(X.double(), gm, bt, 1e-12).float().bfloat16()   # the kernel's bf16 A operand (f64 statistics)
    want = ln.double() @ W.double().T + b.double()
    if epi == "bias_relu":
        want = torch.relu(want)
    if R is not None:
        want = want + R.double()
    kw = dict(relu=epi == "bias_relu", out_bf16=epi == "bias_bf16")
    got = rt.op_ln_gemm(X.to(dev), gm.to(dev), bt.to(dev), 1e-12, W.to(dev), b.to(dev),
                        None if R is None else R.to(dev), **kw)
    sep = rt.op_gemm(rt.op_layernorm(X.to(dev), gm.to(dev), bt.to(dev), 1e-12).bfloat16(), W.to(dev), b.to(dev),
                     None if R is None else R.to(dev), **kw)
    torch.cuda.synchronize()
    tol = 4e-3 if epi == "bias_bf16" else 1e-5
    assert rel(got, want) < tol
    # the two paths round LN(x) to bf16 from f32 values formed in a different operation order: a last-bit
    # difference flips an operand element's bf16 rounding now and then (3e-5 measured at M = 64, N = 512)
    assert rel(got, sep) < (1e-2 if epi == "bias_bf16" else 2e-4)


def test_gemm_identity_asymmetric(dev):
    """A = I with an asymmetric W catches a transposed C write."""
    K = 256
    A = torch.eye(K)
    W = torch.arange(K * 160, dtype=torch.float32).reshape(160, K) % 97
    got = rt.op_gemm(A.to(dev), W.to(dev)).cpu()
    assert torch.equal(got, W.T.contiguous())


@pytest.mark.parametrize("dt", ["f32", "bf16", "bf16_w4"])
@pytest.mark.parametrize("B,Tq,Tk,lens", [(2, 500, 500, [500, 123]), (3, 37, 200, [1, 200, 64]),
                                          (1, 130, 33, [33]), (2, 231, 500, [500, 64]), (1, 300, 129, [0])])
def test_attention(dev, dt, B, Tq, Tk, lens, monkeypatch):
    """f32 / bf16 attention kernels (bf16: the 8-wave kernel of the path; bf16_w4: the 4-wave one)
    incl. ragged and empty key lengths; klen 0 gives zero rows."""
    if dt == "bf16_w4":
        monkeypatch.setenv("PFM_ATTN_WAVES", "4")
    H, dk = 4, 128
    g = torch.Generator().manual_seed(B * 1000 + Tq)
    q = torch.randn(B * Tq, H * dk, generator=g)
    k = torch.randn(B * Tk, H * dk, generator=g)
    v = torch.randn(B * Tk, H * dk, generator=g)
    klen = torch.tensor(lens, dtype=torch.int32)
    if dt != "f32":
        q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    if 0 in lens:   # empty utterance: the kernels write zeros (the reference masks everything -> nan-free 0)
        got = rt.op_attention(q.to(dev), k.to(dev), v.to(dev), klen.to(dev), B, Tq, Tk, H, dk ** -0.5)
        torch.cuda.synchronize()
        assert torch.all(got.cpu() == 0)
        return
    want = ref._attend(q.double().reshape(B, Tq, -1), k.double().reshape(B, Tk, -1), v.double().reshape(B, Tk, -1),
                       (torch.arange(Tk)[None] < klen[:, None]).double(), H).reshape(B * Tq, -1)
    got = rt.op_attention(q.to(dev), k.to(dev), v.to(dev), klen.to(dev), B, Tq, Tk, H, dk ** -0.5)
    torch.cuda.synchronize()
    # f32: exact-f32 products, online softmax; bf16: P and (scaled) q rounded to bf16
    assert rel(got, want) < (2e-6 if dt == "f32" else 1.5e-2)


@pytest.mark.parametrize("M,D", [(1000, 512), (37, 560), (64, 2048), (1, 512), (3, 1024), (77, 2048), (32001, 512)])
def test_layernorm(dev, M, D):
    g = torch.Generator().manual_seed(D)
    x = torch.randn(M, D, generator=g) * 3 + 1
    gm = 1 + 0.1 * torch.randn(D, generator=g)
    bt = 0.1 * torch.randn(D, generator=g)
    want = torch.nn.functional.layer_norm(x.double(), (D,), gm.double(), bt.double(), 1e-12)
    got = rt.op_layernorm(x.to(dev), gm.to(dev), bt.to(dev), 1e-12)
    torch.cuda.synchronize()
    assert (got.double().cpu() - want).abs().max().item() < 2e-6


@pytest.mark.parametrize("M,D", [(1, 512), (77, 2048), (14784, 2048), (5, 1024)])
def test_layernorm_bf16_input(dev, M, D):
    """bf16-input LayerNorm (decoder FFN hidden in fast mode) vs fp64 on the same bf16 values."""
    g = torch.Generator().manual_seed(D + M)
    x = (torch.randn(M, D, generator=g) * 3 + 1).bfloat16()
    gm = 1 + 0.1 * torch.randn(D, generator=g)
    bt = 0.1 * torch.randn(D, generator=g)
    want = torch.nn.functional.layer_norm(x.double(), (D,), gm.double(), bt.double(), 1e-12)
    got = rt.op_layernorm_bf16(x.to(dev), gm.to(dev), bt.to(dev), 1e-12)
    torch.cuda.synchronize()
    assert (got.double().cpu() - want).abs().max().item() < 2e-6


@pytest.mark.parametrize("B,T,lens,left", [(2, 50, [50, 17], 5), (1, 9, [9], 5), (3, 40, [1, 40, 11], 7)])
def test_fsmn(dev, B, T, lens, left):
    D, K = 512, 11
    g = torch.Generator().manual_seed(T)
    v = torch.randn(B * T, D, generator=g)
    w = torch.randn(D, 1, K, generator=g) / K ** 0.5
    res = torch.randn(B * T, D, generator=g)
    L = torch.tensor(lens, dtype=torch.int32)
    m = (torch.arange(T)[None] < L[:, None]).double()
    want = ref.fsmn(v.double().reshape(B, T, D), m, w.double(), left - (K - 1) // 2).reshape(B * T, D) + res.double()
    got = rt.op_fsmn(v.to(dev), L.to(dev), w.to(dev), B, T, left, res=res.to(dev))
    torch.cuda.synchronize()
    assert (got.double().cpu() - want).abs().max().item() < 1e-5


@pytest.mark.parametrize("B,T,lens,left", [(2, 50, [50, 17], 5), (1, 9, [9], 5), (3, 40, [1, 40, 11], 7),
                                           (4, 500, [500, 1, 250, 499], 5)])
def test_fsmn_bf16(dev, B, T, lens, left):
    """Fast-mode FSMN (bf16 in / bf16 out) vs fp64 on the same bf16 inputs: one bf16 output rounding, so
    rel-L2 <= 4e-3 and the padded rows exactly zero."""
    D, K = 512, 11
    g = torch.Generator().manual_seed(T + left)
    v = torch.randn(B * T, D, generator=g).bfloat16()
    w = torch.randn(D, 1, K, generator=g) / K ** 0.5
    L = torch.tensor(lens, dtype=torch.int32)
    m = (torch.arange(T)[None] < L[:, None]).double()
    want = ref.fsmn(v.double().reshape(B, T, D), m, w.double(), left - (K - 1) // 2).reshape(B * T, D)
    got = rt.op_fsmn_bf16(v.to(dev), L.to(dev), w.to(dev), B, T, left)
    torch.cuda.synchronize()
    got = got.double().cpu()
    assert rel(got, want) < 4e-3
    pad = (m.reshape(-1) == 0)
    assert torch.all(got[pad] == 0)


def test_cif_bit_exact(dev):
    """Integrate-and-fire: fire pattern, peaks and token counts bit-exact vs the torch restatement."""
    B, T, D = 3, 300, 512
    g = torch.Generator().manual_seed(3)
    h = torch.randn(B, T, D, generator=g)
    a = torch.sigmoid(torch.randn(B, T, generator=g))
    lens = torch.tensor([300, 211, 7])
    a = a * ref.pad_mask(lens, T)
    hh, aa, tn = ref.tail_process(h, a, lens, 0.45)
    want_emb, want_peak, want_nf = ref.cif(hh, aa, 1.0)
    emb, peaks, nf, nt = rt.op_cif(aa.contiguous().to(dev), hh.contiguous().to(dev), T + 1)
    torch.cuda.synchronize()
    assert torch.equal(nf.cpu().long(), want_nf.long())
    assert torch.equal(peaks.cpu(), want_peak)
    assert torch.equal(nt.cpu().long(), tn.long())
    L = want_emb.shape[1]
    assert torch.equal(emb.cpu()[:, :L], want_emb)
    assert float(emb.cpu()[:, L:].abs().max() if emb.shape[1] > L else 0.0) == 0.0


def _ffn_ref(x, g2, b2n, eps, W1b, b1, W2b, b2):
    """fp64 restatement of the fused FFN sub-layer on the kernel's bf16 operand roundings:
    A = bf16(LN2(x)), H = bf16(relu(A W1^T + b1)), y = x + H W2^T + b2."""
    xd = x.double()
    mu = xd.mean(-1, keepdim=True)
    var = ((xd - mu) ** 2).mean(-1, keepdim=True)
    a = ((xd - mu) / torch.sqrt(var + eps) * g2.double() + b2n.double()).bfloat16().double()
    h = torch.relu(a @ W1b.double().T + b1.double()).bfloat16().double()
    return xd + h @ W2b.double().T + b2.double()


@pytest.mark.parametrize("M", [64, 200, 1000])
@pytest.mark.parametrize("with_next", [False, True])
@pytest.mark.parametrize("hr", ["k1", "k2"])
def test_ffn_fused(dev, M, with_next, hr, monkeypatch):
    """Fused LN2 -> W1 -> relu -> W2 -> residual (-> next LN, bf16) vs fp64 torch on the same bf16 weights:
    FFN increment (y - x) within rel-L2 5e-3 (f32 accumulation order flips a few bf16 roundings of the
    hidden activation), y within rel 1e-4; the next-layer LayerNorm of the kernel's own y within 1.6e-2
    abs (one bf16 ulp at |v| <= 4); rows beyond M untouched by construction (ragged M). Both kernels: the
    64-row k_ffn.hip (k1) and the 128-row k_ffn2.hip (k2)."""
    monkeypatch.setenv("PFM_FFN_KERNEL", "2" if hr == "k2" else "1")
    g = torch.Generator().manual_seed(M + 7 * with_next)
    x = torch.randn(M, 512, generator=g) * 2
    g2 = 1 + 0.1 * torch.randn(512, generator=g)
    b2n = 0.1 * torch.randn(512, generator=g)
    W1 = torch.randn(2048, 512, generator=g) / 512 ** 0.5
    b1 = 0.1 * torch.randn(2048, generator=g)
    W2 = torch.randn(512, 2048, generator=g) / 2048 ** 0.5
    b2 = 0.1 * torch.randn(512, generator=g)
    gn = 1 + 0.1 * torch.randn(512, generator=g) if with_next else None
    bn = 0.1 * torch.randn(512, generator=g) if with_next else None
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    y, xn = rt.op_ffn(d(x), d(g2), d(b2n), 1e-12, d(W1), d(b1), d(W2), d(b2), d(gn), d(bn))
    torch.cuda.synchronize()
    want = _ffn_ref(x, g2, b2n, 1e-12, W1.bfloat16(), b1, W2.bfloat16(), b2)
    yc = y.double().cpu()
    assert rel(yc - x.double(), want - x.double()) < 5e-3
    assert rel(yc, want) < 1e-4
    if with_next:
        mu = yc.mean(-1, keepdim=True)
        var = ((yc - mu) ** 2).mean(-1, keepdim=True)
        ln = (yc - mu) / torch.sqrt(var + 1e-12) * gn.double() + bn.double()
        assert (xn.double().cpu() - ln).abs().max().item() < 1.6e-2
    else:
        assert xn is None


def _ln64(x, g, b, eps):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * g.double() + b.double()


def _ffn_params(g, dec=False):
    p = dict(W1=torch.randn(2048, 512, generator=g) / 512 ** 0.5, b1=0.1 * torch.randn(2048, generator=g),
             W2=torch.randn(512, 2048, generator=g) / 2048 ** 0.5, g2=1 + 0.1 * torch.randn(512, generator=g),
             b2n=0.1 * torch.randn(512, generator=g), gn=1 + 0.1 * torch.randn(512, generator=g),
             bn=0.1 * torch.randn(512, generator=g), Wo=torch.randn(512, 512, generator=g) / 512 ** 0.5,
             bo=0.1 * torch.randn(512, generator=g))
    if dec:
        p.update(gF=1 + 0.1 * torch.randn(2048, generator=g), bF=0.1 * torch.randn(2048, generator=g))
    else:
        p.update(b2=0.1 * torch.randn(512, generator=g))
    return p


@pytest.mark.parametrize("kern", ["1", "2"])
@pytest.mark.parametrize("M", [64, 200, 1000, 4100])
@pytest.mark.parametrize("resid", [True, False])
@pytest.mark.parametrize("eps", [1e-12, 1e-5])
def test_ffn_fused_outproj(dev, M, resid, kern, eps, monkeypatch):
    """The encoder sub-layer tail exactly as the fast path's default dispatch runs it (ffn_fused_kernel OP mode:
    out-projection as phase 0, x1 in the accumulators, LN2 reduced across waves, FFN, next LN1) vs an fp64
    restatement of sanm/encoder.py:120-145 on the kernel's bf16 operand roundings:
      x1 = x + (o Wo^T + bo + f)   (layer 0: no x),  a = bf16(LN2(x1)),  h = bf16(relu(a W1^T + b1)),
      x2 = x1 + h W2^T + b2,  xn = LN1_next(x2).
    Tolerances: the FFN increment x2 - x1 rel-L2 < 5e-3 (f32 accumulation order flips a few bf16 roundings of
    a / h), x2 rel < 1e-4, xn within 1.6e-2 abs of LN1_next of the kernel's own x2 (one bf16 ulp at |v| <= 4).
    Both fused kernels: k_ffn.hip (64 rows per workgroup, PFM_FFN_KERNEL=1) and k_ffn2.hip (128, the default); LN eps
    1e-12 (Paraformer) and 1e-5 (SenseVoiceSmall, BASELINE C4)."""
    monkeypatch.setenv("PFM_FFN_KERNEL", kern)
    g = torch.Generator().manual_seed(31 * M + resid)
    p = _ffn_params(g)
    x = torch.randn(M, 512, generator=g) * 2 if resid else None
    o = torch.randn(M, 512, generator=g).bfloat16()
    f = (0.5 * torch.randn(M, 512, generator=g)).bfloat16()
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    x2, xn = rt.op_ffn_op(d(o), d(f), d(p["Wo"]), d(p["bo"]), d(x), d(p["g2"]), d(p["b2n"]), eps, d(p["W1"]),
                          d(p["b1"]), d(p["W2"]), d(p["b2"]), d(p["gn"]), d(p["bn"]))
    torch.cuda.synchronize()
    x1 = o.double() @ p["Wo"].bfloat16().double().T + p["bo"].double() + f.double()
    if resid:
        x1 = x1 + x.double()
    want = _ffn_ref(x1, p["g2"], p["b2n"], eps, p["W1"].bfloat16(), p["b1"], p["W2"].bfloat16(), p["b2"])
    yc = x2.double().cpu()
    assert rel(yc - x1, want - x1) < 5e-3
    assert rel(yc, want) < 1e-4
    ln = _ln64(yc, p["gn"], p["bn"], eps)
    assert (xn.double().cpu() - ln).abs().max().item() < 1.6e-2


@pytest.mark.parametrize("M", [64, 200, 4100])
@pytest.mark.parametrize("eps", [1e-12, 1e-5])
def test_ffn_fused_outproj_qkv(dev, M, eps):
    """The 128-row kernel's MODE 4 (k_ffn2.hip): the encoder sub-layer tail of test_ffn_fused_outproj and then the
    NEXT layer's q|k|v = LN1_next(x2) Wq^T + bq (attention.py:180-186 on its norm1) from the LayerNorm output held in
    registers, vs fp64 on the kernel's own f32 x2 and the bf16 rounding of LN1_next(x2): qkv rel-L2 < 5e-3 (bf16
    output), x2 as test_ffn_fused_outproj. eps 1e-5 is SenseVoiceSmall's LayerNorm (sense_voice/model.py)."""
    g = torch.Generator().manual_seed(13 * M + int(eps == 1e-5))
    p = _ffn_params(g)
    Wq, bq = torch.randn(1536, 512, generator=g) / 512 ** 0.5, 0.1 * torch.randn(1536, generator=g)
    x = torch.randn(M, 512, generator=g) * 2
    o = torch.randn(M, 512, generator=g).bfloat16()
    f = (0.5 * torch.randn(M, 512, generator=g)).bfloat16()
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    x2, qkv = rt.op_ffn_op_qkv(d(o), d(f), d(p["Wo"]), d(p["bo"]), d(x), d(p["g2"]), d(p["b2n"]), eps, d(p["W1"]),
                               d(p["b1"]), d(p["W2"]), d(p["b2"]), d(p["gn"]), d(p["bn"]), d(Wq), d(bq))
    torch.cuda.synchronize()
    x1 = o.double() @ p["Wo"].bfloat16().double().T + p["bo"].double() + f.double() + x.double()
    want = _ffn_ref(x1, p["g2"], p["b2n"], eps, p["W1"].bfloat16(), p["b1"], p["W2"].bfloat16(), p["b2"])
    yc = x2.double().cpu()
    assert rel(yc - x1, want - x1) < 5e-3
    assert rel(yc, want) < 1e-4
    a = _ln64(yc, p["gn"], p["bn"], eps).bfloat16().double()
    qw = a @ Wq.bfloat16().double().T + bq.double()
    assert rel(qkv.double().cpu(), qw) < 5e-3


@pytest.mark.parametrize("M", [200, 4100])
@pytest.mark.parametrize("xw", [4, 8])
def test_ffn_fused_outproj_qkv_split_v(dev, monkeypatch, M, xw):
    """MODE 5 (PFM_FAST_XW bit 4): MODE 4 with the v rows of Wq as two bf16 planes w0 + w1 (~2^-17 relative).
    q | k as MODE 4 (bf16 weights); v within the bf16 output's rounding of fp64 with the f32 weights, and clearly
    closer to it than to the bf16-weight product (the lo plane is applied). MODE 6 (bit 8): Wo split too -- x2
    within 1e-4 of fp64 with the f32 Wo (the f32 residual stream shows the out-projection's precision)."""
    monkeypatch.setenv("PFM_FAST_XW", str(xw))
    g = torch.Generator().manual_seed(29 * M)
    p = _ffn_params(g)
    Wq, bq = torch.randn(1536, 512, generator=g) / 512 ** 0.5, 0.1 * torch.randn(1536, generator=g)
    x = torch.randn(M, 512, generator=g) * 2
    o = torch.randn(M, 512, generator=g).bfloat16()
    f = (0.5 * torch.randn(M, 512, generator=g)).bfloat16()
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    x2, qkv = rt.op_ffn_op_qkv(d(o), d(f), d(p["Wo"]), d(p["bo"]), d(x), d(p["g2"]), d(p["b2n"]), 1e-12, d(p["W1"]),
                               d(p["b1"]), d(p["W2"]), d(p["b2"]), d(p["gn"]), d(p["bn"]), d(Wq), d(bq))
    torch.cuda.synchronize()
    if xw & 8:
        x1 = o.double() @ p["Wo"].double().T + p["bo"].double() + f.double() + x.double()
        want = _ffn_ref(x1, p["g2"], p["b2n"], 1e-12, p["W1"].bfloat16(), p["b1"], p["W2"].bfloat16(), p["b2"])
        x1b = o.double() @ p["Wo"].bfloat16().double().T + p["bo"].double() + f.double() + x.double()
        assert rel(x2.double().cpu(), want) < 1e-4
        assert rel(x2.double().cpu() - x1b, want - x1b) < 5e-3 and rel(x1, x1b) > 1e-4
    a = _ln64(x2.double().cpu(), p["gn"], p["bn"], 1e-12).bfloat16().double()
    got = qkv.double().cpu()
    qk_bf = a @ Wq[:1024].bfloat16().double().T + bq[:1024].double()
    assert rel(got[:, :1024], qk_bf) < 5e-3
    v_exact = a @ Wq[1024:].double().T + bq[1024:].double()
    v_bf = a @ Wq[1024:].bfloat16().double().T + bq[1024:].double()
    e_exact, e_bf = rel(got[:, 1024:], v_exact), rel(got[:, 1024:], v_bf)
    print(f"MODE 5 v rows: rel-L2 vs f32 weights {e_exact:.2e}, vs bf16 weights {e_bf:.2e}")
    assert e_exact < 5e-3 and e_exact < 0.85 * e_bf


@pytest.mark.parametrize("M,N,K", [(100, 512, 576), (4096, 1536, 512), (777, 512, 2048)])
def test_gemm_split_weights(dev, M, N, K):
    """The split-weight GEMM (x6_terms 2: bf16 A times w = w0 + w1, two bf16 planes) vs fp64 of the same operands:
    the products are exact, so rel < 1e-5 (f32 accumulation); relu + bias and the residual epilogue."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).bfloat16()
    W = torch.randn(N, K, generator=g) / K ** 0.5
    w0 = W.bfloat16()
    w1 = (W - w0.float()).bfloat16()
    bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
    C = rt.op_gemm(A.to(dev), torch.stack([w0, w1]).to(dev), bias=bias.to(dev), res=res.to(dev), relu=True)
    torch.cuda.synchronize()
    want = torch.relu(A.double() @ (w0.double() + w1.double()).T + bias.double()) + res.double()
    assert rel(C.double().cpu(), want) < 1e-5


def _dec_ffn_ref(x1, p, eps=1e-12):
    """fp64 sanm/positionwise_feed_forward.py:26-33 on the kernel's roundings: a = bf16(LN1(x1)),
    h = bf16(relu(a W1^T + b1)); LN_F over the 2048 hidden folded through W2 with W2g = bf16(W2 diag(gamma_F)):
    y = rstd (h W2g^T - mu rowsum(W2g)) + W2 beta_F (= W2 LN_F(h) up to the rounding of W2 gamma_F)."""
    a = _ln64(x1, p["g2"], p["b2n"], eps).bfloat16().double()
    h = torch.relu(a @ p["W1"].bfloat16().double().T + p["b1"].double()).bfloat16().double()
    mu = h.mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(((h - mu) ** 2).mean(-1, keepdim=True) + eps)
    w2g = (p["W2"] * p["gF"][None, :]).bfloat16().double()
    y = rstd * (h @ w2g.T - mu * w2g.sum(-1)[None, :]) + (p["W2"].double() @ p["bF"].double())[None, :]
    exact = (_ln64(h, p["gF"], p["bF"], eps)) @ p["W2"].double().T   # no W2 / gamma rounding
    return y, exact


@pytest.mark.parametrize("kernel", ["1", "2", "3"])
@pytest.mark.parametrize("M", [64, 200, 1000, 4100])
@pytest.mark.parametrize("outproj", [False, True])
def test_ffn_fused_decoder(dev, monkeypatch, M, outproj, kernel):
    """The decoder FFN exactly as the fast path runs it (kernel 1: k_ffn.hip's 64-row DEC mode; kernel 2, the default:
    k_ffn2.hip MODE 7 / 8, 128-row tiles with the hidden split over two workgroups that combine their partials
    through a tile counter: LN1 prologue, LN_F folded through W2, next LayerNorm epilogue; with outproj the previous
    block's cross-attention out-projection as phase 0, x1 = x + o Wo^T + bo written back) vs fp64 on the kernel's
    bf16 roundings: y rel-L2 < 5e-3 (and < 2e-2 vs the unrounded W2 LN_F(h)), xn within 1e-2 of LN_next of the fp64
    y; x1 rel < 1e-6. M = 200 / 1000 / 4100 leave partial tiles and grid padding (tiles past M)."""
    monkeypatch.setenv("PFM_DEC_FFN_FUSED", kernel)
    g = torch.Generator().manual_seed(17 * M + outproj)
    p = _ffn_params(g, dec=True)
    x = torch.randn(M, 512, generator=g) * 2
    o = torch.randn(M, 512, generator=g).bfloat16() if outproj else None
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    xo, xn = rt.op_ffn_dec(d(x), d(p["g2"]), d(p["b2n"]), 1e-12, d(p["W1"]), d(p["b1"]), d(p["W2"]), d(p["gF"]),
                           d(p["bF"]), d(p["gn"]), d(p["bn"]), d(o), d(p["Wo"] if outproj else None),
                           d(p["bo"] if outproj else None))
    torch.cuda.synchronize()
    x1 = x.double()
    if outproj:
        x1 = x1 + o.double() @ p["Wo"].bfloat16().double().T + p["bo"].double()
        assert rel(xo.double().cpu(), x1) < 1e-6
        x1 = xo.double().cpu()   # the FFN runs on the kernel's own f32 x1
    y, exact = _dec_ffn_ref(x1, p)
    if not outproj:
        yc = xo.double().cpu()
        assert rel(yc, y) < 5e-3
        assert rel(yc, exact) < 2e-2
    ln = _ln64(y, p["gn"], p["bn"], 1e-12)
    assert rel(xn.double().cpu(), ln) < 1e-2
    assert (xn.double().cpu() - ln).abs().max().item() < 0.1
