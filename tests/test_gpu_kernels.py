"""Parity of each libllp_hip kernel against the CPU oracle / a torch fp32
reference of the same op.  Run on the MI355X: pytest -m gpu."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import llp_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_hip
    llp_hip.lib()


def K():
    import llp_hip
    return llp_hip


def _bf(t):
    return t.to(torch.bfloat16).float()


# ------------------------------------------------------------------ GEMM NT
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N,Kd", [(300, 70, 37), (1000, 256, 128), (129, 128, 64), (64, 1, 16), (5, 300, 520)])
def test_gemm_nt(dt, M, N, Kd):
    k = K()
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(M, Kd, generator=g)
    W = torch.randn(N, Kd, generator=g) * 0.1
    b = torch.randn(N, generator=g)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    Ad, Wd = A.to(DEV, tdt), W.to(DEV, tdt)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    k.gemm_nt(k.operand(Ad), k.operand(Wd), M, N, Kd, out, k.dtype_code(tdt), bias=b.to(DEV), act=k.ACT_RELU)
    ref = F.relu(F.linear(A if dt == "fp32" else _bf(A), W if dt == "fp32" else _bf(W), b))
    tol = 1e-5 if dt == "fp32" else 2e-3
    assert torch.allclose(out.cpu(), ref, rtol=tol, atol=tol * (1 + ref.abs().max().item())), \
        (out.cpu() - ref).abs().max()


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_gemm_nt_gather_hadamard_and_relu_bwd(dt):
    k = K()
    g = torch.Generator().manual_seed(1)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    N0, H, M, N = 50, 72, 333, 96
    X = torch.randn(N0, H, generator=g)
    ia = torch.randint(0, N0, (M,), generator=g)
    ib = torch.randint(0, N0, (M,), generator=g)
    W = torch.randn(N, H, generator=g) * 0.2
    aux = torch.randn(M, N, generator=g)
    Xd = X.to(DEV, tdt)
    out = torch.empty(M, N, device=DEV, dtype=tdt)
    k.gemm_nt(k.operand(Xd, ia.to(DEV, torch.int32), Xd, ib.to(DEV, torch.int32)), k.operand(W.to(DEV, tdt)), M, N, H,
              out, k.dtype_code(tdt), act=k.ACT_RELU_BWD, aux=aux.to(DEV, tdt), alpha=2.0)
    Xr = X if dt == "fp32" else _bf(X)
    prod = Xr[ia] * Xr[ib]
    if dt == "bf16":
        prod = _bf(prod)
    ref = 2.0 * F.linear(prod, W if dt == "fp32" else _bf(W)) * ((aux if dt == "fp32" else _bf(aux)) > 0)
    tol = 1e-5 if dt == "fp32" else 1e-2
    assert torch.allclose(out.float().cpu(), ref, rtol=tol, atol=tol * (1 + ref.abs().max().item()))


@pytest.mark.parametrize("M,N,Kd,act", [(1000, 256, 128, "relu_bwd"), (700, 1024, 64, "relu"), (300, 40, 192, "none")])
def test_gemm_nt_bf16_large_tile_paths(M, N, Kd, act):
    """Shapes that take the 256x256 glds kernel (bf16, K % 64 == 0, N % 8 == 0),
    with a gathered Hadamard A operand (the predictor's x_i * x_j)."""
    k = K()
    g = torch.Generator().manual_seed(M + N + Kd)
    N0 = 97
    X = torch.randn(N0, Kd, generator=g)
    ia = torch.randint(0, N0, (M,), generator=g)
    ib = torch.randint(0, N0, (M,), generator=g)
    W = torch.randn(N, Kd, generator=g) * 0.1
    b = torch.randn(N, generator=g)
    aux = torch.randn(M, N, generator=g)
    Xd = X.to(DEV, torch.bfloat16)
    iad, ibd = ia.to(DEV, torch.int32), ib.to(DEV, torch.int32)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    code = {"none": k.ACT_NONE, "relu": k.ACT_RELU, "relu_bwd": k.ACT_RELU_BWD}[act]
    auxd = aux.to(DEV, torch.bfloat16)
    k.gemm_nt(k.operand(Xd, iad, Xd, ibd), k.operand(W.to(DEV, torch.bfloat16)), M, N, Kd, out, 1, bias=b.to(DEV),
              act=code, aux=auxd if act == "relu_bwd" else None, alpha=0.5)
    prod = _bf(_bf(X)[ia] * _bf(X)[ib])
    ref = 0.5 * F.linear(prod, _bf(W)) + b
    if act == "relu":
        ref = F.relu(ref)
    if act == "relu_bwd":
        ref = ref * (_bf(aux) > 0)
    assert torch.allclose(out.float().cpu(), ref, rtol=1e-2, atol=1e-2 * (1 + ref.abs().max().item()))
    # plain gathered operand (no Hadamard) through the glds path
    out2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(Xd, iad), k.operand(W.to(DEV, torch.bfloat16)), M, N, Kd, out2, 1)
    ref2 = F.linear(_bf(X)[ia], _bf(W))
    assert torch.allclose(out2.float().cpu(), ref2, rtol=1e-2, atol=1e-2 * (1 + ref2.abs().max().item()))


@pytest.mark.parametrize("M,N,Kd", [(1000, 1024, 128), (513, 256, 256)])
def test_gemm_nt_head_fused(M, N, Kd):
    """Linear(N,1) head fused into the GEMM epilogue == separate head pass."""
    k = K()
    g = torch.Generator().manual_seed(M)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    hw = torch.randn(N, generator=g).to(DEV)
    hb = torch.randn(1, generator=g).to(DEV)
    parts = k.head_parts(N)
    hpart = torch.empty(parts, M, device=DEV)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, C, hw, hpart, bias=b, act=k.ACT_RELU)
    logit = torch.empty(M, device=DEV)
    prob = torch.empty(M, device=DEV)
    k.head_finish(parts, M, hpart, hb, logit=logit, prob=prob)
    y = F.relu(A.float() @ W.float().t() + b)
    assert torch.allclose(C.float(), y, rtol=1e-2, atol=1e-2)
    # the head dot is taken over the stored bf16 outputs (the values the head backward reads)
    ref = C.float() @ hw + hb
    assert torch.allclose(logit, ref, rtol=1e-4, atol=1e-4 * (1 + ref.abs().max().item()))
    assert torch.allclose(logit, y @ hw + hb, rtol=1e-2, atol=1e-2 * (1 + ref.abs().max().item()))
    assert torch.allclose(prob, torch.sigmoid(ref), atol=1e-4)
    # head only (C = None)
    hpart2 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, None, hw, hpart2, bias=b, act=k.ACT_RELU)
    assert torch.equal(hpart, hpart2)


@pytest.mark.parametrize("M,N,Kd", [(1000, 1024, 128), (513, 256, 256), (4096, 1024, 1024)])
def test_gemm_nt_head_lean(M, N, Kd):
    """The head epilogue over the staged bf16 outputs (gemm256.hip epilogue_lean_head, taken
    when N % 256 == 0, the head weights are 16-B aligned and C is 16-B aligned with ldc % 8
    == 0): C bit-identical to the generic head epilogue (forced here by misaligned head
    weights); the head dot over the
    ROUNDED bf16 outputs, within f32 summation-order tolerance of bf16(y) @ hw;
    deterministic with and without C."""
    k = K()
    g = torch.Generator().manual_seed(M + 1)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * (0.3 / Kd ** 0.5)).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    hw = torch.randn(N, generator=g).to(DEV)
    parts = k.head_parts(N)
    hw_odd = torch.empty(N + 1, device=DEV)[1:]          # head weights off 16-B alignment: generic epilogue
    hw_odd.copy_(hw)
    C0 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, C0, hw_odd, torch.empty(parts, M, device=DEV), bias=b,
                   act=k.ACT_RELU)
    C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)                  # lean head epilogue
    h1 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, C1, hw, h1, bias=b, act=k.ACT_RELU)
    h2 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, None, hw, h2, bias=b, act=k.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(C1, C0)
    assert torch.equal(h1, h2)
    ref = C0.float() @ hw
    got = h1.sum(0)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-4 * (1 + ref.abs().max().item())), (got - ref).abs().max()


@pytest.mark.parametrize("M,N,Kd", [(70_000, 256, 256), (20_000, 1024, 1024), (66_000, 512, 128)])
def test_gemm_nt_head_f32(M, N, Kd):
    """fp32 fused head (llp_gemm_nt_head_f32, the persistent f32 kernel's F32_HEAD epilogue): C equals
    the plain ReLU launch bit for bit (the same MFMAs and epilogue values), the head partials summed
    over the column tiles equal relu(y) @ hw within f32 summation-order tolerance, and repeated
    launches are bit-identical (a fixed summation order)."""
    k = K()
    g = torch.Generator().manual_seed(M + N)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(DEV)
    W = (torch.randn(N, Kd, generator=g) * (1.0 / Kd ** 0.5)).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    hw = torch.randn(N, generator=g).to(DEV)
    parts = k.head_parts(N)
    C0 = torch.empty(M, N, device=DEV)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C0, k.LLP_F32, bias=b, act=k.ACT_RELU)
    C1 = torch.empty(M, N, device=DEV)
    h1 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head_f32(k.operand(A), k.operand(W), M, N, Kd, C1, hw, h1, bias=b)
    h2 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head_f32(k.operand(A), k.operand(W), M, N, Kd, torch.empty(M, N, device=DEV), hw, h2, bias=b)
    torch.cuda.synchronize()
    assert torch.equal(C1, C0)
    assert torch.equal(h1, h2)
    ref = C0.double() @ hw.double()
    got = h1.double().sum(0)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-5 * (1 + ref.abs().max().item())), (got - ref).abs().max()


@pytest.mark.parametrize("M,N,Kd", [(70_001, 1024, 1024), (5_000, 256, 128)])
def test_gemm_nt_w4_bit_identical(M, N, Kd):
    """The one-wave-per-SIMD NT kernel (csrc/gemm256_w4.hip, diagnostic entry llp_gemm_nt_w4_probe;
    DESIGN.md §4.1, measured slower, not dispatched) against the shipped persistent kernel: ReLU +
    bias + bit mask, plain, and ReLU-mask backward outputs bit-identical (a partial last m-tile
    included), so its A/B timings compare like for like."""
    import ctypes as C
    k = K()
    L = k.lib()
    L.llp_gemm_nt_w4_probe.restype = C.c_int
    L.llp_gemm_nt_w4_probe.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                       C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_float, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.c_int, C.c_void_p]
    g = torch.Generator().manual_seed(M)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * (1.0 / Kd ** 0.5)).to(DEV, torch.bfloat16)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)

    def w4(C_, act, bias=None, alpha=1.0, mo=None, mi=None):
        m = mo if mo is not None else mi
        k.check(L.llp_gemm_nt_w4_probe(A.data_ptr(), Kd, W.data_ptr(), Kd, M, N, Kd, C_.data_ptr(), N, k.ptr(bias), act,
                                       alpha, k.ptr(mo), k.ptr(mi), m.stride(0) if m is not None else 0, 0,
                                       k.stream_ptr()), "llp_gemm_nt_w4_probe")

    outs = {}
    for name in ("pp8p", "w4"):
        Cr = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        mr = torch.zeros(M, N // 8, device=DEV, dtype=torch.uint8)
        Cn = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        Cb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        if name == "pp8p":
            k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, Cr, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=mr)
            k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, Cn, k.LLP_BF16)
            k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, Cb, k.LLP_BF16, act=k.ACT_RELU_BWD, aux=mr, alpha=2.0)
        else:
            w4(Cr, k.ACT_RELU, bias=b, mo=mr)
            w4(Cn, k.ACT_NONE)
            w4(Cb, k.ACT_RELU_BWD, alpha=2.0, mi=outs["pp8p"][1])
        outs[name] = (Cr, mr, Cn, Cb)
    torch.cuda.synchronize()
    for a, c in zip(outs["pp8p"], outs["w4"]):
        assert torch.equal(a, c)
    ref = F.relu(A.float() @ W.float().t() + b)
    assert torch.allclose(outs["w4"][0].float(), ref, rtol=1e-2, atol=1e-2 * (1 + ref.abs().max().item()))


def test_gemm_nt_relu_lean_and_generic_agree_with_nan():
    """ReLU forward: full 256 x 256 tiles take the lean epilogue (int16 max on the rounded
    pair), partial tiles the generic one (f32); both follow the sign-bit rule, so the same
    rows give the same outputs in a full and in a partial tile, NaN rows included."""
    k = K()
    g = torch.Generator().manual_seed(7)
    M, N, Kd = 256, 256, 128
    A = (torch.randn(M, Kd, generator=g) * 0.5)
    A[3, 5] = float("nan")
    A[77, 0] = -float("nan")
    A[130, :] = float("inf")
    A = A.to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    full = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, full, k.LLP_BF16, bias=b, act=k.ACT_RELU)
    Mp = 200
    part = torch.empty(Mp, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(A[:Mp]), k.operand(W), Mp, N, Kd, part, k.LLP_BF16, bias=b, act=k.ACT_RELU)
    torch.cuda.synchronize()
    f, p_ = full[:Mp].float().cpu(), part.float().cpu()
    assert torch.equal(torch.isnan(f), torch.isnan(p_))
    ok = ~torch.isnan(f)
    assert torch.equal(f[ok], p_[ok])
    assert bool((f[ok] >= 0).all())
    assert bool(torch.isnan(f[3]).any() or (f[3] == 0).all())


def test_gemm_nt_bf16_dropout_matches_fp32_mask():
    """The 256-tile bf16 kernel and the general kernel draw the same dropout mask."""
    k = K()
    M, N, Kd = 600, 256, 128
    A = torch.randn(M, Kd, device=DEV)
    W = torch.randn(N, Kd, device=DEV) * 0.1
    ctr = torch.full((1,), 5, dtype=torch.int64, device=DEV)
    o32 = torch.empty(M, N, device=DEV)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, o32, 0, act=k.ACT_NONE,
              dropout=k.Dropout(0.3, 99, ctr.data_ptr(), 4))
    o16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(A.bfloat16()), k.operand(W.bfloat16()), M, N, Kd, o16, 1, act=k.ACT_NONE,
              dropout=k.Dropout(0.3, 99, ctr.data_ptr(), 4))
    assert torch.equal(o32 != 0, o16.float() != 0)


def test_gemm_nt_dropout_is_deterministic_and_unbiased():
    k = K()
    M, N, Kd = 512, 256, 64
    A = torch.randn(M, Kd, device=DEV)
    W = torch.randn(N, Kd, device=DEV) * 0.1
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    outs = []
    for _ in range(2):
        o = torch.empty(M, N, device=DEV)
        k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, o, 0, act=k.ACT_NONE,
                  dropout=k.Dropout(0.5, 1234, ctr.data_ptr(), 3))
        outs.append(o)
    assert torch.equal(outs[0], outs[1])
    full = A @ W.t()
    kept = outs[0] != 0
    frac = kept.float().mean().item()
    assert 0.48 < frac < 0.52
    assert torch.allclose(outs[0][kept], 2.0 * full[kept], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("p", [0.5, 0.3])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_act_2d_dropout_keep_matches_oracle(p, dt):
    """llp_act_2d's keep pattern is the oracle's dropout_keep bit for bit (8-bit draws at
    p = 0.5, 16-bit at 0.3), on a width that is not a multiple of 64 and a strided view."""
    k = K()
    rows, n, step, off, seed = 37, 200, 3, 5, 4242
    x = torch.ones(rows, n + 8, device=DEV, dtype=dt)[:, :n]
    y = torch.empty(rows, n, device=DEV, dtype=dt)
    ctr = torch.full((1,), step, dtype=torch.int64, device=DEV)
    k.act_2d(x, y, act=k.ACT_RELU, dropout=k.Dropout(p, seed, ctr.data_ptr(), off))
    torch.cuda.synchronize()
    keep = O.dropout_keep(seed, O.STREAMS_PER_STEP * step + off, rows, n, p)
    assert torch.equal(y.cpu() != 0, torch.from_numpy(keep))
    assert torch.allclose(y[y != 0].float(), torch.full((1,), 1.0 / (1.0 - p), device=DEV).to(dt).float())


@pytest.mark.parametrize("M,N,Kd", [(70_000, 256, 512), (70_001, 512, 256), (3_000, 256, 512)])
def test_gemm_nt_dropout_exact_against_relu(M, N, Kd):
    """The bf16 dropout forward (pp8p<EPI_FWD_DROP> above 256 tiles, pp8's generic epilogue
    below) at p = 0.5: scale 2 is exact, so its output is where(keep, 2 * relu output, 0) of
    the ReLU kernel on the same operands bit for bit, keep = the oracle's dropout_keep, and
    its ReLU mask is the bits of that output (partial last m-tile at M = 70,001)."""
    k = K()
    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    ctr = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    R = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, R, k.LLP_BF16, bias=b, act=k.ACT_RELU)
    D = torch.empty_like(R)
    mask = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, D, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=mask,
              dropout=k.Dropout(0.5, 99, ctr.data_ptr(), 2))
    if M > 65_536:
        assert "EPI_FWD_DROP" in k.last_gemm_kernel()
    torch.cuda.synchronize()
    keep = torch.from_numpy(O.dropout_keep(99, O.STREAMS_PER_STEP * 7 + 2, M, N, 0.5)).to(DEV)
    exp = torch.where(keep, R.float() * 2.0, torch.zeros((), device=DEV)).to(torch.bfloat16)
    assert torch.equal(D.view(torch.int16), exp.view(torch.int16))
    bits = (D.float() > 0).view(M, N // 8, 8).to(torch.uint8)
    want = (bits << torch.arange(8, device=DEV, dtype=torch.uint8)).sum(-1).to(torch.uint8)
    assert torch.equal(mask, want)


def test_gemm_nt_dropout_16bit_draws():
    """p = 0.3 (16-bit draws) on the persistent dropout epilogue: the zero pattern is
    keep & (relu output > 0) exactly, the kept values 1/0.7 x the ReLU output to bf16 rounding."""
    k = K()
    M, N, Kd = 70_000, 256, 256
    g = torch.Generator().manual_seed(11)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    ctr = torch.full((1,), 1, dtype=torch.int64, device=DEV)
    R = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, R, k.LLP_BF16, act=k.ACT_RELU)
    D = torch.empty_like(R)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, D, k.LLP_BF16, act=k.ACT_RELU,
              dropout=k.Dropout(0.3, 5, ctr.data_ptr(), 1))
    assert "EPI_FWD_DROP" in k.last_gemm_kernel()
    torch.cuda.synchronize()
    keep = torch.from_numpy(O.dropout_keep(5, O.STREAMS_PER_STEP + 1, M, N, 0.3)).to(DEV)
    assert torch.equal(D != 0, keep & (R > 0))
    kept = D != 0
    assert torch.allclose(D[kept].float(), R[kept].float() / 0.7, rtol=8e-3, atol=0)
    assert abs(keep.float().mean().item() - 0.7) < 0.005


# ------------------------------------------------------------------ GEMM TN (weight grads)
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("M,P,Q", [(1000, 64, 48), (5000, 256, 128), (77, 130, 20), (20000, 128, 256),
                                    (20000, 1024, 136), (20000, 512, 384)])
def test_gemm_tn(dt, M, P, Q):
    """Q = 128 / 384: the 256-tile bf16 kernel's waves 4-7 hold only padding in the (last)
    Q tile and skip their MFMAs; Q = 136 keeps them live for 8 columns."""
    k = K()
    g = torch.Generator().manual_seed(M + P)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    A = torch.randn(M, P, generator=g)
    B = torch.randn(M, Q, generator=g)
    out = torch.empty(P, Q, device=DEV)
    ws = torch.empty(k.gemm_tn_ws_bytes(k.dtype_code(tdt), M, P, Q) // 4 + 16, device=DEV)
    k.gemm_tn(k.operand(A.to(DEV, tdt)), k.operand(B.to(DEV, tdt)), M, P, Q, out, k.dtype_code(tdt), ws)
    ref = (A if dt == "fp32" else _bf(A)).double().t() @ (B if dt == "fp32" else _bf(B)).double()
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= (1e-4 if dt == "fp32" else 2e-3) * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("dt,M,P,Q,qs", [("bf16", 50_003, 256, 512, 256), ("bf16", 9_001, 256, 256, 128),
                                          ("fp32", 20_011, 256, 512, 256), ("fp32", 7_001, 256, 128, 64),
                                          ("bf16", 3_001, 100, 90, 30)])
def test_gemm_tn_split_output(dt, M, P, Q, qs):
    """llp_gemm_tn_split (the SAGE teacher's one weight-gradient GEMM over [agg(x) | x] written
    into lin_l's and lin_r's gradients): columns [0, qs) in C, [qs, Q) in C2, bit-identical to
    the unsplit llp_gemm_tn on every path (bf16 256-tile, f32 256-tile, f32 128-tile (Q <= 128), and the
    scalar slab reduce at unaligned widths), with the fused bias column sums and accumulate."""
    k = K()
    g = torch.Generator().manual_seed(M + Q + qs)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    A = torch.randn(M, P, generator=g).to(DEV, tdt)
    B = torch.randn(M, Q, generator=g).to(DEV, tdt)
    ws = torch.empty(k.gemm_tn_ws_bytes(k.dtype_code(tdt), M, P, Q) // 4 + 16, device=DEV)
    full = torch.randn(P, Q, generator=g).to(DEV)
    cs_full = torch.zeros(P, device=DEV)
    C1 = full[:, :qs].contiguous()
    C2 = full[:, qs:].contiguous()
    cs = torch.zeros(P, device=DEV)
    k.gemm_tn(k.operand(A), k.operand(B), M, P, Q, full, k.dtype_code(tdt), ws, accumulate=True, colsum_a=cs_full)
    k.gemm_tn(k.operand(A), k.operand(B), M, P, Q, C1, k.dtype_code(tdt), ws, accumulate=True, colsum_a=cs,
              split=(qs, C2))
    torch.cuda.synchronize()
    assert torch.equal(C1, full[:, :qs]) and torch.equal(C2, full[:, qs:])
    assert torch.equal(cs, cs_full)


@pytest.mark.parametrize("M,P,Q,with_count", [(30_011, 1024, 1024, False), (4_099, 260, 132, True),
                                               (225_384, 1024, 136, False), (225_384, 1024, 128, False)])
def test_gemm_tn_f32_256(M, P, Q, with_count):
    """The f32 256-tile TN kernel (gemm256_tn_f32.hip: LDS-DMA ring, ds_read_b32 fragments, the
    bias gradient as ones-MFMAs) against float64: the weight gradient and the fused column sums,
    a ragged last stage and P / Q not multiples of 256, a device row count.  (Q <= 128, the
    collab student's first layer, goes to the 128-tile kernel: the same bar.)"""
    k = K()
    g = torch.Generator().manual_seed(M + P + Q)
    A = torch.randn(M, P, generator=g).to(DEV)
    B = torch.randn(M, Q, generator=g).to(DEV)
    cnt = torch.tensor([M - 77], dtype=torch.int32, device=DEV) if with_count else None
    Ml = M - 77 if with_count else M
    out = torch.empty(P, Q, device=DEV)
    cs = torch.empty(P, device=DEV)
    ws = torch.empty(k.gemm_tn_ws_bytes(k.LLP_F32, M, P, Q) // 4 + 16, device=DEV)
    k.gemm_tn(k.operand(A, count=cnt), k.operand(B, count=cnt), M, P, Q, out, k.LLP_F32, ws, colsum_a=cs)
    torch.cuda.synchronize()
    ref = A[:Ml].double().t() @ B[:Ml].double()
    err = (out.double() - ref).abs().max().item()
    assert err <= 1e-4 * (1 + ref.abs().max().item()), err
    refc = A[:Ml].double().sum(0)
    assert (cs.double() - refc).abs().max().item() <= 1e-4 * (1 + refc.abs().max().item())


def test_gemm_tn_gathered_hadamard_operand():
    k = K()
    g = torch.Generator().manual_seed(3)
    M, P, Q, N0 = 3000, 64, 96, 200
    A = torch.randn(M, P, generator=g)
    X = torch.randn(N0, Q, generator=g)
    ia = torch.randint(0, N0, (M,), generator=g)
    ib = torch.randint(0, N0, (M,), generator=g)
    out = torch.empty(P, Q, device=DEV)
    ws = torch.empty(k.gemm_tn_ws_bytes(0, M, P, Q) // 4 + 16, device=DEV)
    Xd = X.to(DEV)
    k.gemm_tn(k.operand(A.to(DEV)), k.operand(Xd, ia.to(DEV, torch.int32), Xd, ib.to(DEV, torch.int32)), M, P, Q,
              out, 0, ws)
    ref = A.double().t() @ (X[ia] * X[ib]).double()
    assert (out.cpu().double() - ref).abs().max().item() < 1e-3


# ------------------------------------------------------------------ Hadamard rows
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H", [200, 128, 256, 512, 1024, 2048])
@pytest.mark.parametrize("R", [1, 7, 1003])
def test_hadamard_rows_exact(dt, H, R):
    """out[r] = a[ia[r]] * b[ib[r]], rounded once to the storage dtype: bit-exact vs torch
    for the thread-per-chunk kernel (bf16 H=200, fp32 H=128/2048) and the row-group kernel
    (rows of 32, 64, 128, 256 16-B chunks), R not a multiple of the rows per wave."""
    k = K()
    g = torch.Generator().manual_seed(H + R)
    es = 2 if dt == torch.bfloat16 else 4
    if (H * es) % 16:
        pytest.skip("rows must be 16-byte multiples")
    na, nb = 300, 41
    a = torch.randn(na, H, generator=g).to(DEV, dt)
    b = torch.randn(nb, H, generator=g).to(DEV, dt)
    ia = torch.randint(0, na, (R,), generator=g, dtype=torch.int32).to(DEV)
    ib = torch.randint(0, nb, (R,), generator=g, dtype=torch.int32).to(DEV)
    out = torch.empty(R, H, device=DEV, dtype=dt)
    k.hadamard_rows(a, ia, b, ib, out)
    ref = (a[ia.long()].float() * b[ib.long()].float()).to(dt)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    out2 = torch.empty(min(R, na), H, device=DEV, dtype=dt)     # no index: rows in order
    k.hadamard_rows(a, None, a, None, out2)
    assert torch.equal(out2, (a[:out2.shape[0]].float() * a[:out2.shape[0]].float()).to(dt))


# ------------------------------------------------------------------ heads, colsum
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("R,H", [(1000, 200), (150_000, 1024)])
def test_head_fwd_bwd_and_colsum(dt, R, H):
    """R=150k: ~18 four-row batches per thread (both halves of the ping-pong loop)."""
    k = K()
    g = torch.Generator().manual_seed(4)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    Z = torch.relu(torch.randn(R, H, generator=g))
    w = torch.randn(H, generator=g) * (200 / H) ** 0.5   # logits O(1) at every H
    b = torch.randn(1, generator=g)
    Zd = Z.to(DEV, tdt)
    Zr = Z if dt == "fp32" else _bf(Z)
    logit = torch.empty(R, device=DEV)
    prob = torch.empty(R, device=DEV)
    k.head_fwd(Zd, R, H, w.to(DEV), b.to(DEV), logit=logit, prob=prob)
    ref = Zr @ w + b
    assert torch.allclose(logit.cpu(), ref, rtol=1e-5, atol=1e-4)
    assert torch.allclose(prob.cpu(), torch.sigmoid(ref), rtol=1e-5, atol=1e-6)
    dlogit = torch.randn(R, generator=g)
    dZ = torch.empty(R, H, device=DEV, dtype=tdt)
    dw = torch.empty(H, device=DEV)
    db = torch.empty(1, device=DEV)
    ws = torch.empty(k.head_bwd_ws_bytes(R, H) // 4 + 16, device=DEV)
    k.head_bwd(dlogit.to(DEV), Zd, R, H, w.to(DEV), True, dZ, dw, db, ws, alpha=1.5)
    ref_dZ = 1.5 * dlogit[:, None] * w[None, :] * (Zr > 0)
    tol = 1e-6 if dt == "fp32" else 1e-2
    assert torch.allclose(dZ.float().cpu(), ref_dZ, rtol=tol, atol=tol)
    assert torch.allclose(dw.cpu(), dlogit @ Zr, rtol=1e-4, atol=1e-3 * max(1.0, (R / 1000) ** 0.5))
    assert torch.allclose(db.cpu(), dlogit.sum().reshape(1), rtol=1e-5, atol=1e-4)
    cs = torch.empty(H, device=DEV)
    k.colsum(Zd, R, H, cs, ws)
    assert torch.allclose(cs.cpu(), Zr.sum(0), rtol=1e-5, atol=1e-3 * max(1.0, R / 1000))


# ------------------------------------------------------------------ fused LLP loss
@pytest.mark.parametrize("B,C,margin", [(37, 12, 0.1), (64, 36, 0.01), (5, 70, 0.2), (3, 2, 0.05), (3, 720, 0.05)])
def test_llp_loss_matches_oracle(B, C, margin):
    """C = 720: the largest contexts per anchor of the collab sweep
    (configurations/collab_transductive.yaml), 258,840 rank pairs per anchor."""
    k = K()
    g = torch.Generator().manual_seed(B * C)
    s_logit = torch.randn(B, C, generator=g) * 2
    t_prob = torch.rand(B, C, generator=g)
    t_prob[0, :2] = 0.5   # exact ties -> y = 0 pairs (Q5)
    n_pos = 50
    out_logit = torch.randn(2 * n_pos, generator=g) * 3
    wl, wd, wr = 0.7, 1.3, 2.1
    dlog = torch.empty(B * C + 2 * n_pos, device=DEV)
    terms = torch.zeros(4, device=DEV)
    ws = torch.empty(k.llp_loss_ws_bytes(B, 2 * n_pos) // 4 + 16, device=DEV)
    sl = s_logit.reshape(-1).to(DEV)
    ol = out_logit.to(DEV)
    k.llp_loss(B, C, sl, t_prob.reshape(-1).to(DEV), 2 * n_pos, n_pos, ol, B, 2 * n_pos, margin, 1.0, wl, wd, wr,
               dlog, dlog[B * C:], terms, ws)
    # oracle through torch autograd (fp64)
    s = s_logit.double().requires_grad_()
    o = out_logit.double().requires_grad_()
    sp = torch.sigmoid(s)
    kl = O.kl_loss(sp, t_prob.double(), 1)
    rk = O.rank_loss(sp, t_prob.double(), margin)
    lab = torch.cat([torch.ones(n_pos), torch.zeros(n_pos)]).double()
    bce = O.bce_loss(torch.sigmoid(o), lab)
    loss = wl * bce + wd * kl + wr * rk
    loss.backward()
    t = terms.cpu()
    assert abs(t[0].item() - loss.item()) < 1e-5 * max(1, abs(loss.item()))
    assert abs(t[1].item() - bce.item()) < 1e-5
    assert abs(t[2].item() - kl.item()) < 1e-5
    assert abs(t[3].item() - rk.item()) < 1e-5
    d = dlog.cpu().double()
    assert torch.allclose(d[:B * C], s.grad.reshape(-1), rtol=1e-4, atol=1e-7)
    assert torch.allclose(d[B * C:], o.grad, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("B,C,n_lab,parts,dense", [(3277, 36, 16384, 4, False), (1, 20, 300, 1, True),
                                                    (0, 1, 5000, 4, False), (70, 100, 0, 2, False)])
def test_llp_loss_heads_one_launch(B, C, n_lab, parts, dense):
    """llp_llp_loss_heads (the student / teacher heads finished in the loss launch, the terms
    summed by its last workgroup on a self-resetting ticket) == llp_head_finish x 2 + the
    separate llp_llp_loss: logits, teacher probabilities, gradients and terms bit for bit, over
    repeated calls (the ticket must come back to zero each time)."""
    k = K()
    g = torch.Generator().manual_seed(B + n_lab)
    R = B * C + n_lab
    n_pos = n_lab // 2
    sp = (torch.randn(parts, max(R, 1), generator=g) * 0.7).to(DEV)
    tp = (torch.randn(parts, max(B * C, 1), generator=g) * 0.7).to(DEV)
    sb = torch.randn(1, generator=g).to(DEV)
    tb = torch.randn(1, generator=g).to(DEV)
    cnt = torch.tensor([n_lab - n_pos - 3], dtype=torch.int32, device=DEV) if dense else None
    ws = torch.empty(k.llp_loss_ws_bytes(B, n_lab) // 4 + 16, device=DEV)
    ticket = k.ticket_block(DEV)
    for it in range(3):
        # reference: the heads finished by their own launches, the loss in three
        logit1 = torch.empty(max(R, 1), device=DEV)
        tprob1 = torch.empty(max(B * C, 1), device=DEV)
        k.head_finish(parts, R, sp, sb, logit=logit1)
        if B > 0:
            k.head_finish(parts, B * C, tp, tb, prob=tprob1)
        d1 = torch.empty(max(R, 1), device=DEV)
        t1 = torch.zeros(4, device=DEV)
        k.llp_loss(B, C, logit1, tprob1, n_lab, n_pos, logit1[B * C:], max(B, 1), n_lab, 0.1, 1.0, 0.3, 1.1, 0.9, d1,
                   d1[B * C:], t1, ws, neg_count=cnt, pos_total=n_pos)
        logit2 = torch.full((max(R, 1),), 7.0, device=DEV)
        tprob2 = torch.full((max(B * C, 1),), 7.0, device=DEV)
        d2 = torch.empty(max(R, 1), device=DEV)
        t2 = torch.zeros(4, device=DEV)
        k.llp_loss(B, C, logit2, tprob2, n_lab, n_pos, logit2[B * C:], max(B, 1), n_lab, 0.1, 1.0, 0.3, 1.1, 0.9, d2,
                   d2[B * C:], t2, ws, neg_count=cnt, pos_total=n_pos, s_head=k.head_in(sp, parts, R, sb),
                   t_head=k.head_in(tp, parts, B * C, tb) if B > 0 else None, ticket=ticket)
        torch.cuda.synchronize()
        assert torch.equal(logit1[:R], logit2[:R]), it
        assert torch.equal(tprob1[:B * C], tprob2[:B * C]), it
        assert torch.equal(d1[:R], d2[:R]), it
        assert torch.equal(t1, t2), it
        assert int(ticket.abs().sum()) == 0
        sp.mul_(1.1)


# ------------------------------------------------------------------ samplers (bit-exact)
@pytest.mark.parametrize("ps,rw_step,hops,ns_rate", [("nb", 3, 3, 3), ("rw", 2, 2, 1), ("nb", 1, 15, 0),
                                                    ("nb", 20, 2, 1), ("nb", 61, 1, 0)])
@pytest.mark.parametrize("sorted_", [False, True])
def test_context_sampler_bit_exact(ps, rw_step, hops, ns_rate, sorted_):
    import llp_engine
    k = K()
    rng = np.random.default_rng(5)
    N = 500
    u = rng.integers(0, N, 3000)
    v = rng.integers(0, N, 3000)
    pairs = np.stack([u, v], 1)
    ei = np.stack([pairs, pairs[:, ::-1]], 1).reshape(-1, 2).T   # interleaved, unsorted (Q1)
    ei = ei[:, ei[0] % 17 != 3]                                   # leave some isolated nodes (deg 0)
    rowptr, col = llp_engine.build_sampler_csr(ei[0], ei[1], N, sorted_)
    start = rng.permutation(N)[:123].astype(np.int32)
    C1 = 1 + rw_step * hops * (1 + ns_rate)
    out = torch.empty(123, C1, dtype=torch.int32, device=DEV)
    ctr = torch.tensor([7], dtype=torch.int64, device=DEV)
    k.context_sampler(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(col).to(DEV), N,
                      torch.from_numpy(start).to(DEV), 123, ps, rw_step, hops, ns_rate, 99, ctr, 0, out, b_offset=0)
    pos, neg = O.neighbor_samplers(rowptr.astype(np.int64), col.astype(np.int64), start, N, rw_step, ps, ns_rate,
                                   hops, seed=99, stream_base=O.STREAMS_PER_STEP * 7)
    ref = np.concatenate([pos, neg], 1)
    assert np.array_equal(out.cpu().numpy(), ref)
    # shard invariance: anchors [60, 123) drawn by a second "rank" match
    out2 = torch.empty(63, C1, dtype=torch.int32, device=DEV)
    k.context_sampler(torch.from_numpy(rowptr).to(DEV), torch.from_numpy(col).to(DEV), N,
                      torch.from_numpy(start[60:]).to(DEV), 63, ps, rw_step, hops, ns_rate, 99, ctr, 0, out2,
                      b_offset=60)
    assert np.array_equal(out2.cpu().numpy(), ref[60:])


@pytest.mark.parametrize("ps,rw_step,hops,ns_rate", [("nb", 3, 3, 3), ("rw", 2, 2, 1), ("nb", 2, 3, 0),
                                                    ("nb", 20, 2, 1)])
@pytest.mark.parametrize("b_off,p_off", [(0, 0), (40, 300)])
def test_minibatch_sample_equals_separate_kernels(ps, rw_step, hops, ns_rate, b_off, p_off):
    """llp_minibatch_sample == context_sampler + randint_pairs + build_targets +
    pair_index_from_samples, bit for bit (also for a rank's shard)."""
    import llp_engine
    k = K()
    rng = np.random.default_rng(11)
    N, B, P, P_total, E = 400, 77, 150, 600, 2000
    u, v = rng.integers(0, N, E), rng.integers(0, N, E)
    ei = np.stack([np.stack([u, v], 1), np.stack([v, u], 1)], 1).reshape(-1, 2).T
    ei = ei[:, ei[0] % 13 != 5]                                   # some isolated nodes
    rowptr, col = (torch.from_numpy(a).to(DEV) for a in llp_engine.build_sampler_csr(ei[0], ei[1], N, False))
    pairs = torch.from_numpy(np.stack([u, v], 1).astype(np.int32)).to(DEV)
    start = torch.from_numpy(rng.permutation(N)[:B].astype(np.int32)).to(DEV)
    perm = torch.from_numpy(rng.integers(0, E, P).astype(np.int32)).to(DEV)
    C = rw_step * hops * (1 + ns_rate)
    C1, R1 = C + 1, B * (C + 1) + 4 * P
    ctr = torch.tensor([5], dtype=torch.int64, device=DEV)
    s1, s2 = (torch.full((B, C1), -1, dtype=torch.int32, device=DEV) for _ in range(2))
    n1, n2 = (torch.full((2, P), -1, dtype=torch.int32, device=DEV) for _ in range(2))
    t1, t2 = (torch.full((R1,), -1, dtype=torch.int32, device=DEV) for _ in range(2))
    a1, a2, b1, b2 = (torch.full((B * C,), -1, dtype=torch.int32, device=DEV) for _ in range(4))
    k.context_sampler(rowptr, col, N, start, B, ps, rw_step, hops, ns_rate, 31, ctr, 0, s1, b_offset=b_off)
    k.randint_pairs(N, P, 31, ctr, O.RANDINT_STREAM, n1, n_total=P_total, offset=p_off)
    k.build_targets(B, C1, s1, pairs, perm, None, 0, P, n1, t1)
    k.pair_index_from_samples(B, C, s1, a1, b1)
    k.minibatch_sample(rowptr, col, N, start, B, ps, rw_step, hops, ns_rate, 31, ctr, 0, pairs, perm, P, P_total,
                       p_off, O.RANDINT_STREAM, s2, n2, t2, a2, b2, b_offset=b_off)
    for x, y in ((s1, s2), (n1, n2), (t1, t2), (a1, a2), (b1, b2)):
        assert torch.equal(x, y)


def test_random_walk_follows_unsorted_csr_semantics():
    """Q1: with coalesced=False the walk indexes col in array order."""
    import llp_engine
    row = np.array([1, 0, 2, 0, 1, 2])
    col = np.array([0, 1, 0, 2, 2, 1])
    rowptr, colv = llp_engine.build_sampler_csr(row, col, 3, False)
    assert rowptr.tolist() == [0, 2, 4, 6]
    assert colv.tolist() == [0, 1, 0, 2, 2, 1]   # node 0's "neighbours" = col[0:2] = [0, 1] (unsorted order)


def test_randint_pairs_bit_exact_and_sharded():
    k = K()
    ctr = torch.tensor([3], dtype=torch.int64, device=DEV)
    out = torch.empty(2, 1000, dtype=torch.int32, device=DEV)
    k.randint_pairs(12345, 1000, 77, ctr, O.RANDINT_STREAM, out)
    ref = O.randint_edges(12345, 1000, seed=77, stream=O.STREAMS_PER_STEP * 3 + O.RANDINT_STREAM)
    assert np.array_equal(out.cpu().numpy(), ref)
    part = torch.empty(2, 300, dtype=torch.int32, device=DEV)
    k.randint_pairs(12345, 300, 77, ctr, O.RANDINT_STREAM, part, n_total=1000, offset=500)
    assert np.array_equal(part.cpu().numpy(), ref[:, 500:800])


# ------------------------------------------------------------------ SAGE aggregate
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("F_", [128, 256, 30, 8, 24, 48, 200, 1000])
def test_csr_mean_aggregate_fwd_bwd(dt, F_):
    import llp_sage
    k = K()
    rng = np.random.default_rng(F_)
    N = 700
    u = rng.integers(0, N, 5000)
    v = rng.integers(0, N, 5000)
    ei = torch.from_numpy(np.stack([np.concatenate([u, v, u[:100]]), np.concatenate([v, u, v[:100]])]))  # dup edges
    g = llp_sage.Graph(ei, N, DEV)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    x = torch.randn(N, F_)
    xr = x if dt == "fp32" else _bf(x)
    out = torch.empty(N, F_, device=DEV, dtype=tdt)
    k.csr_aggregate(N, F_, g.rowptr, g.col, x.to(DEV, tdt), None, 0, out)
    ref = O.sage_mean_aggregate(xr, ei[0], ei[1], N)
    tol = 1e-5 if dt == "fp32" else 1e-2
    assert torch.allclose(out.float().cpu(), ref, rtol=tol, atol=tol)
    # backward: d/dx of sum(out * gout)
    gout = torch.randn(N, F_)
    xg = xr.clone().requires_grad_()
    (O.sage_mean_aggregate(xg, ei[0], ei[1], N) * (gout if dt == "fp32" else _bf(gout))).sum().backward()
    gx = torch.empty(N, F_, device=DEV, dtype=tdt)
    k.csr_aggregate(N, F_, g.rowptr_t, g.col_t, gout.to(DEV, tdt), g.inv_deg, 1, gx)
    assert torch.allclose(gx.float().cpu(), xg.grad, rtol=tol, atol=tol * 2)


def _bf16_rne(a):
    """f32 -> bf16 (round to nearest even) -> f32, in numpy."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("F_", [64, 128, 256, 512])
def test_csr_mean_aggregate_hubs_bit_exact(dt, F_):
    """The LDS-staged aggregate (csr_agg_lds_kernel) with hub rows whose neighbour lists
    overflow the workgroup's staged slice (AGG_CAP = 1,024 indices: the excess is read from
    global memory), a tile whose rows together overflow it, empty rows and duplicate edges:
    bit for bit the f32 neighbour-order sum times 1/deg, rounded once (PyG mean, Q2), which is
    what the rows-per-wave kernel computed."""
    import llp_sage
    if dt == "fp32" and F_ == 512:
        pytest.skip("128 chunks per row: the lane-group kernel (a different, fixed summation order)")
    k = K()
    rng = np.random.default_rng(F_ + (0 if dt == "fp32" else 1))
    N = 3000
    src = [rng.integers(0, N, 20000)]
    dst = [rng.integers(0, N, 20000)]
    for hub, deg in ((5, 2500), (6, 700), (7, 700), (1777, 4000)):   # 6, 7 share a tile: 1,400 > 1,024
        src.append(rng.integers(0, N, deg))
        dst.append(np.full(deg, hub))
    src, dst = np.concatenate(src), np.concatenate(dst)
    keep = (dst < 2000) | (dst > 2100)                     # rows 2000-2100 empty
    ei = torch.from_numpy(np.stack([src[keep], dst[keep]]))
    g = llp_sage.Graph(ei, N, DEV)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    x = torch.randn(N, F_).to(tdt)
    out = torch.empty(N, F_, device=DEV, dtype=tdt)
    k.csr_aggregate(N, F_, g.rowptr, g.col, x.to(DEV), None, 0, out)
    rp, cl = g.rowptr.cpu().numpy(), g.col.cpu().numpy()
    xf = x.float().numpy()
    ref = np.zeros((N, F_), np.float32)
    for r in range(N):
        acc = np.zeros(F_, np.float32)
        for e in range(rp[r], rp[r + 1]):
            acc = acc + xf[cl[e]]
        ref[r] = acc * (np.float32(1.0) / np.float32(max(rp[r + 1] - rp[r], 1)))
    if dt == "bf16":
        ref = _bf16_rne(ref)
    assert np.array_equal(out.float().cpu().numpy(), ref)
    assert int(np.diff(rp).max()) >= 4000
    # degree-weighted (mode 1, the mean's backward over the transposed CSR) against the oracle
    gout = torch.randn(N, F_).to(tdt)
    gx = torch.empty(N, F_, device=DEV, dtype=tdt)
    k.csr_aggregate(N, F_, g.rowptr_t, g.col_t, gout.to(DEV), g.inv_deg, 1, gx)
    xg = x.float().clone().requires_grad_()
    (O.sage_mean_aggregate(xg, ei[0], ei[1], N) * gout.float()).sum().backward()
    tol = 1e-5 if dt == "fp32" else 1e-2
    assert torch.allclose(gx.float().cpu(), xg.grad, rtol=tol, atol=tol * 2)


# ------------------------------------------------------------------ clip + Adam
# (shape, group, shadows) per tensor.  "big": one tensor of 275 chunks (> 256 finalize
# threads, so threads sum several chunk partials), eight clip groups, bf16 shadow and
# transposed shadow (the transpose kernel also advances the step counter).
_ADAM_CASES = {
    "small": [((64, 32), 0, False), ((64,), 0, False), ((1, 64), 1, False), ((1,), 1, False)],
    "big": [((1100, 1024), 0, True), ((1024,), 0, False), ((300, 257), 1, True), ((257,), 1, False),
            ((5000,), 2, False), ((3,), 3, False), ((70, 70), 4, True), ((9000,), 5, False), ((1,), 6, False),
            ((129, 65), 7, True)],
}


@pytest.mark.parametrize("case", sorted(_ADAM_CASES))
@pytest.mark.parametrize("nan_group", [None, 1])
@pytest.mark.parametrize("fused", [False, True])
def test_clip_and_adam_match_oracle(case, nan_group, fused):
    """grad_sumsq (chunk partials + one-pass finalize) + clip per group + Adam
    against the oracle's clip_grad_norm_ / Adam (src/main.py:132-138); a NaN
    gradient turns its group's clip coefficient into NaN, as torch.clamp does.
    fused: the one-launch forms (llp_grad_sumsq_t with a ticket block, llp_adam_step_t with the
    step counter advanced after it, as llp_step_end2 does)."""
    k = K()
    tickets = k.ticket_block(DEV) if fused else None
    spec = _ADAM_CASES[case]
    g = torch.Generator().manual_seed(9 + len(spec))
    shapes = [sh for sh, _, _ in spec]
    groups = [gr for _, gr, _ in spec]
    n_groups = max(groups) + 1
    params = [torch.randn(*s, generator=g) for s in shapes]
    grads = [torch.randn(*s, generator=g) * 3 for s in shapes]
    if nan_group is not None:
        i_nan = groups.index(nan_group)
        grads[i_nan].view(-1)[grads[i_nan].numel() // 2] = float("nan")
    dp = [p.to(DEV).clone() for p in params]
    dg = [x.to(DEV).clone() for x in grads]
    m = [torch.zeros_like(p) for p in dp]
    v = [torch.zeros_like(p) for p in dp]
    sh, sht = [], []
    descs = []
    for i, p in enumerate(dp):
        rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
        s_ = st_ = None
        if spec[i][2]:
            s_ = torch.zeros(rows, cols, dtype=torch.bfloat16, device=DEV)
            st_ = torch.zeros(cols, rows, dtype=torch.bfloat16, device=DEV)
        sh.append(s_)
        sht.append(st_)
        descs.append(k.TensorDesc(p.data_ptr(), dg[i].data_ptr(), m[i].data_ptr(), v[i].data_ptr(),
                                  k.ptr(s_), k.ptr(st_), p.numel(), rows, cols, groups[i],
                                  k.LLP_BF16 if s_ is not None else 0))
    max_numel = max(p.numel() for p in dp)
    assert case != "big" or -(-max_numel // 4096) > 256
    dd = k.descs_to_device(descs, DEV)
    sumsq = torch.zeros(n_groups, device=DEV)
    ws = torch.empty(k.grad_sumsq_ws_bytes(len(dp), max_numel) // 4 + 16, device=DEV)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    adam = O.AdamState(params, lr=0.01)
    cur = [p.clone() for p in params]
    for it in range(3):
        gs = [x * (it + 1) for x in grads]
        for i in range(len(dp)):
            dg[i].copy_(gs[i].to(DEV))
        k.grad_sumsq(dd, len(dp), max_numel, n_groups, sumsq, ws, ticket=tickets)
        k.adam_step(dd, len(dp), max_numel, sumsq, 1.0, 0.01, 0.9, 0.999, 1e-8, step, fused=fused)
        if fused:
            assert step.item() == it        # read, not advanced
            step += 1
        assert step.item() == it + 1       # one increment per adam_step
        assert not fused or int(tickets.abs().sum()) == 0
        clipped = []
        for gr in range(n_groups):
            idx = [i for i in range(len(dp)) if groups[i] == gr]
            cg, _ = O.clip_grad_norm([gs[i] for i in idx])
            ref = sum(float((gs[i].double() ** 2).sum()) for i in idx)   # exact; torch's f32 norm is ~3e-5 off here
            if ref == ref:
                assert abs(sumsq[gr].item() - ref) <= 1e-5 * ref + 1e-6, (gr, sumsq[gr].item(), ref)
            else:
                assert sumsq[gr].item() != sumsq[gr].item()
            clipped.append(dict(zip(idx, cg)))
        cg_all = [clipped[groups[i]][i] for i in range(len(dp))]
        cur = adam.step(cur, cg_all)
    for i, (a, b) in enumerate(zip(dp, cur)):
        if nan_group is not None and groups[i] == nan_group:
            assert torch.isnan(a).all() and torch.isnan(b).all(), i
            continue
        assert torch.allclose(a.cpu(), b, rtol=1e-5, atol=1e-6), i
        if sh[i] is not None:
            rows, cols = sh[i].shape
            assert torch.equal(sh[i], a.view(rows, cols).to(torch.bfloat16))
            assert torch.equal(sht[i], a.view(rows, cols).t().to(torch.bfloat16))


def test_clip_and_adam_one_launch_bit_identical():
    """The one-launch norm and Adam (tickets) give the two-launch forms' parameters, moments,
    gradients, bf16 shadows and transposed shadows bit for bit (big case, 3 steps; the fused
    form's step counter advanced by llp_step_end2, as the engines do), on the 2-D grids and on
    the compact grids of llp_grad_sumsq_w / llp_adam_step_w (round 5, the engines' default)."""
    k = K()
    spec = _ADAM_CASES["big"]
    g = torch.Generator().manual_seed(77)
    shapes = [sh for sh, _, _ in spec]
    groups = [gr for _, gr, _ in spec]
    n_groups = max(groups) + 1
    params = [torch.randn(*s, generator=g) for s in shapes]
    grads = [torch.randn(*s, generator=g) * 3 for s in shapes]
    max_numel = max(p.numel() for p in params)
    runs = []
    for fused, compact in ((False, False), (True, False), (True, True)):
        dp = [p.to(DEV).clone() for p in params]
        dg = [x.to(DEV).clone() for x in grads]
        m = [torch.zeros_like(p) for p in dp]
        v = [torch.zeros_like(p) for p in dp]
        sh, descs = [], []
        for i, p in enumerate(dp):
            rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
            s_ = st_ = None
            if spec[i][2]:
                s_ = torch.zeros(rows, cols, dtype=torch.bfloat16, device=DEV)
                st_ = torch.zeros(cols, rows, dtype=torch.bfloat16, device=DEV)
            sh += [s_, st_]
            descs.append(k.TensorDesc(p.data_ptr(), dg[i].data_ptr(), m[i].data_ptr(), v[i].data_ptr(),
                                      k.ptr(s_), k.ptr(st_), p.numel(), rows, cols, groups[i],
                                      k.LLP_BF16 if s_ is not None else 0))
        dd = k.descs_to_device(descs, DEV)
        sumsq = torch.zeros(n_groups, device=DEV)
        ws = torch.empty(k.grad_sumsq_ws_bytes(len(dp), max_numel) // 4 + 16, device=DEV)
        step = torch.zeros(1, dtype=torch.int64, device=DEV)
        tickets = k.ticket_block(DEV)
        loss, loss_sum = torch.ones(1, device=DEV), torch.zeros(1, dtype=torch.float64, device=DEV)
        ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
        for it in range(3):
            for i in range(len(dp)):
                dg[i].copy_((grads[i] * (it + 1)).to(DEV))
            nw_s, nw_a = k.work_items([(p.numel(), *((p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())),
                                        bool(spec[i][2])) for i, p in enumerate(dp)]) if compact else (0, 0)
            k.grad_sumsq(dd, len(dp), max_numel, n_groups, sumsq, ws, ticket=tickets if fused else None, n_work=nw_s)
            k.adam_step(dd, len(dp), max_numel, sumsq, 1.0, 0.01, 0.9, 0.999, 1e-8, step, fused=fused, n_work=nw_a)
            if fused:
                k.step_end(loss, 2.0, loss_sum, ctr, adam_step=step)
        torch.cuda.synchronize()
        assert not fused or (int(ctr.item()) == 3 and float(loss_sum.item()) == 6.0
                             and int(tickets.abs().sum()) == 0)
        runs.append((dp, dg, m, v, [x for x in sh if x is not None], sumsq, int(step.item())))
    for r in runs[1:]:
        for a, b in zip(runs[0][:5], r[:5]):
            for x, y in zip(a, b):
                assert torch.equal(x, y)
        assert torch.equal(runs[0][5], r[5]) and runs[0][6] == r[6] == 3


# ------------------------------------------------------------------ unique-node compaction
@pytest.mark.parametrize("N,R,hot,hub", [(235868, 747214, 2000, 0.0), (3000, 40000, 0, 0.3), (50, 1000, 0, 0.0)])
def test_dedup_segsort_wave(N, R, hot, hub):
    """dedup.hip's segment sort: segments of 33..1024 rows ranked one wave each across the
    grid (segsort_mid_wave_kernel), longer ones by a block; outputs equal the stable sort's.
    hot: a quarter of the rows on ids 0..hot-1 (the stress probe: ~94-row segments on
    neighbouring ids); hub: as test_dedup_rows_and_segment_sum (a 12k-row segment)."""
    k = K()
    g = torch.Generator().manual_seed(R + 5)
    target = torch.randint(0, N, (R,), generator=g, dtype=torch.int32)
    if hot:
        target[: R // 4] = torch.randint(0, hot, (R // 4,), generator=g, dtype=torch.int32)
    if hub:
        u = torch.rand(R, generator=g)
        target[u < hub] = 7
    tg = target.to(DEV)
    uniq = torch.empty(R, dtype=torch.int32, device=DEV)
    pos = torch.empty(R, dtype=torch.int32, device=DEV)
    nu = torch.empty(1, dtype=torch.int32, device=DEV)
    segp = torch.empty(R + 1, dtype=torch.int32, device=DEV)
    segr = torch.empty(R, dtype=torch.int32, device=DEV)
    ws = torch.empty(k.dedup_ws_bytes(N, R) // 4 + 16, device=DEV)
    k.dedup_rows(N, R, tg, uniq, pos, nu, segp, segr, ws)
    torch.cuda.synchronize()
    u_ref, inv = np.unique(target.numpy(), return_inverse=True)
    U = int(nu.item())
    assert U == u_ref.size
    assert np.array_equal(uniq[:U].cpu().numpy(), u_ref)
    assert np.array_equal(pos.cpu().numpy(), inv)
    assert np.array_equal(segr.cpu().numpy(), np.argsort(inv, kind="stable"))


@pytest.mark.parametrize("N,R,hub", [(50, 1000, 0.0), (235868, 20000, 0.0), (7, 7, 0.0), (3000, 40000, 0.3)])
def test_dedup_rows_and_segment_sum(N, R, hub):
    """hub > 0: that fraction of the rows on node 7 and 2 % on each of nodes 11..15, so the
    counting path's long-segment sorts run from LDS (~800 rows) and from scratch (12k rows)."""
    k = K()
    g = torch.Generator().manual_seed(R)
    target = torch.randint(0, N, (R,), generator=g, dtype=torch.int32)
    if hub:
        u = torch.rand(R, generator=g)
        target[u < hub] = 7
        for j, v in enumerate(range(11, 16)):
            lo = hub + 0.02 * j
            target[(u >= lo) & (u < lo + 0.02)] = v
    tg = target.to(DEV)
    uniq = torch.empty(R, dtype=torch.int32, device=DEV)
    pos = torch.empty(R, dtype=torch.int32, device=DEV)
    nu = torch.empty(1, dtype=torch.int32, device=DEV)
    segp = torch.empty(R + 1, dtype=torch.int32, device=DEV)
    segr = torch.empty(R, dtype=torch.int32, device=DEV)
    ws = torch.empty(k.dedup_ws_bytes(N, R) // 4 + 16, device=DEV)
    k.dedup_rows(N, R, tg, uniq, pos, nu, segp, segr, ws)
    torch.cuda.synchronize()
    u_ref, inv = np.unique(target.numpy(), return_inverse=True)
    U = int(nu.item())
    assert U == u_ref.size
    assert np.array_equal(uniq[:U].cpu().numpy(), u_ref)
    assert np.array_equal(pos.cpu().numpy(), inv)
    rows_ref = np.argsort(inv, kind="stable")          # rows grouped by slot, in row order
    assert np.array_equal(segr.cpu().numpy(), rows_ref)
    assert np.array_equal(segp[:U + 1].cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(inv))]))
    for dt in (torch.float32, torch.bfloat16):
        src = torch.randn(R, 64, generator=g).to(DEV, dt)
        out = torch.empty(U, 64, device=DEV, dtype=dt)
        k.segment_sum_rows(U, segp, segr, src, out)
        ref = torch.zeros(U, 64).index_add_(0, torch.from_numpy(inv).long(), src.float().cpu())
        tol = 1e-5 if dt == torch.float32 else 2e-2
        assert torch.allclose(out.float().cpu(), ref, rtol=tol, atol=tol * max(1.0, ref.abs().max().item()))
    idx = torch.randint(0, R, (333,), generator=g, dtype=torch.int32)
    o = torch.empty(333, dtype=torch.int32, device=DEV)
    k.gather_i32(idx.to(DEV), pos, o)
    assert np.array_equal(o.cpu().numpy(), inv[idx.numpy()])


@pytest.mark.parametrize("N,R,hot,hub", [(235868, 747214, 2000, 0.0), (3000, 40000, 0, 0.3), (50, 1000, 0, 0.0),
                                         (7, 7, 0, 0.0), (31044, 263_000, 0, 0.0), (200_000, 5, 0, 0.0)])
def test_dedup_rows2_four_launches(N, R, hot, hub):
    """llp_dedup_rows2 (counts, one look-back scan + compaction pass, scatter, one fused segment
    sort) == the stable sort's outputs, on one workspace over five calls with fresh targets
    (the persistent counts / epoch-tagged flags / ticket must come back clean each time, and the
    first call zeroes them), the rows of absent nodes zeroed, the others untouched, and the
    look-back's error word clear.  Hot / hub cases put 33..1024-row and 12k-row segments on
    neighbouring ids (the wave and block sorts inside the one launch)."""
    k = K()
    g = torch.Generator().manual_seed(N + R)
    dws = k.DedupWorkspace(N, R, DEV)
    H = 24
    for call in range(5):
        target = torch.randint(0, N, (R,), generator=g, dtype=torch.int32)
        if hot:
            target[: R // 4] = torch.randint(0, hot, (R // 4,), generator=g, dtype=torch.int32)
        if hub:
            u = torch.rand(R, generator=g)
            target[u < hub] = 7
            for j, v in enumerate(range(11, 16)):
                lo = hub + 0.02 * j
                target[(u >= lo) & (u < lo + 0.02)] = v
        tg = target.to(DEV)
        uniq = torch.empty(R, dtype=torch.int32, device=DEV)
        pos = torch.empty(R, dtype=torch.int32, device=DEV)
        nu = torch.empty(1, dtype=torch.int32, device=DEV)
        segp = torch.empty(R + 1, dtype=torch.int32, device=DEV)
        segr = torch.empty(R, dtype=torch.int32, device=DEV)
        rows = torch.full((N, H), 5.0, device=DEV, dtype=torch.bfloat16)
        k.dedup_rows2(N, R, tg, uniq, pos, nu, segp, segr, dws, zero_rows=rows if call % 2 == 0 else None)
        torch.cuda.synchronize()
        assert int(dws.error_word().item()) == 0
        u_ref, inv = np.unique(target.numpy(), return_inverse=True)
        U = int(nu.item())
        assert U == u_ref.size, call
        assert np.array_equal(uniq[:U].cpu().numpy(), u_ref), call
        assert np.array_equal(pos.cpu().numpy(), inv), call
        assert np.array_equal(segr.cpu().numpy(), np.argsort(inv, kind="stable")), call
        assert np.array_equal(segp[:U + 1].cpu().numpy(), np.concatenate([[0], np.cumsum(np.bincount(inv))])), call
        present = np.zeros(N, dtype=bool)
        present[u_ref] = True
        r = rows.float().cpu().numpy()
        if call % 2 == 0:
            assert (r[~present] == 0).all() and (r[present] == 5).all(), call
        else:
            assert (r == 5).all(), call


@pytest.mark.parametrize("dtype,F", [(torch.bfloat16, 128), (torch.bfloat16, 13), (torch.float32, 37)])
def test_gather_rows(dtype, F):
    """llp_gather_rows: out[r] = x[idx[r]] bit-exact, rows past the device count untouched
    (x[this_target], src/main.py:95)."""
    k = K()
    g = torch.Generator().manual_seed(F)
    N, R, live = 1000, 777, 500
    x = torch.randn(N, F, generator=g).to(DEV, dtype)
    idx = torch.randint(0, N, (R,), generator=g, dtype=torch.int32).to(DEV)
    out = torch.full((R, F), 7.0, device=DEV, dtype=dtype)
    k.gather_rows(x, idx, out)
    assert torch.equal(out, x[idx.long()])
    out.fill_(7.0)
    cnt = torch.tensor([live], dtype=torch.int32, device=DEV)
    k.gather_rows(x, idx, out, count=cnt)
    assert torch.equal(out[:live], x[idx[:live].long()])
    assert bool((out[live:] == 7.0).all())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("inner", [False, True])
@pytest.mark.parametrize("N,H", [(400, 256), (400, 1024), (5, 512)])
def test_hadamard_bwd_segments(dtype, inner, N, H):
    """Fused Hadamard backward reduced onto unique nodes == per-row gradients
    (anchor rows sum their C contexts) index-added by node, f32.  H picks the
    thread-group kernel (bf16 H=256) or the wave-per-node kernel (rows of 64, 128
    or 256 16-B chunks); N=5 gives segments longer than one wave's 64 rows."""
    k = K()
    g = torch.Generator().manual_seed(5)
    B, C, L2 = 37, 6, 53
    R1 = B * (C + 1) + 2 * L2
    R2 = B * C + L2
    target = torch.randint(0, N, (R1,), generator=g, dtype=torch.int32)
    tg = target.to(DEV)
    uniq = torch.empty(R1, dtype=torch.int32, device=DEV)
    pos = torch.empty(R1, dtype=torch.int32, device=DEV)
    nu = torch.empty(1, dtype=torch.int32, device=DEV)
    segp = torch.empty(R1 + 1, dtype=torch.int32, device=DEV)
    segr = torch.empty(R1, dtype=torch.int32, device=DEV)
    ws = torch.empty(k.dedup_ws_bytes(N, R1) // 4 + 16, device=DEV)
    k.dedup_rows(N, R1, tg, uniq, pos, nu, segp, segr, ws)
    U = int(nu.item())
    h = torch.randn(U, H, generator=g).to(DEV, dtype)
    dZ = torch.randn(R2, H, generator=g).to(DEV, dtype)
    drow = torch.randn(R2, generator=g).to(DEV)
    out = torch.empty(U, H, device=DEV, dtype=dtype)
    arow = torch.empty(B, H, device=DEV, dtype=dtype)
    k.hadamard_bwd_segments(U, B, C, L2, H, segp, segr, pos, None if inner else dZ, h, out, arow,
                            drow=drow if inner else None)
    # bit-identical to the two-kernel path (row gradients, then the per-node segment sum)
    rows_dev = torch.empty(R1, H, device=DEV, dtype=dtype)
    k.hadamard_bwd_blocks(B, C, L2, H, None if inner else dZ, h, rows_dev, drow=drow if inner else None, hidx=pos)
    out2 = torch.empty(U, H, device=DEV, dtype=dtype)
    k.segment_sum_rows(U, segp, segr, rows_dev, out2)
    torch.cuda.synchronize()
    assert torch.equal(out, out2), (out.float() - out2.float()).abs().max().item()
    hr = h.float().cpu()[pos.cpu().long()]                              # [R1, H] rows of h per target row
    d = drow.cpu().unsqueeze(1).expand(R2, H) if inner else dZ.float().cpu()
    C1 = C + 1
    rows = torch.zeros(R1, H)
    for b in range(B):
        a = b * C1
        for cc in range(C):
            z = b * C + cc
            rows[a] += d[z] * hr[a + 1 + cc]
            rows[a + 1 + cc] = d[z] * hr[a]
    base = B * C1
    for i in range(L2):
        z = B * C + i
        rows[base + i] = d[z] * hr[base + L2 + i]
        rows[base + L2 + i] = d[z] * hr[base + i]
    ref = torch.zeros(U, H).index_add_(0, pos.cpu().long(), rows)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(out.float().cpu(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("dtype,out_f32", [(torch.float32, False), (torch.bfloat16, False), (torch.bfloat16, True)])
@pytest.mark.parametrize("inner", [False, True])
@pytest.mark.parametrize("H", [128, 256, 1024])
def test_hadamard_bwd_segments_label_rows_onto_nodes(dtype, out_f32, inner, H):
    """The full-batch form (DistillEngine._hadamard_bwd_nodes): B = C = 0, pos = [ia | ib]
    node ids, h the [N, H] node table, each node's sum written to row out_rows[u] = its
    node id of a zeroed [N, H] output (compute dtype, or f32 unrounded): bit-identical to
    llp_hadamard_bwd_blocks + llp_segment_sum_rows(out_rows) (the round-3 path)."""
    k = K()
    g = torch.Generator().manual_seed(H + 3 * inner)
    N, R = 700, 2500                                   # R pairs, 2R endpoint rows, skewed degrees
    ia = (torch.randint(0, N, (R,), generator=g) ** 2 // N).to(torch.int32)
    ib = torch.randint(0, N, (R,), generator=g).to(torch.int32)
    tgt = torch.cat([ia, ib]).to(DEV)
    R2 = 2 * R
    uniq, pos = (torch.empty(R2, dtype=torch.int32, device=DEV) for _ in range(2))
    nu = torch.empty(1, dtype=torch.int32, device=DEV)
    segp = torch.empty(R2 + 1, dtype=torch.int32, device=DEV)
    segr = torch.empty(R2, dtype=torch.int32, device=DEV)
    ws = torch.empty(k.dedup_ws_bytes(N, R2) // 4 + 16, device=DEV)
    k.dedup_rows(N, R2, tgt, uniq, pos, nu, segp, segr, ws)
    h = torch.randn(N, H, generator=g).to(DEV, dtype)
    dZ = torch.randn(R, H, generator=g).to(DEV, dtype)
    drow = torch.randn(R, generator=g).to(DEV)
    odt = torch.float32 if out_f32 else dtype
    out = torch.full((N, H), 5.0, device=DEV, dtype=odt)
    out.zero_()
    U = min(R2, N)
    k.hadamard_bwd_segments(U, 0, 0, R, H, segp, segr, tgt, None if inner else dZ, h, out, None,
                            drow=drow if inner else None, count=nu, out_rows=uniq)
    rows = torch.empty(R2, H, device=DEV, dtype=dtype)
    k.hadamard_bwd_blocks(0, 1, R, H, None if inner else dZ, h, rows, drow=drow if inner else None, hidx=tgt)
    out2 = torch.zeros(N, H, device=DEV, dtype=odt)
    k.segment_sum_rows(U, segp, segr, rows, out2, count=nu, out_rows=uniq)
    torch.cuda.synchronize()
    assert torch.equal(out, out2), (out.float() - out2.float()).abs().max().item()
    # and against the definition: d(h[ia] * h[ib]) summed per node
    d = drow.cpu().unsqueeze(1).expand(R, H) if inner else dZ.float().cpu()
    hf = h.float().cpu()
    ref = torch.zeros(N, H)
    ref.index_add_(0, ia.long(), d * hf[ib.long()])
    ref.index_add_(0, ib.long(), d * hf[ia.long()])
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert torch.allclose(out.float().cpu(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("M,N,Kd", [(1000, 1024, 128), (517, 96, 256), (300, 288, 64)])
def test_gemm_relu_bit_mask(M, N, Kd):
    """act=RELU with a uint8 aux writes bit c%8 of byte c/8 = (bf16 output > 0);
    act=RELU_BWD reading that mask equals RELU_BWD reading the bf16 activations."""
    k = K()
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    mask = torch.full((M, N // 8), 0xAB, dtype=torch.uint8, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)          # kept alive: the kernel reads it
    drop = k.Dropout(0.25, 77, ctr.data_ptr(), 3)
    k.gemm_nt(k.operand(x), k.operand(w), M, N, Kd, y, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=mask, dropout=drop)
    y2 = torch.empty_like(y)
    k.gemm_nt(k.operand(x), k.operand(w), M, N, Kd, y2, k.LLP_BF16, bias=b, act=k.ACT_RELU, dropout=drop)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)                                      # writing the mask changes nothing else
    pos = (y.float() > 0).cpu().numpy()
    bits = np.unpackbits(mask.cpu().numpy(), axis=1, bitorder="little")
    assert np.array_equal(bits.astype(bool), pos)
    gy = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    # any [M, N] product exercises the RELU_BWD epilogue: C = gy . w^T (B = w, [N, Kd])
    assert w.shape == (N, Kd)
    d_aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    d_msk = torch.empty_like(d_aux)
    k.gemm_nt(k.operand(gy), k.operand(w), M, N, Kd, d_aux, k.LLP_BF16, act=k.ACT_RELU_BWD, aux=y, alpha=1.5)
    k.gemm_nt(k.operand(gy), k.operand(w), M, N, Kd, d_msk, k.LLP_BF16, act=k.ACT_RELU_BWD, aux=mask, alpha=1.5)
    torch.cuda.synchronize()
    assert torch.equal(d_aux, d_msk)


# ------------------------------------------------------------------ device row count (llp_operand.rows_dev)
@pytest.mark.parametrize("dt", ["fp32", "bf16"])
@pytest.mark.parametrize("Mmax,Mlive", [(3000, 2311), (1000, 0), (700, 700), (257, 1)])
def test_gemm_device_row_count(dt, Mmax, Mlive):
    """A GEMM launched for Mmax rows with rows_dev = Mlive: rows < Mlive are
    bit-identical to a launch for exactly Mlive rows, rows past it untouched
    (NT: C rows; TN and its fused bias gradient: only live rows contract).
    This is the unique-node student's sync-free path (no host read of U)."""
    k = K()
    g = torch.Generator().manual_seed(Mmax + Mlive)
    tdt = torch.float32 if dt == "fp32" else torch.bfloat16
    code = k.dtype_code(tdt)
    N0, Kd, N = 4000, 128, 256
    X = torch.randn(N0, Kd, generator=g).to(DEV, tdt)
    idx = torch.randint(0, N0, (Mmax,), generator=g, dtype=torch.int32).to(DEV)
    W = (torch.randn(N, Kd, generator=g) * 0.1).to(DEV, tdt)
    b = torch.randn(N, generator=g).to(DEV)
    cnt = torch.tensor([Mlive], dtype=torch.int32, device=DEV)
    sentinel = torch.full((Mmax, N), 7.0, device=DEV, dtype=tdt)
    out = sentinel.clone()
    k.gemm_nt(k.operand(X, idx, count=cnt), k.operand(W), Mmax, N, Kd, out, code, bias=b, act=k.ACT_RELU)
    ref = sentinel.clone()
    if Mlive:
        k.gemm_nt(k.operand(X, idx[:Mlive]), k.operand(W), Mlive, N, Kd, ref[:Mlive], code, bias=b, act=k.ACT_RELU)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # TN with the bias gradient fused: dW = A^T X[idx], db = colsum(A)
    A = torch.randn(Mmax, N, generator=g).to(DEV, tdt)
    ws = torch.empty(k.gemm_tn_ws_bytes(code, Mmax, N, Kd) // 4 + 16, device=DEV)
    dW = torch.empty(N, Kd, device=DEV)
    db = torch.empty(N, device=DEV)
    k.gemm_tn(k.operand(A, count=cnt), k.operand(X, idx, count=cnt), Mmax, N, Kd, dW, code, ws, colsum_a=db)
    torch.cuda.synchronize()
    Ar, Xr = A[:Mlive].double().cpu(), X[idx[:Mlive].long()].double().cpu()
    refW = Ar.t() @ Xr
    refb = Ar.sum(0)
    tol = 1e-4 if dt == "fp32" else 2e-3
    assert (dW.cpu().double() - refW).abs().max().item() <= tol * (1 + refW.abs().max().item())
    assert (db.cpu().double() - refb).abs().max().item() <= tol * (1 + refb.abs().max().item())
    # segment sum over min(U, count) groups
    R = 2 * Mmax + 1
    segp = torch.arange(0, R + 1, 2, dtype=torch.int32, device=DEV)[:Mmax + 1].contiguous()
    segr = torch.arange(R, dtype=torch.int32, device=DEV)
    src = torch.randn(R, 64, generator=g).to(DEV, tdt)
    o = torch.full((Mmax, 64), 7.0, device=DEV, dtype=tdt)
    k.segment_sum_rows(Mmax, segp, segr, src, o, count=cnt)
    torch.cuda.synchronize()
    exp = src.float().cpu()[:2 * Mmax].view(Mmax, 2, 64).sum(1)
    got = o.float().cpu()
    assert torch.allclose(got[:Mlive], exp[:Mlive], rtol=1e-2, atol=1e-2)
    assert bool((got[Mlive:] == 7.0).all())


@pytest.mark.parametrize("off,nbytes", [(0, 4096), (3, 517), (16, 15), (1, 1), (5, 1_000_003)])
def test_zero_bytes_exact_region(off, nbytes):
    """llp_zero (a kernel, not a memset node): exactly bytes [off, off + nbytes) become 0."""
    k = K()
    buf = torch.full((nbytes + off + 64,), 0xAB, dtype=torch.uint8, device=DEV)
    view = buf[off:off + nbytes]
    k.zero_(view)
    torch.cuda.synchronize()
    h = buf.cpu()
    assert int((h[off:off + nbytes] != 0).sum()) == 0
    assert int((h[:off] != 0xAB).sum()) == 0 and int((h[off + nbytes:] != 0xAB).sum()) == 0


def _nt_sliced(k, A, W, M, N, Kd, dtype_code, slice_rows, **kw):
    """The same GEMM in row slices of <= 256 tiles each (the non-persistent pp8 kernel)."""
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    mask = kw.pop("mask", None)
    aux = kw.pop("aux", None)
    for s in range(0, M, slice_rows):
        e = min(M, s + slice_rows)
        k.gemm_nt(k.operand(A[s:e]), k.operand(W), e - s, N, Kd, C[s:e], dtype_code,
                  aux=(mask[s:e] if mask is not None else (aux[s:e] if aux is not None else None)), **kw)
    return C


@pytest.mark.parametrize("mode,M,N,Kd", [("relu", 70_000, 1024, 1024), ("none", 70_001, 512, 256),
                                          ("bwd", 70_000, 1024, 1024), ("relu", 70_000, 256, 128),
                                          ("none", 2_000, 9216, 256)])
def test_gemm_nt_f32_persistent(mode, M, N, Kd):
    """gemm_nt_f32_pp8p (the bf16 persistent kernel's LDS-DMA pipeline on f32 operands, launched
    above 256 tiles) against the register-staged 128 x 128 f32 kernel on row slices of <= 256
    tiles, and against a float64 reference: bias + ReLU (torch's NaN rule), plain, ReLU backward
    through stored f32 activations with alpha 2; a partial last m-tile, a walk along one m-tile's
    n-tiles (N = 9216) and a device row count."""
    k = K()
    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randn(M, Kd, generator=g).to(DEV)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    kw = {}
    if mode == "relu":
        kw = dict(bias=b, act=k.ACT_RELU)
    elif mode == "none":
        kw = dict(bias=b)
    else:
        Y = torch.relu(torch.randn(M, N, generator=g)).to(DEV)
        kw = dict(act=k.ACT_RELU_BWD, aux=Y, alpha=2.0)
    C1 = torch.empty(M, N, device=DEV)
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C1, k.LLP_F32, **kw)
    assert "f32_pp8p" in k.last_gemm_kernel(), k.last_gemm_kernel()
    sl = min(64, 256 // (N // 256)) * 256
    C2 = torch.empty(M, N, device=DEV)
    aux = kw.pop("aux", None)
    for s in range(0, M, sl):
        e = min(M, s + sl)
        k.gemm_nt(k.operand(A[s:e]), k.operand(W), e - s, N, Kd, C2[s:e], k.LLP_F32,
                  aux=aux[s:e] if aux is not None else None, **kw)
    assert "f32_pp8p" not in k.last_gemm_kernel()
    torch.cuda.synchronize()
    ref = A.double() @ W.double().t()
    if mode == "bwd":
        ref = 2.0 * ref * (aux.double() > 0)
    else:
        ref = ref + b.double()
        if mode == "relu":
            ref = torch.relu(ref)
    scale = 1 + ref.abs().max().item()
    assert (C1.double() - ref).abs().max().item() <= 2e-5 * scale
    # the same k order per accumulator as the register-staged kernel
    assert torch.equal(C1, C2)
    if mode == "relu":   # device row count: rows past it untouched
        cnt = torch.tensor([M - 300], dtype=torch.int32, device=DEV)
        C3 = torch.full((M, N), 7.0, device=DEV)
        k.gemm_nt(k.operand(A, count=cnt), k.operand(W), M, N, Kd, C3, k.LLP_F32, **kw)
        torch.cuda.synchronize()
        assert torch.equal(C3[:M - 300], C1[:M - 300])
        assert bool((C3[M - 300:] == 7.0).all())


@pytest.mark.parametrize("mode,M,N,Kd", [("relu_mask", 70_000, 1024, 1024), ("relu_mask", 70_000, 1024, 128),
                                          ("none", 70_001, 512, 256), ("bwd_mask", 70_000, 1024, 1024),
                                          ("relu", 70_000, 256, 1024), ("none", 2_000, 9216, 256)])
def test_gemm_nt_persistent_bit_identical(mode, M, N, Kd):
    """gemm_nt_bf16_pp8p (one workgroup per CU, the next tile's first K-tile prefetched under
    the epilogue; launched above 256 tiles) against pp8 on row slices of 64 m-tiles (<= 256
    tiles): C and the ReLU bit masks bit for bit, including a partial last m-tile, m-tile
    counts that are not a multiple of 8 and a walk along one m-tile's n-tiles (N = 9216)."""
    k = K()
    g = torch.Generator().manual_seed(M + Kd)
    A = torch.relu(torch.randn(M, Kd, generator=g)).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV) * 0.1
    sl = min(64, 256 // (N // 256)) * 256
    if mode in ("relu_mask", "relu"):
        C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        m1 = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8) if mode == "relu_mask" else None
        k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C1, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=m1)
        m2 = torch.empty_like(m1) if m1 is not None else None
        C2 = _nt_sliced(k, A, W, M, N, Kd, k.LLP_BF16, sl, bias=b, act=k.ACT_RELU, mask=m2)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2)
        if m1 is not None:
            assert torch.equal(m1, m2)
    elif mode == "none":
        C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C1, k.LLP_BF16)
        C2 = _nt_sliced(k, A, W, M, N, Kd, k.LLP_BF16, sl)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2)
    else:
        Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        mask = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8)
        k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, Y, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=mask)
        G = (torch.randn(M, Kd, generator=g)).to(DEV, torch.bfloat16)
        Wt = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
        # dX [M, N] = (G @ Wt^T) * (mask bits), alpha 2
        C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        k.gemm_nt(k.operand(G), k.operand(Wt), M, N, Kd, C1, k.LLP_BF16, act=k.ACT_RELU_BWD, aux=mask, alpha=2.0)
        C2 = _nt_sliced(k, G, Wt, M, N, Kd, k.LLP_BF16, sl, act=k.ACT_RELU_BWD, aux=mask, alpha=2.0)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2)
        ref = 2.0 * (G.float() @ Wt.float().t()) * (Y.float() > 0)
        assert torch.allclose(C1.float(), ref, rtol=2e-2, atol=2e-2 * (1 + ref.abs().max().item()))


@pytest.mark.parametrize("mode", ["relu_mask", "bwd_mask"])
def test_gemm_nt_persistent_race_screen(mode):
    """Race screen of the persistent kernel's DMA schedule (three half K-tiles in flight, the
    next tile's K-tile 0 issued across the tile boundary) at the collab student shape: six
    launches on fresh random operands, each bit-identical to pp8 on row slices."""
    k = K()
    M, N, Kd = 225_280, 1024, 1024
    g = torch.Generator().manual_seed(5)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV) * 0.1
    mask = None
    if mode == "bwd_mask":
        mask = torch.randint(0, 256, (M, N // 8), generator=g, dtype=torch.uint8).to(DEV)
    for it in range(6):
        A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
        C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        if mode == "relu_mask":
            m1 = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8)
            k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C1, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=m1)
            m2 = torch.empty_like(m1)
            C2 = _nt_sliced(k, A, W, M, N, Kd, k.LLP_BF16, 64 * 256, bias=b, act=k.ACT_RELU, mask=m2)
            torch.cuda.synchronize()
            assert torch.equal(m1, m2), it
        else:
            k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C1, k.LLP_BF16, act=k.ACT_RELU_BWD, aux=mask, alpha=0.5)
            C2 = _nt_sliced(k, A, W, M, N, Kd, k.LLP_BF16, 64 * 256, act=k.ACT_RELU_BWD, aux=mask, alpha=0.5)
            torch.cuda.synchronize()
        assert torch.equal(C1, C2), it


def test_gemm_nt_persistent_device_row_count():
    """The persistent kernel with a device row count (the unique-node student): rows past the
    count are neither computed nor stored, the live rows equal pp8 on row slices."""
    k = K()
    g = torch.Generator().manual_seed(11)
    Mh, Ml, N, Kd = 80_000, 71_333, 1024, 1024
    A = torch.relu(torch.randn(Mh, Kd, generator=g)).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV) * 0.1
    cnt = torch.tensor([Ml], dtype=torch.int32, device=DEV)
    C1 = torch.full((Mh, N), 7.0, device=DEV, dtype=torch.bfloat16)
    m1 = torch.zeros(Mh, N // 8, device=DEV, dtype=torch.uint8)
    k.gemm_nt(k.operand(A, count=cnt), k.operand(W), Mh, N, Kd, C1, k.LLP_BF16, bias=b, act=k.ACT_RELU, aux=m1)
    m2 = torch.zeros(Ml, N // 8, device=DEV, dtype=torch.uint8)
    C2 = _nt_sliced(k, A[:Ml], W, Ml, N, Kd, k.LLP_BF16, 64 * 256, bias=b, act=k.ACT_RELU, mask=m2)
    torch.cuda.synchronize()
    assert torch.equal(C1[:Ml], C2) and torch.equal(m1[:Ml], m2)
    assert bool((C1[Ml:].float() == 7.0).all()) and int(m1[Ml:].sum()) == 0


@pytest.mark.parametrize("M,N,Kd,with_c", [(70_000, 1024, 1024, True), (70_000, 1024, 1024, False),
                                           (3_000, 9216, 256, True)])
def test_gemm_nt_persistent_head_bit_identical(M, N, Kd, with_c):
    """The fused-head GEMM (predictor's last hidden layer + Linear(N,1)) in the persistent
    kernel (gemm_nt_bf16_pp8p<EPI_HEAD_LEAN>: bias and head weights DMA'd into LDS per tile,
    the quad partials in the mask region) against pp8<EPI_HEAD_LEAN> on row slices of
    <= 256 tiles: C and every head partial bit for bit, with and without C."""
    k = K()
    g = torch.Generator().manual_seed(M + N)
    A = torch.relu(torch.randn(M, Kd, generator=g)).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV) * 0.1
    hw = torch.randn(N, generator=g).to(DEV)
    parts = k.head_parts(N)
    C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if with_c else None
    h1 = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, C1, hw, h1, bias=b, act=k.ACT_RELU)
    sl = min(64, 256 // (N // 256)) * 256
    C2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    h2 = torch.empty(parts, M, device=DEV)
    for s in range(0, M, sl):
        e = min(M, s + sl)
        hs = torch.empty(parts, e - s, device=DEV)
        k.gemm_nt_head(k.operand(A[s:e]), k.operand(W), e - s, N, Kd, C2[s:e], hw, hs, bias=b, act=k.ACT_RELU)
        h2[:, s:e] = hs
    torch.cuda.synchronize()
    if with_c:
        assert torch.equal(C1, C2)
    assert torch.equal(h1, h2)
    ref = C2.float() @ hw
    assert torch.allclose(h1.sum(0), ref, rtol=1e-4, atol=1e-4 * (1 + ref.abs().max().item()))


@pytest.mark.parametrize("with_c", [True, False])
def test_gemm_nt_persistent_head_dropout(with_c):
    """The teacher predictor's hidden layer in training (ReLU + dropout + fused Linear(N,1) head,
    gemm_nt_bf16_pp8p<EPI_HEAD_DROP>) at p = 0.5: C is where(keep, 2 x the no-dropout head
    GEMM's C, 0) bit for bit (keep = the oracle's dropout_keep), and the head partials sum to
    that C times the head weights."""
    k = K()
    M, N, Kd = 131_072, 256, 256
    g = torch.Generator().manual_seed(21)
    A = torch.randn(M, Kd, generator=g).to(DEV, torch.bfloat16)
    W = (torch.randn(N, Kd, generator=g) * Kd ** -0.5).to(DEV, torch.bfloat16)
    b = torch.randn(N, generator=g).to(DEV) * 0.1
    hw = torch.randn(N, generator=g).to(DEV)
    parts = k.head_parts(N)
    R = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, R, hw, torch.empty(parts, M, device=DEV), bias=b,
                   act=k.ACT_RELU)
    ctr = torch.full((1,), 3, dtype=torch.int64, device=DEV)
    D = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if with_c else None
    h = torch.empty(parts, M, device=DEV)
    k.gemm_nt_head(k.operand(A), k.operand(W), M, N, Kd, D, hw, h, bias=b, act=k.ACT_RELU,
                   dropout=k.Dropout(0.5, 17, ctr.data_ptr(), 4))
    assert "EPI_HEAD_DROP" in k.last_gemm_kernel()
    torch.cuda.synchronize()
    keep = torch.from_numpy(O.dropout_keep(17, O.STREAMS_PER_STEP * 3 + 4, M, N, 0.5)).to(DEV)
    exp = torch.where(keep, R.float() * 2.0, torch.zeros((), device=DEV)).to(torch.bfloat16)
    if with_c:
        assert torch.equal(D.view(torch.int16), exp.view(torch.int16))
    ref = exp.float() @ hw
    assert torch.allclose(h.sum(0), ref, rtol=1e-4, atol=1e-4 * (1 + ref.abs().max().item()))


def _mask_bits(m, N):
    sh = torch.arange(8, device=m.device, dtype=torch.int32)
    return ((m.to(torch.int32).unsqueeze(-1) >> sh) & 1).reshape(m.shape[0], N)


@pytest.mark.parametrize("M,N,Kd,relu", [(31_044, 256, 8_448, True), (7_761, 256, 8_448, True),
                                         (1_000, 512, 2_048, False)])
def test_gemm_nt_splitk(M, N, Kd, relu):
    """Split-K bf16 GEMM (llp_gemm_nt_splitk: f32 slabs over K ranges, one ordered reduce
    with bias, bf16 rounding, ReLU and the bit mask) at the physics first-layer shapes:
    deterministic, within bf16 rounding of the fp32 product, equal to the unsplit GEMM
    except where the two f32 sums round to neighbouring bf16 values, mask == (C != 0)."""
    k = K()
    S = k.gemm_nt_splitk_plan(M, N, Kd)
    assert S > 1
    g = torch.Generator().manual_seed(M + Kd)
    A = (torch.rand(M, Kd, generator=g) < 0.05).to(DEV, torch.bfloat16)      # binary features, as coauthor-physics
    W = (torch.randn(N, Kd, generator=g) * 0.05).to(DEV, torch.bfloat16)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV)
    act = k.ACT_RELU if relu else k.ACT_NONE
    ws = torch.empty(k.gemm_nt_splitk_ws_bytes(M, N, S) // 4, device=DEV)
    C1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    m1 = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8) if relu else None
    k.gemm_nt_splitk(k.operand(A), k.operand(W), M, N, Kd, C1, S, ws, bias=b, act=act, mask=m1)
    C2 = torch.empty_like(C1)
    m2 = torch.empty_like(m1) if relu else None
    k.gemm_nt_splitk(k.operand(A), k.operand(W), M, N, Kd, C2, S, ws, bias=b, act=act, mask=m2)
    C0 = torch.empty_like(C1)
    m0 = torch.empty_like(m1) if relu else None
    k.gemm_nt(k.operand(A), k.operand(W), M, N, Kd, C0, k.LLP_BF16, bias=b, act=act, aux=m0)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2) and (not relu or torch.equal(m1, m2))
    ref = A.float() @ W.float().t() + b
    if relu:
        ref = torch.relu(ref)
    err = (C1.float() - ref).abs()
    assert bool((err <= 2.0 ** -8 * ref.abs() + 1e-5).all()), err.max()
    diff = C1 != C0
    assert diff.float().mean().item() < 0.01
    assert bool(((C1.float() - C0.float()).abs()[diff] <= 2.0 ** -7 * C0.float().abs()[diff] + 1e-6).all())
    if relu:
        assert torch.equal(_mask_bits(m1, N), (C1 != 0).to(torch.int32))


# ------------------------------------------------------------------ owner decomposition (bit-exact)
def _owner_case(seed, N, B, C, P, n_neg, skew):
    g = np.random.default_rng(seed)
    C1 = C + 1
    if skew:   # most keys in the first node range: heavy overflow into the other ranks
        samples = np.minimum(g.integers(0, max(1, N // 5), (B, C1)), N - 1)
    else:
        samples = g.integers(0, N, (B, C1))
    pos = g.integers(0, N, (2, P))
    neg = g.integers(0, N, (2, n_neg))
    return samples, pos, neg


@pytest.mark.parametrize("N,B,C,P,n_neg", [(235_868, 13_110, 36, 65_536, 65_536), (1000, 37, 5, 111, 90),
                                           (50, 3, 2, 0, 7), (10, 1, 1, 1, 0)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("table", [False, True])
def test_pair_owner_assign_matches_oracle(N, B, C, P, n_neg, world, skew, table):
    """llp_pair_owner_assign == oracle pair_owner_assign for the three categories of one
    minibatch (context pairs keyed by the context node, label pairs by their source): sel,
    gpos and every rank's [ia | ib] rows, at the collab shape and small / skewed cases, with
    owners by id ranges or by a node -> owner table (DistillEngine's locality ownership)."""
    k = K()
    samples, pos, neg = _owner_case(B * 7 + world, N, B, C, P, n_neg, skew)
    tab = np.random.default_rng(N + world).integers(0, world, N).astype(np.int32) if table else None
    tab_d = torch.from_numpy(tab).to(DEV) if table else None
    C1 = C + 1
    n_lab = P + n_neg
    # the whole batch's this_target layout: samples.flat | src | dst (src/main.py:95)
    tgt = np.concatenate([samples.reshape(-1), pos[0], neg[0], pos[1], neg[1]]).astype(np.int32)
    td = torch.from_numpy(tgt).to(DEV)
    BC1 = B * C1
    ns = (B * C, P, n_neg)
    n_all = sum(ns)
    for rank in range(world):
        caps = [(rank + 1) * n // world - rank * n // world for n in ns]
        R2 = sum(caps)
        cats = [k.owner_cat(B * C, td, td, (C, C1, 0, 0), (C, C1, 1, 1), key_b=True),
                k.owner_cat(P, td[BC1:], td[BC1 + n_lab:]),
                k.owner_cat(n_neg, td[BC1 + P:], td[BC1 + n_lab + P:])]
        sel = torch.full((max(n_all, 1),), -7, dtype=torch.int32, device=DEV)
        gpos = torch.full((max(n_all, 1),), -7, dtype=torch.int32, device=DEV)
        rows = torch.full((max(2 * R2, 1),), -7, dtype=torch.int32, device=DEV)
        ws = torch.empty(k.pair_owner_ws_bytes(ns, world) // 4 + 16, dtype=torch.int32, device=DEV)
        k.pair_owner_assign(cats, N, world, rank, sel, ws, gpos=gpos, target=rows, R2=R2, owner_tab=tab_d)
        sel_h, gpos_h, rows_h = sel.cpu().numpy(), gpos.cpu().numpy(), rows.cpu().numpy()
        base = 0
        ia, ib = [], []
        keys = (samples[:, 1:].reshape(-1), pos[0], neg[0])
        ends = ((np.repeat(samples[:, 0], C), samples[:, 1:].reshape(-1)), (pos[0], pos[1]), (neg[0], neg[1]))
        for key, n, (ea, eb) in zip(keys, ns, ends):
            ref, off = O.pair_owner_assign(key, N, world, tab)
            assert np.array_equal(sel_h[base:base + n], ref)
            inv = np.empty(n, np.int64)
            inv[ref] = np.arange(n)
            assert np.array_equal(gpos_h[base:base + n], inv)
            mine = ref[off[rank]:off[rank + 1]]
            ia.append(ea[mine])
            ib.append(eb[mine])
            base += n
        assert np.array_equal(rows_h[:2 * R2], np.concatenate(ia + ib))
    # the oracle's rank split of the whole batch equals pair_owner_rank_items
    cs, ps, ns_ = O.pair_owner_rank_items(samples, pos, neg, N, world, world - 1)
    assert len(cs) + len(ps) + len(ns_) == sum((world * n) // world - ((world - 1) * n) // world for n in ns)


def test_pair_owner_scatter_and_loss_term_range():
    """llp_pair_owner_scatter places a rank's context logits into the [B, C] grid (zeros
    elsewhere); the sum over ranks is the whole grid, and llp_llp_loss with term ranges
    [rB/W, (r+1)B/W) gives the whole-batch terms summed over ranks, every gradient written."""
    k = K()
    N, B, C, W = 500, 24, 6, 3
    samples, pos, neg = _owner_case(5, N, B, C, 0, 0, False)
    key = samples[:, 1:].reshape(-1)
    sel, off = O.pair_owner_assign(key, N, W)
    gpos = np.empty(B * C, np.int64)
    gpos[sel] = np.arange(B * C)
    g = torch.Generator().manual_seed(3)
    s_all = torch.randn(B * C, generator=g)
    t_all = torch.rand(B * C, generator=g)
    gp = torch.from_numpy(gpos.astype(np.int32)).to(DEV)
    tot_s = torch.zeros(B * C, device=DEV)
    tot_t = torch.zeros(B * C, device=DEV)
    terms_sum = torch.zeros(4)
    for r in range(W):
        mine = torch.from_numpy(sel[off[r]:off[r + 1]])
        s_loc, t_loc = s_all[mine].to(DEV), t_all[mine].to(DEV)
        fs = torch.full((B * C,), 9.0, device=DEV)
        ft = torch.full((B * C,), 9.0, device=DEV)
        k.pair_owner_scatter(B * C, gp, int(off[r]), int(off[r + 1]), s_loc, t_loc, fs, ft)
        tot_s += fs
        tot_t += ft
        d = torch.empty(B * C, device=DEV)
        terms = torch.zeros(4, device=DEV)
        ws = torch.empty(k.llp_loss_ws_bytes(B, 0) // 4 + 16, device=DEV)
        k.llp_loss(B, C, s_all.to(DEV), t_all.to(DEV), 0, 0, None, B, 1, 0.05, 1.0, 1.0, 1.0, 1.0, d, None, terms, ws,
                   term_range=(r * B // W, (r + 1) * B // W))
        terms_sum += terms.cpu()
    assert torch.equal(tot_s.cpu(), s_all) and torch.equal(tot_t.cpu(), t_all)
    d1 = torch.empty(B * C, device=DEV)
    t1 = torch.zeros(4, device=DEV)
    ws = torch.empty(k.llp_loss_ws_bytes(B, 0) // 4 + 16, device=DEV)
    k.llp_loss(B, C, s_all.to(DEV), t_all.to(DEV), 0, 0, None, B, 1, 0.05, 1.0, 1.0, 1.0, 1.0, d1, None, t1, ws)
    assert torch.allclose(terms_sum, t1.cpu(), rtol=1e-5, atol=1e-7)
    assert torch.equal(d.cpu(), d1.cpu())    # every anchor's gradient, whatever the term range
