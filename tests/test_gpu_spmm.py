"""Sparse-input first layer (csrc/spmm.hip: llp_spmm_rows / llp_spmm_tn) against a numpy
restatement of nn.Linear on the sparse x (src/models.py:48) that sums in the kernels' order
(interleaved streams, butterfly): bit for bit, ReLU bit masks included.  Binary values (bag-of-words) and small-integer
values (every fma exact in f64, rounded once to f32 as fmaf does)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def K():
    import llp_hip
    return llp_hip


def _bf16_round(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16)


def _x(N, F, dens, values, seed):
    rng = np.random.default_rng(seed)
    x = (rng.random((N, F)) < dens).astype(np.float32)
    x[N // 3] = 0                                # an empty row
    if values:
        x *= rng.choice(np.array([0.5, 2.0, 3.0], np.float32), size=(N, F))
    return x


def _fma_seq(acc, v, w):
    """acc (f32) <- fmaf(v, w, acc), elementwise: exact in f64 for these operands, one rounding."""
    return (acc.astype(np.float64) + np.float64(v) * w.astype(np.float64)).astype(np.float32)


def _streams(idx, vals, rows_of, streams):
    """The kernels' sum over one index list: stream s takes positions s, s + streams, .. (fmaf
    in order), then the butterfly ((s0+s1)+(s2+s3)) .. in f32."""
    parts = []
    for s in range(streams):
        acc = np.zeros(rows_of.shape[1], np.float32)
        for j in range(s, len(idx), streams):
            acc = _fma_seq(acc, vals[j], rows_of[idx[j]])
        parts.append(acc)
    while len(parts) > 1:
        parts = [(parts[i] + parts[i + 1]).astype(np.float32) for i in range(0, len(parts), 2)]
    return parts[0]


@pytest.mark.parametrize("H", [256, 64, 520, 136])
@pytest.mark.parametrize("values", [False, True])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_spmm_rows_bit_exact(H, values, relu, dtype):
    k = K()
    N, F = 203, 700
    x = _x(N, F, 0.02, values, H + values)
    g = torch.Generator().manual_seed(5)
    Wt = (torch.randn(F, H, generator=g) * 0.2).to(dtype)
    bias = torch.randn(H, generator=g) * 0.1
    xs = k.SparseRows(torch.from_numpy(x).to(DEV), round_bf16=dtype == torch.bfloat16)
    assert (xs.val is None) == (not values)
    r0, rows = 17, 150
    Y = torch.full((rows + 3, H), 7.0, dtype=dtype, device=DEV)
    bf = dtype == torch.bfloat16
    mask = torch.full((rows, H // 8), 0xAB, dtype=torch.uint8, device=DEV) if bf and relu and H % 8 == 0 else None
    Wt_d = Wt.to(DEV)
    k.spmm_rows(xs, rows, r0, Wt_d, bias.to(DEV), Y, act=k.ACT_RELU if relu else k.ACT_NONE, mask=mask)
    torch.cuda.synchronize()
    Wf = Wt.float().numpy()
    ref = np.zeros((rows, H), np.float32)
    for r in range(rows):
        cols = np.nonzero(x[r0 + r])[0]
        ref[r] = _streams(cols, x[r0 + r, cols], Wf, 4) + bias.numpy()
    got = Y[:rows].cpu()
    if not bf:   # f32 rows: the same sums, no rounding to bf16; ReLU keeps the f32 value
        if relu:
            ref = np.where(ref < 0, np.float32(0), ref)
        assert np.array_equal(got.numpy(), ref)
        assert torch.equal(Y[rows:].cpu(), torch.full((3, H), 7.0))
        return
    refb = _bf16_round(ref)
    if relu:
        refb = torch.where(refb.view(torch.int16) < 0, torch.zeros_like(refb), refb)
    assert torch.equal(got.view(torch.int16), refb.view(torch.int16))
    assert torch.equal(Y[rows:].cpu().float(), torch.full((3, H), 7.0))     # rows past `rows` untouched
    if mask is not None:
        nz = (refb.view(torch.int16) != 0).numpy().reshape(rows, H // 8, 8)
        ref_mask = (nz * (1 << np.arange(8))).sum(-1).astype(np.uint8)
        assert np.array_equal(mask.cpu().numpy(), ref_mask)


@pytest.mark.parametrize("H", [256, 128, 1024, 136])
@pytest.mark.parametrize("values", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_spmm_tn_bit_exact(H, values, dtype):
    k = K()
    N, F = 240, 333
    x = _x(N, F, 0.03, values, 7 * H + values)
    x[:, 5:40:3] = (np.random.default_rng(H).random((N, 12)) < 0.9) * (2.0 if values else 1.0)   # heavy columns
    g = torch.Generator().manual_seed(11)
    xs = k.SparseRows(torch.from_numpy(x).to(DEV), round_bf16=dtype == torch.bfloat16)
    r0, n = 30, 180
    dY = (torch.randn(n, H, generator=g) * 0.3).to(dtype)
    dW = torch.full((H, F + 5), 3.0, device=DEV)[:, :F]     # row stride F + 5
    for accumulate in (False, True):
        k.spmm_tn(xs, r0, n, dY.to(DEV), dW, accumulate=accumulate)
    torch.cuda.synchronize()
    dYf = dY.float().numpy()
    ref = np.zeros((F, H), np.float32)
    heavy = k.load().llp_spmm_heavy_nnz()
    n_heavy = 0
    for f in range(F):
        rws = np.nonzero(x[r0:r0 + n, f])[0]                   # ascending rows of the slice
        if len(rws) >= heavy:                                    # four contiguous quarters
            n_heavy += 1
            q = [len(rws) * w // 4 for w in range(5)]
            w = [_streams(rws[q[i]:q[i + 1]], x[r0 + rws[q[i]:q[i + 1]], f], dYf, 8) for i in range(4)]
            ref[f] = ((w[0] + w[1]).astype(np.float32) + (w[2] + w[3]).astype(np.float32)).astype(np.float32)
        else:
            ref[f] = _streams(rws, x[r0 + rws, f], dYf, 8)
    assert xs.csc(r0, n)[4] == n_heavy and 0 < n_heavy < F      # both schedules exercised
    got = dW.cpu().numpy()
    assert np.array_equal(got, (ref.T + ref.T).astype(np.float32))   # second call accumulated once more


def test_spmm_csc_slices():
    """SparseRows.csc: per-slice column lists (local rows, ascending) reproduce the slice."""
    k = K()
    x = _x(97, 50, 0.1, True, 3)
    xs = k.SparseRows(torch.from_numpy(x).to(DEV))
    for r0, n in [(0, 97), (10, 40), (96, 1)]:
        colptr, rowidx, val, perm, n_heavy = xs.csc(r0, n)
        cnt = np.diff(colptr.cpu().numpy())
        assert np.array_equal(perm.cpu().numpy(), np.argsort(-cnt, kind="stable"))
        dense = np.zeros((n, 50), np.float32)
        cp, ri, vv = colptr.cpu().numpy(), rowidx.cpu().numpy(), val.cpu().numpy()
        for f in range(50):
            rows = ri[cp[f]:cp[f + 1]]
            assert np.all(np.diff(rows) > 0)
            dense[rows, f] = vv[cp[f]:cp[f + 1]]
        assert np.array_equal(dense, x[r0:r0 + n])


def test_spmm_rejects_bad_shapes():
    k = K()
    xs = k.SparseRows(torch.from_numpy(_x(8, 300, 0.05, False, 1)).to(DEV))
    Wt = torch.zeros(300, 12, dtype=torch.bfloat16, device=DEV)        # H % 8 != 0
    with pytest.raises(RuntimeError):
        k.spmm_rows(xs, 8, 0, Wt, None, torch.zeros(8, 12, dtype=torch.bfloat16, device=DEV))
    Wt = torch.zeros(300, 20, dtype=torch.bfloat16, device=DEV)[:, :16]   # rows not 16-B aligned
    with pytest.raises(RuntimeError):
        k.spmm_rows(xs, 8, 0, Wt, None, torch.zeros(8, 16, dtype=torch.bfloat16, device=DEV))
