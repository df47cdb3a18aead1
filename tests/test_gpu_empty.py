"""Empty inputs through the C-ABI (the reference's torch ops accept them: an empty link
batch, a shard with no anchors, a graph whose nodes have no neighbours).  torch gives a
zero-element tensor a null data pointer, so every entry point must accept null buffers
when the sizes that address them are zero, and a reduction over zero rows writes the empty
sum (0) into its outputs, or leaves them as they are when accumulating -- what
torch.mm / sum / the ogb Hits formula give on the same empty inputs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_hip
    return llp_hip


def _e(*shape, dtype=torch.bfloat16):
    return torch.empty(*shape, device=DEV, dtype=dtype)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_gemm_nt_zero_rows(dt):
    K = _K()
    A, W, C = _e(0, 64, dtype=dt), torch.randn(256, 64, device=DEV).to(dt), _e(0, 256, dtype=dt)
    b = torch.randn(256, device=DEV)
    K.gemm_nt(K.operand(A), K.operand(W), 0, 256, 64, C, K.dtype_code(dt), bias=b, act=K.ACT_RELU)
    mask = _e(0, 32, dtype=torch.uint8)
    K.gemm_nt(K.operand(A), K.operand(W), 0, 256, 64, C, K.dtype_code(dt), bias=b, act=K.ACT_RELU, aux=mask)
    torch.cuda.synchronize()


def test_gemm_nt_head_zero_rows():
    K = _K()
    A, W = _e(0, 64), torch.randn(256, 64, device=DEV).to(torch.bfloat16)
    hw, b = torch.randn(256, device=DEV), torch.randn(256, device=DEV)
    parts = K.head_parts(256)
    hp = _e(parts, 0, dtype=torch.float32)
    K.gemm_nt_head(K.operand(A), K.operand(W), 0, 256, 64, None, hw, hp, bias=b)
    K.head_finish(parts, 0, hp, torch.zeros(1, device=DEV), logit=_e(0, dtype=torch.float32),
                  prob=_e(0, dtype=torch.float32))
    torch.cuda.synchronize()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_tn_zero_rows_is_the_empty_sum(dt, accumulate):
    """dW = A^T B over zero rows: 0 (torch.mm of [P,0] x [0,Q]), or C unchanged when
    accumulating; the fused bias gradient likewise."""
    K = _K()
    P, Q = 256, 128
    A, B = _e(0, P, dtype=dt), _e(0, Q, dtype=dt)
    Cw = torch.full((P, Q), 7.0, device=DEV)
    cs = torch.full((P,), 3.0, device=DEV)
    ws = torch.empty(max(K.gemm_tn_ws_bytes(K.dtype_code(dt), 0, P, Q), 16), dtype=torch.uint8, device=DEV)
    K.gemm_tn(K.operand(A), K.operand(B), 0, P, Q, Cw, K.dtype_code(dt), ws, accumulate=accumulate, colsum_a=cs)
    torch.cuda.synchronize()
    want = 7.0 if accumulate else 0.0
    assert bool((Cw == want).all())
    assert bool((cs == (3.0 if accumulate else 0.0)).all())
    assert torch.equal(torch.mm(A.float().t(), B.float()), torch.zeros(P, Q, device=DEV))


@pytest.mark.parametrize("accumulate", [False, True])
def test_colsum_and_head_bwd_zero_rows(accumulate):
    K = _K()
    H = 256
    out = torch.full((H,), 5.0, device=DEV)
    ws = torch.empty(max(K.colsum_ws_bytes(0, H), 16), dtype=torch.uint8, device=DEV)
    K.colsum(_e(0, H), 0, H, out, ws, accumulate=accumulate)
    dw, db = torch.full((H,), 5.0, device=DEV), torch.full((1,), 5.0, device=DEV)
    ws2 = torch.empty(max(K.head_bwd_ws_bytes(0, H), 16), dtype=torch.uint8, device=DEV)
    K.head_bwd(_e(0, dtype=torch.float32), _e(0, H), 0, H, torch.randn(H, device=DEV), True, _e(0, H), dw, db, ws2,
               accumulate=accumulate)
    torch.cuda.synchronize()
    want = 5.0 if accumulate else 0.0
    for t in (out, dw, db):
        assert bool((t == want).all())


def test_row_kernels_zero_rows():
    """Hadamard rows, gathers, activations, the head forward: nothing to do, no error."""
    K = _K()
    H = 256
    h = torch.randn(10, H, device=DEV).to(torch.bfloat16)
    i0 = _e(0, dtype=torch.int32)
    K.hadamard_rows(h, i0, h, i0, _e(0, H))
    K.gather_rows(h, i0, _e(0, H))
    K.gather_i32(i0, torch.arange(10, dtype=torch.int32, device=DEV), _e(0, dtype=torch.int32))
    K.act_2d(_e(0, H), _e(0, H))
    K.relu_bwd_2d(_e(0, H), _e(0, H), 1.0, _e(0, H))
    K.head_fwd(_e(0, H), 0, H, torch.randn(H, device=DEV), torch.zeros(1, device=DEV), logit=_e(0, dtype=torch.float32))
    torch.cuda.synchronize()


def test_norms_zero_rows():
    """LayerNorm over zero rows: nothing; BatchNorm's column sums over zero rows: 0."""
    K = _K()
    H = 64
    y, out = _e(0, H), _e(0, H)
    K.norm_fwd(K.NORM_LAYER, y, out, _e(2, 0, dtype=torch.float32), gamma=torch.ones(H, device=DEV),
               beta=torch.zeros(H, device=DEV))
    sums = torch.full((2, H), 9.0, device=DEV, dtype=torch.float64)
    ws = torch.empty(max(K.norm_ws_bytes(0, H), 16), dtype=torch.uint8, device=DEV)
    K.norm_colsums(y, sums, ws)
    torch.cuda.synchronize()
    assert bool((sums == 0).all())


def test_samplers_zero_draws():
    """No anchors / no label pairs in a shard."""
    K = _K()
    rowptr = torch.zeros(11, dtype=torch.int32, device=DEV)
    col = torch.zeros(1, dtype=torch.int32, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    K.context_sampler(rowptr, col, 10, _e(0, dtype=torch.int32), 0, "nb", 3, 3, 3, 1, ctr, 0,
                      _e(0, 37, dtype=torch.int32))
    K.randint_pairs(10, 0, 1, ctr, 0, _e(2, 0, dtype=torch.int32))
    K.pair_index_from_samples(0, 36, _e(0, 37, dtype=torch.int32), _e(0, dtype=torch.int32), _e(0, dtype=torch.int32))
    torch.cuda.synchronize()


def test_dedup_zero_rows():
    K = _K()
    N = 50
    uniq, pos = _e(0, dtype=torch.int32), _e(0, dtype=torch.int32)
    n_unique = torch.full((1,), 7, dtype=torch.int32, device=DEV)
    seg_ptr = torch.full((N + 1,), 7, dtype=torch.int32, device=DEV)
    seg_rows = _e(0, dtype=torch.int32)
    ws = torch.empty(max(K.dedup_ws_bytes(N, 0), 16), dtype=torch.uint8, device=DEV)
    K.dedup_rows(N, 0, _e(0, dtype=torch.int32), uniq, pos, n_unique, seg_ptr, seg_rows, ws)
    torch.cuda.synchronize()
    assert int(n_unique.item()) == 0 and int(seg_ptr[0].item()) == 0


def test_hits_with_no_negatives_is_one():
    """ogb's Hits@K: fewer negatives than K scores 1.0 (len(y_pred_neg) < K)."""
    K = _K()
    pos = torch.rand(20, device=DEV)
    assert K.hits_at_k(pos, _e(0, dtype=torch.float32), [1, 20, 50]) == [1.0, 1.0, 1.0]
    neg = torch.rand(5, device=DEV)
    assert K.hits_at_k(pos, neg, [10])[0] == 1.0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_aggregate_isolated_nodes_and_zero_rows(dt):
    """PyG mean aggregation: a node with no in-edges aggregates to 0 (Q2); zero rows: nothing."""
    K = _K()
    N, F = 6, 64
    # edges 0->1, 2->1, 3->4 (CSR by destination); nodes 0, 2, 3, 5 have none
    rowptr = torch.tensor([0, 0, 2, 2, 2, 3, 3], dtype=torch.int32, device=DEV)
    col = torch.tensor([0, 2, 3], dtype=torch.int32, device=DEV)
    x = torch.randn(N, F, device=DEV).to(dt)
    deg = (rowptr[1:] - rowptr[:-1]).float()
    inv = torch.where(deg > 0, 1.0 / deg.clamp(min=1), torch.zeros_like(deg))
    out = torch.full((N, F), 9.0, device=DEV).to(dt)
    K.csr_aggregate(N, F, rowptr, col, x, inv, 0, out)
    torch.cuda.synchronize()
    xf = x.float()
    ref = torch.zeros(N, F, device=DEV)
    ref[1] = (xf[0] + xf[2]) / 2
    ref[4] = xf[3]
    tol = 1e-6 if dt == torch.float32 else 1e-2
    assert torch.allclose(out.float(), ref, atol=tol, rtol=tol)
    K.csr_aggregate(0, F, rowptr[:1], col, x, inv[:0], 0, _e(0, F, dtype=dt))
    torch.cuda.synchronize()
