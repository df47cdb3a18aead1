"""norm_type 'layer' / 'batch' (src/models.py:14,27-37,50-51,84-101,114-115) on the
GPU: the fused norm + ReLU + dropout kernels (csrc/norm.hip) against torch's
LayerNorm / BatchNorm1d in fp32, the module-level MLP against the reference's own
module (tests/golden/models_norm_fwd_bwd.npz), and the engines' norm paths
(unique-node student, bf16, hipGraph capture).  The golden replays of the engines
with norms are in test_gpu_engine / test_gpu_fullbatch / test_gpu_teacher /
test_gpu_multirank (the *_layernorm_* / *_batchnorm_* cases)."""
import types

import pytest
import torch
import torch.nn.functional as F

import golden_io as G

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_hip
    return llp_hip


def _ref(kind, y, gamma, beta, rm, rv, training=True, eps=1e-5):
    if kind == "layer":
        return F.relu(F.layer_norm(y, (y.shape[1],), gamma, beta, eps))
    return F.relu(F.batch_norm(y, rm, rv, gamma, beta, training, 0.1, eps))


@pytest.mark.parametrize("kind", ["layer", "batch"])
@pytest.mark.parametrize("shape", [(1000, 256), (77, 40), (3, 1030)])
def test_norm_kernels_match_torch_fp32(kind, shape):
    """Forward (output, running statistics) and backward (gy, dgamma, dbeta) of
    relu(norm(y)) with the ReLU mask taken from the output, against torch autograd in
    fp32; strided input / output (a [M, 2H] buffer's right half, as the SAGE teacher
    lays them out)."""
    K = _K()
    M, H = shape
    g = torch.Generator().manual_seed(M + H)
    big = torch.randn(M, 2 * H, generator=g).to(DEV) * 0.7 + 0.3
    y = big[:, H:]
    gamma = (1 + 0.3 * torch.randn(H, generator=g)).to(DEV)
    beta = (0.2 * torch.randn(H, generator=g)).to(DEV)
    rm0 = (0.1 * torch.randn(H, generator=g)).to(DEV)
    rv0 = (1 + 0.2 * torch.rand(H, generator=g)).to(DEV)
    gout = torch.randn(M, H, generator=g).to(DEV)
    kd = K.NORM_LAYER if kind == "layer" else K.NORM_BATCH
    # ours
    rm, rv, nbt = rm0.clone(), rv0.clone(), torch.zeros((), dtype=torch.int64, device=DEV)
    outbuf = torch.full((M, 2 * H), 7.0, device=DEV)
    out = outbuf[:, H:]
    stats = torch.empty(2, H if kind == "batch" else M, device=DEV)
    ws = torch.empty(K.norm_ws_bytes(M, H), dtype=torch.uint8, device=DEV)
    sums = torch.empty(2, H, dtype=torch.float64, device=DEV)
    if kind == "batch":
        K.norm_colsums(y, sums, ws)
    K.norm_fwd(kd, y, out, stats, gamma, beta, 1e-5, True, sums, float(M), 0.1, rm, rv, nbt)
    dg = torch.empty(H, device=DEV)
    db = torch.empty(H, device=DEV)
    bs = torch.empty(2, H, dtype=torch.float64, device=DEV)
    K.norm_bwd_sums(kd, gout, out, 1.0, y, stats, bs, ws, dgamma=dg, dbeta=db)
    gy = torch.empty(M, H, device=DEV)
    K.norm_bwd(kd, gout, out, 1.0, y, stats, gy, gamma, bs, float(M))
    torch.cuda.synchronize()
    assert torch.all(outbuf[:, :H] == 7.0)                 # the left half untouched
    # torch
    yt = y.detach().clone().requires_grad_()
    gt = gamma.clone().requires_grad_()
    bt = beta.clone().requires_grad_()
    rmt, rvt = rm0.clone(), rv0.clone()
    ref = _ref(kind, yt, gt, bt, rmt, rvt)
    ref.backward(gout)
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5), (out - ref).abs().max()
    assert torch.allclose(gy, yt.grad, rtol=1e-4, atol=1e-5), (gy - yt.grad).abs().max()
    assert torch.allclose(dg, gt.grad, rtol=1e-4, atol=1e-4), (dg - gt.grad).abs().max()
    assert torch.allclose(db, bt.grad, rtol=1e-4, atol=1e-4), (db - bt.grad).abs().max()
    if kind == "batch":
        assert torch.allclose(rm, rmt, rtol=1e-5, atol=1e-6) and torch.allclose(rv, rvt, rtol=1e-5, atol=1e-6)
        assert int(nbt.item()) == 1
        # eval mode: running statistics
        ev = torch.empty(M, H, device=DEV)
        K.norm_fwd(kd, y, ev, stats, gamma, beta, 1e-5, False, None, 0.0, 0.1, rm, rv, nbt)
        ref_e = _ref(kind, y, gamma, beta, rm.clone(), rv.clone(), training=False)
        assert torch.allclose(ev, ref_e, rtol=1e-5, atol=1e-5)
        assert int(nbt.item()) == 1


@pytest.mark.parametrize("kind", ["layer", "batch"])
def test_norm_kernels_bf16_and_deterministic(kind):
    """bf16 storage (f32 statistics) within bf16 rounding of the fp32 result; two calls
    are bit-identical (fixed-order column sums)."""
    K = _K()
    M, H = 4099, 512
    g = torch.Generator().manual_seed(5)
    y32 = torch.randn(M, H, generator=g).to(DEV)
    y = y32.to(torch.bfloat16)
    gamma = (1 + 0.3 * torch.randn(H, generator=g)).to(DEV)
    beta = (0.2 * torch.randn(H, generator=g)).to(DEV)
    gout = torch.randn(M, H, generator=g).to(DEV).to(torch.bfloat16)
    kd = K.NORM_LAYER if kind == "layer" else K.NORM_BATCH
    outs = []
    for _ in range(2):
        out = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
        stats = torch.empty(2, H if kind == "batch" else M, device=DEV)
        ws = torch.empty(K.norm_ws_bytes(M, H), dtype=torch.uint8, device=DEV)
        sums = torch.empty(2, H, dtype=torch.float64, device=DEV)
        K.norm_colsums(y, sums, ws)
        K.norm_fwd(kd, y, out, stats, gamma, beta, 1e-5, True, sums, float(M))
        bs = torch.empty(2, H, dtype=torch.float64, device=DEV)
        dg = torch.empty(H, device=DEV)
        K.norm_bwd_sums(kd, gout, out, 1.0, y, stats, bs, ws, dgamma=dg)
        gy = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
        K.norm_bwd(kd, gout, out, 1.0, y, stats, gy, gamma, bs, float(M))
        outs.append((out.clone(), gy.clone(), dg.clone()))
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    yt = y.float().requires_grad_()
    ref = _ref(kind, yt, gamma, beta, torch.zeros(H, device=DEV), torch.ones(H, device=DEV))
    ref.backward(gout.float())
    out, gy, dg = outs[0]
    assert (out.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert (gy.float() - yt.grad).abs().max().item() <= 3e-2 * yt.grad.abs().max().item()


def test_layernorm_device_row_count():
    """LayerNorm with a device row count (the unique-node student): rows past it are
    left alone and the column sums cover the live rows only."""
    K = _K()
    M, H, live = 300, 64, 211
    y = torch.randn(M, H, device=DEV)
    out = torch.full((M, H), 5.0, device=DEV)
    stats = torch.empty(2, M, device=DEV)
    cnt = torch.tensor([live], dtype=torch.int32, device=DEV)
    K.norm_fwd(K.NORM_LAYER, y, out, stats, None, None, 1e-5, True, rows=cnt)
    gout = torch.randn(M, H, device=DEV)
    bs = torch.empty(2, H, dtype=torch.float64, device=DEV)
    ws = torch.empty(K.norm_ws_bytes(M, H), dtype=torch.uint8, device=DEV)
    db = torch.empty(H, device=DEV)
    K.norm_bwd_sums(K.NORM_LAYER, gout, out, 1.0, y, stats, bs, ws, dbeta=db, rows=cnt)
    torch.cuda.synchronize()
    assert torch.all(out[live:] == 5.0)
    ref = F.relu(F.layer_norm(y[:live], (H,)))
    assert torch.allclose(out[:live], ref, atol=1e-5)
    assert torch.allclose(db, (gout[:live] * (ref > 0)).sum(0), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("kind", ["layer", "batch"])
def test_norm_mlp_module_matches_reference(kind):
    """models.MLP(norm_type=...) through the module-level autograd ops against the
    reference's own MLP (gen_golden.run_norm_model_case): train-mode forward and
    backward, BatchNorm running statistics, eval-mode forward."""
    _K()
    import models
    z = G.load("models_norm_fwd_bwd")
    pre = f"mlp_{kind}"
    m = models.MLP(3, 24, 40, 40, 0.0, kind).to(DEV)
    keys = [str(k) for k in z[f"{pre}/param_keys"]]
    with torch.no_grad():
        for (n, p), k in zip(m.named_parameters(), keys):
            assert n == k
            p.copy_(torch.from_numpy(z[f"{pre}/{k}"]))
    x = torch.from_numpy(z[f"{pre}/x"]).to(DEV).requires_grad_()
    y = m(x)
    assert torch.allclose(y.cpu(), torch.from_numpy(z[f"{pre}/y"]), atol=2e-5), (y.cpu() - torch.from_numpy(z[f"{pre}/y"])).abs().max()
    y.backward(torch.from_numpy(z[f"{pre}/gy"]).to(DEV))
    assert torch.allclose(x.grad.cpu(), torch.from_numpy(z[f"{pre}/gx"]), atol=2e-5)
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad.cpu(), torch.from_numpy(z[f"{pre}/grad/{n}"]), atol=2e-5, rtol=1e-4), n
    if kind == "batch":
        for i in range(2):
            for w in ("running_mean", "running_var"):
                got = getattr(m.norms[i], w).cpu()
                assert torch.allclose(got, torch.from_numpy(z[f"{pre}/norms.{i}.{w}"]), atol=1e-6), (i, w)
            assert int(m.norms[i].num_batches_tracked.item()) == 1
    m.eval()
    with torch.no_grad():
        ye = m(torch.from_numpy(z[f"{pre}/x_eval"]).to(DEV))
    assert torch.allclose(ye.cpu(), torch.from_numpy(z[f"{pre}/y_eval"]), atol=2e-5)


@pytest.mark.parametrize("conv_kind", ["sage", "updated"])
@pytest.mark.parametrize("kind", ["layer", "batch"])
def test_norm_sage_module_matches_oracle(conv_kind, kind):
    """models.SAGE(norm_type=...) forward / backward through the autograd ops against
    the oracle's restatement (conv, norm, ReLU between layers)."""
    _K()
    import llp_sage
    import models
    from oracle import llp_oracle as O
    torch.manual_seed(4)
    N, F_, H = 150, 24, 32
    ei = torch.randint(0, N, (2, 900))
    conv = llp_sage.SAGEConv_updated if conv_kind == "updated" else llp_sage.SAGEConv
    m = models.SAGE("cora", F_, H, H, 3, 0.0, conv, kind).to(DEV)
    with torch.no_grad():
        for nm in m.norms:
            nm.weight.uniform_(0.7, 1.3)
            nm.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, F_)
    xg = x.to(DEV).requires_grad_()
    h = m(xg, ei.to(DEV))
    gh = torch.randn_like(h)
    h.backward(gh)
    convs = [(c.lin_l.weight.detach().cpu().requires_grad_(), c.lin_l.bias.detach().cpu().requires_grad_(),
              c.lin_r.weight.detach().cpu().requires_grad_()) for c in m.convs]
    nps = [t.detach().cpu().requires_grad_() for nm in m.norms for t in (nm.weight, nm.bias)]
    bufs = [t for _ in m.norms for t in (torch.zeros(H), torch.ones(H), torch.tensor(0))]
    xo = x.clone().requires_grad_()
    ho = O.sage_forward(xo, ei, convs, 0.0, updated=conv_kind == "updated", norms=O.make_norms(kind, nps, bufs))
    ho.backward(gh.cpu())
    assert torch.allclose(h.detach().cpu(), ho.detach(), rtol=1e-4, atol=1e-5)
    assert torch.allclose(xg.grad.cpu(), xo.grad, rtol=1e-3, atol=1e-5)
    for nm, (w, b) in zip(m.norms, zip(nps[0::2], nps[1::2])):
        assert torch.allclose(nm.weight.grad.cpu(), w.grad, rtol=1e-3, atol=1e-5)
        assert torch.allclose(nm.bias.grad.cpu(), b.grad, rtol=1e-3, atol=1e-5)


def _problem(norm_type, dtype, dedup=True, N=3000, L=3):
    import llp_engine
    import models
    F_, H = 128, 256
    args = types.SimpleNamespace(rw_step=3, hops=3, ns_rate=3, ps_method="nb", dropout=0.0, margin=0.01,
                                 LLP_D=1.0, LLP_R=1.0, True_label=1.0, predictor="mlp", lr=0.001)
    g = torch.Generator().manual_seed(0)
    u = torch.randint(0, N, (20000,), generator=g)
    v = torch.randint(0, N, (20000,), generator=g)
    keep = u != v
    pairs = torch.stack([u[keep], v[keep]], 1)
    ei = torch.stack([pairs, pairs.flip(1)], 1).reshape(-1, 2).t()
    x = torch.randn(N, F_, generator=g) * 0.3
    t_h = torch.randn(N, 256, generator=g) * 0.3
    torch.manual_seed(3)
    model = models.MLP(L, F_, H, H, 0.0, norm_type).to(DEV)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(DEV)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(DEV)
    for p in tpred.parameters():
        p.requires_grad = False
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=args.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, x.to(DEV), t_h.to(DEV), ei[0].numpy(), ei[1].numpy(), N, args,
                                   opt, dtype=dtype, seed=5, dedup=dedup)
    anchors = torch.randperm(N, generator=torch.Generator().manual_seed(1))[:300].to(torch.int32).to(DEV)
    link = torch.randperm(pairs.size(0), generator=torch.Generator().manual_seed(2))[:2048].to(torch.int32).to(DEV)
    return eng, model, pred, anchors, link, pairs.to(torch.int32).to(DEV)


def _grads(model, pred):
    return [p.grad.detach().cpu().clone() for p in list(model.parameters()) + list(pred.parameters())]


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_layernorm_unique_node_student_matches_rowwise(dtype):
    """LayerNorm is row-wise, so the unique-node student (device row count through the
    norm kernels) gives the row-wise student's step."""
    _K()
    res = {}
    for dd in (True, False):
        eng, model, pred, a, l, pr = _problem("layer", dtype, dedup=dd)
        eng.step_minibatch(a, l, pr)
        torch.cuda.synchronize()
        res[dd] = (eng.terms.cpu().clone(), _grads(model, pred))
    (t1, g1), (t0, g0) = res[True], res[False]
    tol = 1e-5 if dtype == "fp32" else 2e-3
    assert torch.allclose(t1[:4], t0[:4], rtol=tol, atol=tol)
    for a, b in zip(g1, g0):
        if dtype == "fp32":
            assert (a - b).abs().max().item() <= 2e-4 * max(b.abs().max().item(), 1e-6) + 1e-7
        else:
            cos = F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
            assert cos > 0.99, cos


@pytest.mark.parametrize("norm_type", ["layer", "batch"])
def test_norm_engine_bf16_tracks_fp32(norm_type):
    """bf16 engine with norms against the fp32 engine on the same draws."""
    _K()
    res = {}
    for dt in ("fp32", "bf16"):
        eng, model, pred, a, l, pr = _problem(norm_type, dt)
        eng.step_minibatch(a, l, pr)
        torch.cuda.synchronize()
        res[dt] = (eng.terms.cpu().clone(), _grads(model, pred))
    (t32, g32), (t16, g16) = res["fp32"], res["bf16"]
    for i in range(4):
        assert abs(t16[i] - t32[i]) <= 2e-2 * max(abs(t32[i].item()), 1e-3), (i, t16[i].item(), t32[i].item())
    free = {1, 3} if norm_type == "batch" else set()     # Linear biases feeding a BatchNorm: zero gradient
    for i, (a, b) in enumerate(zip(g16, g32)):
        if i in free:
            assert a.abs().max().item() < 1e-3 * max(g.abs().max().item() for g in g32)
            continue
        cos = F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
        assert cos > 0.98, (i, tuple(a.shape), cos)


@pytest.mark.parametrize("norm_type", ["layer", "batch"])
def test_norm_engine_graph_replay_matches_eager(norm_type):
    """The minibatch step with norms captured in a hipGraph replays bit-identically
    to eager steps (BatchNorm's running statistics included)."""
    _K()
    out = {}
    for graph in (False, True):
        eng, model, pred, a, l, pr = _problem(norm_type, "bf16")
        eng.step_minibatch(a, l, pr)
        if graph:
            g = eng.capture_minibatch(a, l, pr)
            for _ in range(2):
                g.replay()
        else:
            for _ in range(2):
                eng.step_minibatch(a, l, pr)
        torch.cuda.synchronize()
        out[graph] = ([p.detach().cpu().clone() for p in list(model.parameters()) + list(pred.parameters())] +
                      [b.detach().cpu().clone() for b in model.buffers()])
    for x0, x1 in zip(out[False], out[True]):
        assert torch.equal(x0, x1)
