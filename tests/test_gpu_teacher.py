"""GraphSAGE teacher on the GPU: TeacherEngine replays
the reference's own teacher train() (tests/golden/gen_golden.py, recorded
permutations and negatives injected) — BCE within 1e-4, gradients, epoch
losses, final weights and the eval embedding; plus the module-level SAGE
(autograd ops) against the oracle."""
import pytest
import torch

import golden_io as G
from oracle import llp_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _build(c, dtype="fp32", dropout=0.0):
    import llp_sage
    import llp_teacher
    import models
    if c.encoder == "gcn":
        model = models.GCN(c.F, c.H, c.H, c.L, dropout).to(DEV)
    else:
        conv = llp_sage.SAGEConv_updated if c.updated else llp_sage.SAGEConv
        model = models.SAGE(c.dataset, c.F, c.H, c.H, c.L, dropout, conv, c.norm_type).to(DEV)
    pred = models.LinkPredictor("mlp", c.H, c.H, 1, 2, dropout).to(DEV)
    G.set_state(model, c.enc0, c.enc_buf0)
    with torch.no_grad():
        for p, v in zip(pred.parameters(), c.pred0):
            p.copy_(v)
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=0.005)
    eng = llp_teacher.TeacherEngine(model, pred, c.x.to(DEV), c.edge_index, c.N, opt, dtype=dtype, seed=3)
    return eng, model, pred


@pytest.mark.parametrize("name", G.TEACHER_CASES)
def test_teacher_engine_replays_reference(name):
    _need_gpu()
    c = G.load_teacher_case(name)
    eng, model, pred = _build(c)
    pairs = c.pos_train_edge.to(torch.int32).to(DEV).contiguous()
    params = list(model.parameters()) + list(pred.parameters())
    steps_per_epoch = len(c.steps) // len(c.epoch_losses)
    tot = 0
    eng.begin_epoch()
    for i, st in enumerate(c.steps):
        n_neg = eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, neg=st.neg_edge.to(DEV))
        assert n_neg == st.neg_edge.shape[1]
        torch.cuda.synchronize()
        bce = eng.terms[1].item()
        assert abs(bce - st.bce) <= 1e-4 * max(1.0, abs(st.bce)), (name, i, bce, st.bce)
        rtol = 2e-4 if i == 0 else 2e-3
        for p, ref in zip(params, st.grads):
            err = (p.grad.detach().cpu() - ref).abs().max().item()
            assert err <= rtol * max(ref.abs().max().item(), 1e-6) + 1e-7, (name, i, tuple(p.shape), err)
        tot += st.edge.size(1)
        if (i + 1) % steps_per_epoch == 0:
            ep = eng.end_epoch(tot)
            assert abs(ep - c.epoch_losses[(i + 1) // steps_per_epoch - 1]) < 1e-4, ep
            tot = 0
            eng.begin_epoch()
    free = G.free_params(c, per_layer=3)
    for i, (p, ref) in enumerate(zip(params, c.enc_final + c.pred_final)):
        d = (p.detach().cpu() - ref).abs()
        if i not in free:
            assert (d <= 1e-4).float().mean().item() > 0.99, (name, tuple(p.shape), d.max().item())
        assert d.max().item() <= 2 * 0.005 * len(c.steps), (name, tuple(p.shape), d.max().item())
    if c.norm_type == "batch":
        shift = 0.1 * 2 * 0.005 * len(c.steps)
        for b, ref, nm in zip(model.buffers(), c.enc_buf_final, c.enc_buffer_names):
            tol = 1e-5 + (shift if nm.endswith("running_mean") else 0.0)
            assert (b.detach().cpu().to(ref.dtype) - ref).abs().max().item() <= tol + 1e-4 * ref.abs().max().item(), \
                (name, nm)
        # the eval embedding on the reference's final state (the free biases' drift stays out)
        G.set_state(model, c.enc_final, c.enc_buf_final)
        eng.refresh_weights()
    h = eng.embed().cpu()
    assert torch.allclose(h, c.h_eval, rtol=1e-3, atol=1e-3 * c.h_eval.abs().max().item()), \
        (h - c.h_eval).abs().max()


@pytest.mark.parametrize("name", ["teacher_sage_small", "teacher_updated_production_small", "teacher_gcn_small"])
def test_teacher_engine_bf16_and_dropout_run(name):
    """bf16 engine tracks fp32 on the first step; dropout + device negatives run."""
    _need_gpu()
    c = G.load_teacher_case(name)
    pairs = c.pos_train_edge.to(torch.int32).to(DEV).contiguous()
    st = c.steps[0]
    res = {}
    for dt in ("fp32", "bf16"):
        eng, model, pred = _build(c, dt)
        eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, neg=st.neg_edge.to(DEV))
        torch.cuda.synchronize()
        res[dt] = (eng.terms[1].item(), [p.grad.detach().cpu().clone() for p in
                                         list(model.parameters()) + list(pred.parameters())])
    assert abs(res["bf16"][0] - res["fp32"][0]) < 2e-2
    for a, b in zip(res["bf16"][1], res["fp32"][1]):
        assert torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item() > 0.97
    eng, model, pred = _build(c, "bf16", dropout=0.5)
    for _ in range(3):
        eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, dense_negatives=(c.dataset != "collab"))
    torch.cuda.synchronize()
    assert torch.isfinite(eng.terms).all()
    for p in model.parameters():
        assert torch.isfinite(p).all()


@pytest.mark.parametrize("updated", [False, True])
def test_sage_module_forward_backward(updated):
    """models.SAGE through the autograd ops (eval / API surface) vs the oracle."""
    _need_gpu()
    import llp_sage
    import models
    torch.manual_seed(0)
    N, F_, H = 150, 40, 64
    ei = torch.randint(0, N, (2, 700))
    conv = llp_sage.SAGEConv_updated if updated else llp_sage.SAGEConv
    model = models.SAGE("cora", F_, H, H, 3, 0.0, conv).to(DEV)
    x = torch.randn(N, F_)
    xd = x.to(DEV).requires_grad_()
    h = model(xd, ei.to(DEV))
    gh = torch.randn_like(h)
    h.backward(gh)
    convs = [(c.lin_l.weight.detach().cpu().requires_grad_(), c.lin_l.bias.detach().cpu().requires_grad_(),
              c.lin_r.weight.detach().cpu().requires_grad_()) for c in model.convs]
    xr = x.clone().requires_grad_()
    href = O.sage_forward(xr, ei, convs, 0.0, updated=updated)
    href.backward(gh.cpu())
    assert torch.allclose(h.detach().cpu(), href.detach(), rtol=1e-4, atol=1e-4)
    assert torch.allclose(xd.grad.cpu(), xr.grad, rtol=1e-3, atol=1e-4)
    for c, (wl, bl, wr) in zip(model.convs, convs):
        assert torch.allclose(c.lin_l.weight.grad.cpu(), wl.grad, rtol=1e-3, atol=1e-4)
        assert torch.allclose(c.lin_r.weight.grad.cpu(), wr.grad, rtol=1e-3, atol=1e-4)


def test_gcn_module_forward_backward():
    """models.GCN through the autograd ops (GCNConv: lin, normalised propagation
    with self-loops, bias) vs the oracle, on a directed graph with self-loops."""
    _need_gpu()
    import models
    torch.manual_seed(1)
    N, F_, H = 160, 48, 64
    ei = torch.randint(0, N, (2, 800))
    ei[:, :10] = torch.arange(10).repeat(2, 1)          # input self-loops (dropped by gcn_norm)
    model = models.GCN(F_, H, H, 3, 0.0).to(DEV)
    with torch.no_grad():
        for c in model.convs:
            c.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, F_)
    xd = x.to(DEV).requires_grad_()
    h = model(xd, ei.to(DEV))
    gh = torch.randn_like(h)
    h.backward(gh)
    convs = [(c.lin.weight.detach().cpu().requires_grad_(), c.bias.detach().cpu().requires_grad_())
             for c in model.convs]
    xr = x.clone().requires_grad_()
    href = O.gcn_forward(xr, ei, convs, 0.0)
    href.backward(gh.cpu())
    assert torch.allclose(h.detach().cpu(), href.detach(), rtol=1e-4, atol=1e-4)
    assert torch.allclose(xd.grad.cpu(), xr.grad, rtol=1e-3, atol=1e-4)
    for c, (w, b) in zip(model.convs, convs):
        assert torch.allclose(c.lin.weight.grad.cpu(), w.grad, rtol=1e-3, atol=1e-4)
        assert torch.allclose(c.bias.grad.cpu(), b.grad, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_teacher_step_is_deterministic(dtype):
    """Two runs of the same teacher steps give bit-identical gradients and
    weights: the predictor-input backward is a fixed-order per-node sum
    (no float atomics), the TN splits reduce in a fixed order."""
    _need_gpu()
    c = G.load_teacher_case(G.TEACHER_CASES[0])
    pairs = c.pos_train_edge.to(torch.int32).to(DEV).contiguous()
    runs = []
    for _ in range(2):
        eng, model, pred = _build(c, dtype=dtype)
        for st in c.steps[:3]:
            eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, neg=st.neg_edge.to(DEV))
        torch.cuda.synchronize()
        ps = list(model.parameters()) + list(pred.parameters())
        runs.append([p.detach().cpu().clone() for p in ps] + [p.grad.detach().cpu().clone() for p in ps])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_teacher_bf16_relu_bit_masks_match_activation_masks():
    """bf16 SAGE teacher with dropout: the ReLU/dropout bit masks written by the
    forward GEMMs give bit-identical gradients and weights to the data-gradient
    GEMMs masking on the stored bf16 activations."""
    _need_gpu()
    c = G.load_teacher_case("teacher_sage3_collab_small")   # H = 32, 3 layers: layer 2 takes a mask
    pairs = c.pos_train_edge.to(torch.int32).to(DEV).contiguous()
    runs = []
    for use_mask in (True, False):
        eng, model, pred = _build(c, dtype="bf16", dropout=0.5)
        if not use_mask:
            for L in eng.layers:
                L.pop("M", None)
        else:
            assert "M" in eng.layers[2]
        for st in c.steps[:3]:
            eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, neg=st.neg_edge.to(DEV))
        torch.cuda.synchronize()
        ps = list(model.parameters()) + list(pred.parameters())
        runs.append([p.detach().cpu().clone() for p in ps])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["teacher_sage_small", "teacher_gcn_small", "teacher_updated_production_small"])
def test_teacher_locality_order_same_results(name):
    """TeacherEngine(reorder=True), the default: nodes renumbered by llp_sage.locality_order inside
    the engine (edges relabelled in their order, pairs and negatives mapped).  Against
    reorder=False on the same steps: the eval embedding (returned in the original node order) and
    the BCE are identical -- every row's neighbour sum runs in the same order -- and the
    gradients agree up to the order of the weight-gradient sums over the (renumbered) nodes."""
    _need_gpu()
    import llp_sage
    import llp_teacher
    import models
    c = G.load_teacher_case(name)
    pairs = c.pos_train_edge.to(torch.int32).to(DEV).contiguous()
    res = {}
    for reorder in (False, True):
        eng, model, pred = _build(c)
        if not reorder:   # rebuild without the order (same modules and weights)
            opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=0.005)
            eng = llp_teacher.TeacherEngine(model, pred, c.x.to(DEV), c.edge_index, c.N, opt, dtype="fp32", seed=3,
                                            reorder=False)
        else:
            assert eng._pi is not None
        h0 = eng.embed().cpu()
        st = c.steps[0]
        eng.step(st.link_perm.to(torch.int32).to(DEV), pairs, neg=st.neg_edge.to(DEV))
        torch.cuda.synchronize()
        res[reorder] = (h0, eng.terms[1].item(), [p.grad.detach().cpu().clone() for p in
                                                   list(model.parameters()) + list(pred.parameters())])
    assert torch.equal(res[True][0], res[False][0])
    assert abs(res[True][1] - res[False][1]) <= 1e-6 * max(1.0, abs(res[False][1]))
    for a, b in zip(res[True][2], res[False][2]):
        assert (a - b).abs().max().item() <= 1e-4 * max(b.abs().max().item(), 1e-6) + 1e-7

