"""Full BASELINE size (ogbl-collab LLP, configs[2]: N=235,868, F=128,
E=2,358,104, H=1024, L=3, B=13,110 anchors x C=36 contexts, P=65,536 edges,
bf16): size-independent properties of one distillation step, since the CPU
oracle cannot run this size in a test.

* determinism: the same step from the same state gives bit-identical loss
  terms and gradients (fixed-order reductions everywhere, no atomics);
* the unique-node student (dropout-free MLP on the distinct nodes of
  x[this_target]) gives the row-wise student's loss terms bit for bit and its
  gradients to bf16 summation-order accuracy;
* the loss terms are finite and the step moves every parameter."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def collab():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, REPO)
    import llp_data
    from bench import collab_args
    return llp_data.synthetic_collab(seed=0, with_eval=False), collab_args()


def _one_step(collab, dedup):
    import llp_engine
    import models
    data, a = collab
    N, F_, H, L = data.N, data.F, a.hidden_channels, a.num_layers
    torch.manual_seed(1)
    model = models.MLP(L, F_, H, H, 0.0).to(DEV)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(DEV)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(DEV)
    for p in tpred.parameters():
        p.requires_grad = False
    t_h = torch.randn(N, 256, generator=torch.Generator().manual_seed(2)) * 0.3
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(DEV), t_h.to(DEV), data.edge_index[0].numpy(),
                                   data.edge_index[1].numpy(), N, a, opt, dtype="bf16", seed=123, dedup=dedup)
    E = data.train_pairs.shape[0]
    P = a.link_batch_size
    B = int(N / (E / P))
    g = torch.Generator().manual_seed(3)
    anchors = torch.randperm(N, generator=g)[:B].to(torch.int32).to(DEV)
    links = torch.randperm(E, generator=g)[:P].to(torch.int32).to(DEV)
    pairs = data.train_pairs.to(torch.int32).to(DEV).contiguous()
    params0 = [p.detach().clone() for p in list(model.parameters()) + list(pred.parameters())]
    eng.step_minibatch(anchors, links, pairs, B_total=B, P_total=P)
    torch.cuda.synchronize()
    out = {"terms": eng.terms.cpu().clone(), "rows": eng.last_student_rows, "B": B,
           "grads": [p.grad.detach().float().cpu().clone() for p in list(model.parameters()) + list(pred.parameters())],
           "moved": [bool((p.detach() != p0).any()) for p, p0 in zip(list(model.parameters()) + list(pred.parameters()),
                                                                      params0)]}
    del eng, model, pred, tpred, opt
    torch.cuda.empty_cache()
    return out


def test_fullsize_step_properties(collab):
    a1 = _one_step(collab, dedup=True)
    a2 = _one_step(collab, dedup=True)
    rw = _one_step(collab, dedup=False)
    data, a = collab
    C = a.rw_step * a.hops * (1 + a.ns_rate)
    assert a1["B"] == 13110 and C == 36
    assert torch.isfinite(a1["terms"]).all()
    assert all(a1["moved"])
    # determinism
    assert torch.equal(a1["terms"], a2["terms"])
    for x, y in zip(a1["grads"], a2["grads"]):
        assert torch.equal(x, y)
    # unique-node student == row-wise student
    assert a1["rows"] < rw["rows"] == 13110 * (C + 1) + 4 * a.link_batch_size
    assert torch.equal(a1["terms"][:4], rw["terms"][:4])
    for x, y in zip(a1["grads"], rw["grads"]):
        rel = float((x - y).norm() / (y.norm() + 1e-30))
        assert rel < 2e-2, rel
