"""Evaluation path on the GPU (src/train_teacher_gnn.py:76-268): Hits@K equal to
the ogb formula (exact, ties and short negative lists included), AUC equal to
sklearn's, edge scores / embeddings within fp32 tolerance of the oracle."""
import numpy as np
import pytest
import torch

from oracle import llp_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_eval
    import llp_hip
    import models
    return llp_hip, llp_eval, models


@pytest.mark.parametrize("n_pos,n_neg,ties", [(1000, 5000, False), (3000, 100000, True), (50, 30, False),
                                              (7, 1, True), (2000, 2000, True)])
def test_hits_and_auc_exact(n_pos, n_neg, ties):
    K, _, _ = _mods()
    g = torch.Generator().manual_seed(n_pos + n_neg)
    pos = torch.rand(n_pos, generator=g) * 0.8 + 0.2
    neg = torch.rand(n_neg, generator=g)
    if ties:   # sigmoid outputs collide often in practice; quantise to force ties
        pos = (pos * 64).floor() / 64
        neg = (neg * 64).floor() / 64
    Ks = [1, 10, 20, 30, 50, 100]
    got = K.hits_at_k(pos.to(DEV), neg.to(DEV), Ks)
    for k, v in zip(Ks, got):
        assert v == O.hits_at_k(pos, neg, k), (k, v, O.hits_at_k(pos, neg, k))
    a = K.auc(pos.to(DEV), neg.to(DEV))
    assert abs(a - O.auc(pos, neg)) < 1e-12, (a, O.auc(pos, neg))


@pytest.mark.parametrize("kind", ["mlp", "inner"])
def test_embed_and_score_match_oracle(kind):
    K, E, models = _mods()
    torch.manual_seed(0)
    N, F_, H, L = 700, 96, 128, 3
    mlp = models.MLP(L, F_, H, H, 0.3).to(DEV).eval()
    pred = models.LinkPredictor(kind, H, H, 1, L, 0.3).to(DEV).eval()
    x = torch.randn(N, F_)
    h = E.embed_mlp(mlp, x.to(DEV))
    hw = [l.weight.detach().cpu() for l in mlp.layers]
    hb = [l.bias.detach().cpu() for l in mlp.layers]
    href = O.mlp_forward(x, hw, hb, 0.3, training=False)
    assert torch.allclose(h.cpu(), href, atol=1e-4, rtol=1e-4)
    edges = torch.randint(0, N, (5000, 2))
    s = E.EdgeScorer(pred, chunk=1536)(h, edges.to(DEV))
    pw = [l.weight.detach().cpu() for l in pred.lins]
    pb = [l.bias.detach().cpu() for l in pred.lins]
    sref = O.link_predictor_forward(href[edges[:, 0]], href[edges[:, 1]], pw, pb, kind, 0.3,
                                    training=False).squeeze(-1)
    assert torch.allclose(s.cpu(), sref, atol=1e-5, rtol=1e-4), (s.cpu() - sref).abs().max()


def test_test_transductive_layout():
    K, E, models = _mods()
    torch.manual_seed(1)
    N, H = 400, 64
    pred = models.LinkPredictor("mlp", H, H, 1, 2, 0.0).to(DEV).eval()
    h = torch.randn(N, H, device=DEV)
    split = {s: {"edge": torch.randint(0, N, (300, 2)), "edge_neg": torch.randint(0, N, (900, 2))}
             for s in ("valid", "test")}
    for ds, Ks in (("cora", (10, 20, 30, 50)), ("collab", (10, 50, 100))):
        res, h2 = E.test_transductive(h, pred, split, ds)
        assert h2 is h
        assert set(res) == {f"Hits@{k}" for k in Ks} | {"AUC"}
        sc = E.EdgeScorer(pred)
        for i, s in enumerate(("valid", "test")):
            p = sc(h, split[s]["edge"].to(DEV)).cpu()
            n = sc(h, split[s]["edge_neg"].to(DEV)).cpu()
            for k in Ks:
                assert res[f"Hits@{k}"][i] == O.hits_at_k(p, n, k)
            assert abs(res["AUC"][i] - O.auc(p, n)) < 1e-12
