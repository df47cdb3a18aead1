"""Evaluation on MI355X: full-graph student embedding, edge scoring and
Hits@K / AUC on the device.

Reference: ``test_transductive`` (src/train_teacher_gnn.py:76-155) and
``test_production`` (src/train_teacher_gnn.py:157-268); metrics are ogb 1.3.6
``Evaluator`` hits@K and sklearn ``roc_auc_score``.  The result dictionaries
have the reference's keys and tuple layouts, so ``logger.py`` and the
printing code of ``main.py`` consume them unchanged.

Scores are computed by ``EdgeScorer``: the predictor's first GEMM reads
``h[e0] * h[e1]`` through a gathered operand (no materialised pair tensor),
hidden layers keep bias+ReLU in the epilogue, and the Linear(H,1)+sigmoid
head is one reduction kernel.  Chunks of ``chunk`` edges bound the scratch.
"""
from __future__ import annotations

import torch

import llp_hip as K

TRANSDUCTIVE_KS = (10, 20, 30, 50)          # src/train_teacher_gnn.py:118
COLLAB_KS = (10, 50, 100)                   # src/train_teacher_gnn.py:132


def _as_pairs(edges: torch.Tensor) -> torch.Tensor:
    """[E, 2] int32 contiguous on the device (the reference keeps [E, 2])."""
    if edges.dim() != 2 or edges.shape[1] != 2:
        raise ValueError("edges must be [E, 2]")
    return edges.to(torch.int32).contiguous()


class EdgeScorer:
    """predictor(h[e0], h[e1]) (src/models.py:139-150) in eval mode."""

    def __init__(self, predictor, dtype=torch.float32, chunk: int = 1 << 18):
        self.predictor = predictor
        self.dtype = dtype
        self.chunk = int(chunk)
        self.kind = predictor.predictor

    def _weights(self):
        lins = list(self.predictor.lins)
        hid = [(l.weight.detach().to(self.dtype).contiguous(), l.bias.detach().float().contiguous())
               for l in lins[:-1]]
        head = (lins[-1].weight.detach().float().reshape(-1).contiguous(), lins[-1].bias.detach().float().contiguous())
        return hid, head

    @torch.no_grad()
    def __call__(self, h: torch.Tensor, edges: torch.Tensor) -> torch.Tensor:
        if h.device.type != "cuda":
            raise RuntimeError("EdgeScorer runs only on a HIP device (no CPU fallback)")
        h = h.to(self.dtype).contiguous()
        pairs = _as_pairs(edges.to(h.device))
        E = pairs.shape[0]
        out = torch.empty(E, dtype=torch.float32, device=h.device)
        if E == 0:
            return out
        e0 = pairs[:, 0].contiguous()
        e1 = pairs[:, 1].contiguous()
        dc = K.dtype_code(self.dtype)
        if self.kind == "inner":
            K.head_fwd(h, E, h.shape[1], None, None, prob=out, Z2=h, iz=e0, iz2=e1)
            return out
        hid, (w2, b2) = self._weights()
        for s in range(0, E, self.chunk):
            n = min(self.chunk, E - s)
            i0, i1 = e0[s:s + n], e1[s:s + n]
            A = K.operand(h, i0, h, i1)
            z = None
            for W, b in hid:
                z = torch.empty(n, W.shape[0], dtype=self.dtype, device=h.device)
                K.gemm_nt(A, K.operand(W), n, W.shape[0], W.shape[1], z, dc, bias=b, act=K.ACT_RELU)
                A = K.operand(z)
            K.head_fwd(z, n, z.shape[1], w2, b2, prob=out[s:s + n])
        return out


@torch.no_grad()
def embed_mlp(model, x: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """model(x) for the student MLP in eval mode (no dropout, src/models.py:45-54; with
    norm_type 'layer' / 'batch' the norm runs in eval mode, BatchNorm on its running
    statistics)."""
    if x.device.type != "cuda":
        raise RuntimeError("embed_mlp runs only on a HIP device (no CPU fallback)")
    dc = K.dtype_code(dtype)
    A = K.operand(x.to(dtype).contiguous())
    layers = list(model.layers)
    norms = list(getattr(model, "norms", []))
    h = None
    M = x.shape[0]
    for l, lin in enumerate(layers):
        last = l == len(layers) - 1
        W = lin.weight.detach().to(dtype).contiguous()
        h = torch.empty(M, W.shape[0], dtype=dtype, device=x.device)
        normed = norms and not last
        K.gemm_nt(A, K.operand(W), M, W.shape[0], W.shape[1], h, dc, bias=lin.bias.detach().float(),
                  act=K.ACT_NONE if (last or normed) else K.ACT_RELU)
        if normed:
            nm = norms[l]
            batch = isinstance(nm, torch.nn.BatchNorm1d)
            stats = torch.empty(2, W.shape[0] if batch else M, dtype=torch.float32, device=x.device)
            K.norm_fwd(K.NORM_BATCH if batch else K.NORM_LAYER, h, h, stats,
                       None if nm.weight is None else nm.weight.detach(), None if nm.bias is None else nm.bias.detach(),
                       float(nm.eps), not batch, running_mean=getattr(nm, "running_mean", None),
                       running_var=getattr(nm, "running_var", None), relu=True)
        A = K.operand(h)
    return h


def hits_and_auc(pos: torch.Tensor, neg: torch.Tensor, Ks):
    return dict(zip(Ks, K.hits_at_k(pos, neg, Ks))), K.auc(pos, neg)


@torch.no_grad()
def test_transductive(h: torch.Tensor, predictor, split_edge, dataset: str, dtype=torch.float32):
    """src/train_teacher_gnn.py:76-155 given the node embeddings ``h``.
    Returns (results, h) with results['Hits@K'] = (valid, test), results['AUC']."""
    score = EdgeScorer(predictor, dtype)
    dev = h.device
    pv = score(h, split_edge["valid"]["edge"].to(dev))
    nv = score(h, split_edge["valid"]["edge_neg"].to(dev))
    pt = score(h, split_edge["test"]["edge"].to(dev))
    nt = score(h, split_edge["test"]["edge_neg"].to(dev))
    Ks = COLLAB_KS if dataset == "collab" else TRANSDUCTIVE_KS
    hv = K.hits_at_k(pv, nv, Ks)
    ht = K.hits_at_k(pt, nt, Ks)
    results = {f"Hits@{k}": (a, b) for k, a, b in zip(Ks, hv, ht)}
    results["AUC"] = (K.auc(pv, nv), K.auc(pt, nt))
    return results, h


@torch.no_grad()
def test_production(h_val: torch.Tensor, h_inf: torch.Tensor, predictor, val_pos, val_neg, test_edge_bundle,
                    negative_samples, dtype=torch.float32):
    """src/train_teacher_gnn.py:157-268 given the embeddings of val_data (h_val)
    and inference_data (h_inf).  test_edge_bundle = (old_old, old_new, new_new,
    test) as [2, E] tensors; negative_samples [E, 2].  Returns (results, h_val)
    with 5-tuples (val, test, old_old, old_new, new_new)."""
    score = EdgeScorer(predictor, dtype)
    dev = h_val.device
    pv = score(h_val, val_pos.to(dev))
    nv = score(h_val, val_neg.to(dev))
    oo, on, nn_, te = (t.t().to(dev) for t in test_edge_bundle)
    pt = score(h_inf, te)
    poo = score(h_inf, oo)
    pon = score(h_inf, on)
    pnn = score(h_inf, nn_)
    nt = score(h_inf, negative_samples.t().to(dev))   # negative_samples is [2, E] (src/train_teacher_gnn.py:168)
    Ks = TRANSDUCTIVE_KS
    cols = [K.hits_at_k(p, n, Ks) for p, n in ((pv, nv), (pt, nt), (poo, nt), (pon, nt), (pnn, nt))]
    results = {f"Hits@{k}": tuple(c[i] for c in cols) for i, k in enumerate(Ks)}
    results["AUC"] = tuple(K.auc(p, n) for p, n in ((pv, nv), (pt, nt), (poo, nt), (pon, nt), (pnn, nt)))
    return results, h_val
