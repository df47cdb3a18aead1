"""BASELINE configs[1]: citeseer transductive LLP distillation, fp32 parity vs
the CPU restatement at the dataset's shape (N=3,327, F=3,703, H=256, L=2, the
citeseer script's LLP_D=0.001 / LLP_R=1000 / True_label=0.001, hops=1,
ns_rate=4, rw_step=3 -> C=15; scripts/LLP_transductive.sh:2).  One full-batch
``train`` step (src/main.py:147-236) on the fp32 engine against the oracle on
the same inputs: contexts from the oracle's Philox sampler (the device
sampler's streams), negatives injected.  Dropout is 0 here: the reference's
dropout streams are torch-version and device dependent and the
dropout kernel is checked on its own.  Bar: loss terms within 1e-4 relative,
logits' gradients within rtol 1e-3 of the largest element (f32, K up to 3,703
in a different summation order)."""
import types

import numpy as np
import pytest
import torch

from oracle import llp_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_citeseer_fullbatch_step_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_datasets
    import llp_engine
    import models
    data, split_edge = llp_datasets.synthetic_transductive("citeseer")
    N, F_ = data.x.shape
    H, L = 256, 2
    args = types.SimpleNamespace(rw_step=3, hops=1, ns_rate=4, ps_method="nb", dropout=0.0, margin=0.1,
                                 LLP_D=0.001, LLP_R=1000.0, True_label=0.001, KD_RM=0.0, KD_LM=0.0,
                                 predictor="mlp", lr=0.01)
    C = args.rw_step * args.hops * (1 + args.ns_rate)
    assert C == 15
    pairs = split_edge["train"]["edge"]                      # both directions (do_edge_split)
    row, col = data.adj_t                                    # src/main.py:148-149
    E = pairs.shape[0]
    B = int(N / (E / 65536))                                 # node_batch_size (src/main.py:335); >= N here
    B = min(B, N)
    P = min(65536, E)
    torch.manual_seed(0)
    model = models.MLP(L, F_, H, H, 0.0)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0)
    t_h = torch.randn(N, 256) * 0.3
    stu0 = [p.detach().clone() for p in model.parameters()]
    pred0 = [p.detach().clone() for p in pred.parameters()]
    tp = [p.detach().clone() for p in tpred.parameters()]

    g = torch.Generator().manual_seed(4)
    node_perm = torch.randperm(N, generator=g)[:B]
    link_perm = torch.randperm(E, generator=g)[:P]
    rowptr, colc = O.build_rowptr(row.numpy(), col.numpy(), N)
    pos, negs = O.neighbor_samplers(rowptr, colc, node_perm.numpy(), N, args.rw_step, "nb", args.ns_rate,
                                    args.hops, 99, 0)
    samples = torch.from_numpy(np.concatenate([pos, negs], 1)).long()     # src/main.py:94,183
    assert samples.shape == (B, 1 + C)
    neg = torch.randint(0, N, (2, P), generator=g)

    # oracle (CPU, fp32)
    sw = [p.clone().requires_grad_() for p in stu0[0::2]]
    sb = [p.clone().requires_grad_() for p in stu0[1::2]]
    pw = [p.clone().requires_grad_() for p in pred0[0::2]]
    pb = [p.clone().requires_grad_() for p in pred0[1::2]]
    edge = pairs[link_perm].t()
    res = O.distill_losses_fullbatch(data.x, t_h, samples, node_perm, edge, neg, sw, sb, pw, pb,
                                     tp[0::2], tp[1::2], args)
    stu_params = [p for pair in zip(sw, sb) for p in pair]
    pred_params = [p for pair in zip(pw, pb) for p in pair]
    _, grads, _ = O.distill_step(stu_params, pred_params, O.AdamState(stu_params + pred_params, lr=args.lr),
                                 res["loss"])

    # engine (fp32, same inputs)
    model, pred, tpred = model.to(DEV), pred.to(DEV), tpred.to(DEV)
    for p in tpred.parameters():
        p.requires_grad = False
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=args.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(DEV), t_h.to(DEV), row.numpy(), col.numpy(), N,
                                   args, opt, dtype="fp32", seed=5)
    n_neg = eng.step_fullbatch(node_perm.to(torch.int32).to(DEV), link_perm.to(torch.int32).to(DEV),
                               pairs.to(torch.int32).to(DEV).contiguous(), samples=samples.to(DEV),
                               neg=neg.to(DEV))
    torch.cuda.synchronize()
    assert n_neg == P
    t = eng.terms.cpu().double()
    for i, ref in ((1, res["label_loss"]), (2, res["llp_d"]), (3, res["llp_r"])):
        ref = float(ref)
        assert abs(t[i].item() - ref) <= 1e-4 * max(abs(ref), 1e-3), (i, t[i].item(), ref)
    for p, ref in zip(list(model.parameters()) + list(pred.parameters()), grads):
        got = p.grad.detach().cpu()
        err = float((got - ref).abs().max())
        assert err <= 1e-3 * max(float(ref.abs().max()), 1e-8) + 1e-9, (tuple(p.shape), err)
