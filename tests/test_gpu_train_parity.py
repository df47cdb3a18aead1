"""End-to-end training parity (BASELINE configs[0] shape, north_star's "within
1e-4 on logits and exactly on Hits@K"): the fp32 engine and the CPU oracle
train the same student for 20 full-batch ``train`` epochs on a synthetic
cora-shape graph (N=2,708, F=1,433, the cora transductive script's LLP
settings: LLP_D=0.001, LLP_R=1, True_label=0.1, rw_step=3, hops=2, ns_rate=1 ->
C=12, lr=0.01; scripts/LLP_transductive.sh:1), with every random draw shared
(contexts from the oracle's Philox sampler, negatives injected, dropout 0:
the reference's dropout streams are not portable).  One link batch
per epoch, as on cora.  After every 5 epochs both sides evaluate
(``test_transductive``, src/train_teacher_gnn.py:76-155): the GPU path
(device MLP forward, device scoring, device ogb hits@K) against the oracle
(torch-CPU forward, ogb's hits@K formula on CPU).

Bars.  (1) Eval parity on the weights the GPU trained: the test-edge logits
within 1e-4 (absolute, on logits of O(1)) and Hits@10/20/50 on valid and
test equal up to one edge flipping at a near-tie (|diff| <= 1 / #positives).
(2) The two training trajectories, which drift apart in fp32 (a near-zero
gradient's sign differs between summation orders and Adam moves that weight
by ~lr): the loss within 1e-3 relative at every epoch and Hits@20 of the
GPU-trained model within 0.02 of the oracle-trained model's (north_star's
bar against the reference is 0.1)."""
import types

import numpy as np
import pytest
import torch

from oracle import llp_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_cora_training_tracks_oracle_on_logits_and_hits():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import llp_datasets
    import llp_engine
    import llp_train
    import models
    data, split_edge = llp_datasets.synthetic_transductive("cora")
    N, F_ = data.x.shape
    H, L = 256, 2
    args = types.SimpleNamespace(rw_step=3, hops=2, ns_rate=1, ps_method="nb", dropout=0.0, margin=0.1,
                                 LLP_D=0.001, LLP_R=1.0, True_label=0.1, KD_RM=0.0, KD_LM=0.0, predictor="mlp",
                                 lr=0.01)
    pairs = split_edge["train"]["edge"]
    row, col = data.adj_t
    E = pairs.shape[0]
    B = min(int(N / (E / 65536)), N)
    P = min(65536, E)
    torch.manual_seed(0)
    model = models.MLP(L, F_, H, H, 0.0)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0)
    t_h = torch.randn(N, 256) * 0.3
    stu = [p.detach().clone().requires_grad_() for p in model.parameters()]
    prd = [p.detach().clone().requires_grad_() for p in pred.parameters()]
    tp = [p.detach().clone() for p in tpred.parameters()]
    adam = O.AdamState(stu + prd, lr=args.lr)

    model, pred, tpred = model.to(DEV), pred.to(DEV), tpred.to(DEV)
    for p in tpred.parameters():
        p.requires_grad = False
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=args.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(DEV), t_h.to(DEV), row.numpy(), col.numpy(), N,
                                   args, opt, dtype="fp32", seed=5)
    pairs_d = pairs.to(torch.int32).to(DEV).contiguous()
    rowptr, colc = O.build_rowptr(row.numpy(), col.numpy(), N)
    g = torch.Generator().manual_seed(4)

    def oracle_eval(sw, sb, pw, pb):
        with torch.no_grad():
            h = O.mlp_forward(data.x, sw, sb, 0.0, training=False)
            out = {}
            for split in ("valid", "test"):
                pos = split_edge[split]["edge"].t()
                neg = split_edge[split]["edge_neg"].t()
                sp, lp = O.link_predictor_forward(h[pos[0]], h[pos[1]], pw, pb, "mlp", 0.0, False, return_logit=True)
                sn = O.link_predictor_forward(h[neg[0]], h[neg[1]], pw, pb, "mlp", 0.0, False)
                out[split] = (sp.squeeze(-1), sn.squeeze(-1), lp.squeeze(-1))
        return out

    drift = []
    for epoch in range(1, 21):
        node_perm = torch.randperm(N, generator=g)[:B]
        link_perm = torch.randperm(E, generator=g)[:P]
        pos, negs = O.neighbor_samplers(rowptr, colc, node_perm.numpy(), N, args.rw_step, "nb", args.ns_rate,
                                        args.hops, 99, O.STREAMS_PER_STEP * epoch)
        samples = torch.from_numpy(np.concatenate([pos, negs], 1)).long()
        neg = torch.randint(0, N, (2, P), generator=g)
        # oracle step
        r = O.distill_losses_fullbatch(data.x, t_h, samples, node_perm, pairs[link_perm].t(), neg, stu[0::2],
                                       stu[1::2], prd[0::2], prd[1::2], tp[0::2], tp[1::2], args)
        new, _, _ = O.distill_step(stu, prd, adam, r["loss"])
        stu = [p.clone().requires_grad_() for p in new[:len(stu)]]
        prd = [p.clone().requires_grad_() for p in new[len(stu):]]
        # engine step, same inputs
        eng.step_fullbatch(node_perm.to(torch.int32).to(DEV), link_perm.to(torch.int32).to(DEV), pairs_d,
                           samples=samples.to(DEV), neg=neg.to(DEV))
        torch.cuda.synchronize()
        loss_gpu, loss_ref = float(eng.terms[0]), float(r["loss"])
        drift.append(abs(loss_gpu - loss_ref) / max(abs(loss_ref), 1e-6))
        if epoch % 5:
            continue
        res, h = llp_train.test_transductive(model, pred, data, split_edge, None, 65536, "mlp", "cora")
        model.train()
        pred.train()
        # (1) eval parity on the weights the GPU trained: oracle forward + ogb hits@K on CPU
        sw = [p.detach().cpu() for p in model.parameters()]
        pw = [p.detach().cpu() for p in pred.parameters()]
        ref = oracle_eval(sw[0::2], sw[1::2], pw[0::2], pw[1::2])
        with torch.no_grad():
            tpos = split_edge["test"]["edge"].t().to(DEV)
            prob = pred(h[tpos[0]], h[tpos[1]]).squeeze(-1).float().cpu()     # device scorer (HIP ops)
            W = [w.double() for w in pw]
            hd = h.double().cpu()
            z = hd[tpos[0].cpu()] * hd[tpos[1].cpu()]
            logit = (torch.relu(z @ W[0].t() + W[1]) @ W[2].t() + W[3]).squeeze(-1)
        assert (prob - ref["test"][0]).abs().max().item() <= 2.5e-5, epoch
        dlog = (logit - ref["test"][2].double()).abs().max().item()
        assert dlog <= 1e-4, (epoch, dlog)
        for K in (10, 20, 50):
            for i, split in enumerate(("valid", "test")):
                got = res[f"Hits@{K}"][i]
                want = O.hits_at_k(ref[split][0], ref[split][1], K)
                n_pos = split_edge[split]["edge"].shape[0]
                assert abs(got - want) <= 1.0 / n_pos + 1e-12, (epoch, K, split, got, want)
        # (2) the two training trajectories: the GPU-trained model against the oracle-trained one
        mine = oracle_eval(stu[0::2], stu[1::2], prd[0::2], prd[1::2])
        h20 = [res["Hits@20"][i] for i in range(2)]
        h20_ref = [O.hits_at_k(mine[s_][0], mine[s_][1], 20) for s_ in ("valid", "test")]
        print(f"epoch {epoch}: loss drift max {max(drift):.2e}, Hits@20 gpu {h20} oracle-trained {h20_ref}")
        assert all(abs(a - b) <= 0.02 for a, b in zip(h20, h20_ref)), (epoch, h20, h20_ref)
    assert max(drift) <= 1e-3, drift
