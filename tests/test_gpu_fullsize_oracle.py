"""Oracle parity at the headline configuration's full size (BASELINE configs[2], ogbl-collab:
N = 235,868, F = 128, H = 1024, L = 3, B = 13,110 anchors, C = 36 contexts, P = 65,536 positive
edges), fp32: ONE train_minibatch link batch (src/main.py:73-143) on the HIP engine against the
CPU oracle (oracle/llp_oracle.py distill_losses_minibatch + distill_step) on the same injected
samples and negatives.

The golden fixtures pin the oracle to the reference at small sizes; this test closes the gap to
the benchmarked size, where the engine's unique-node student (~225k of 747k rows), the
multi-block compaction scans, the persistent GEMMs' tile walks and the long-segment sorts all
run at their production shapes.

State (VERDICT r05 "next" 1a): the weights at default init give gradients of 1e-9..1e-5 and a
clip coefficient of 1, so a post-Adam check there covers only the head.  The test scales every
student / predictor weight by 4 and the frozen teacher predictor's by 3 (t_h ~ N(0, 1)), with the
collab script's loss weights (True_label = 1, margin = 0.01; LLP_D = LLP_R = 1 so that every term
runs): student logits spread over (0, 0.99), gradient norms ~6 and ~12 (clip coefficients < 1 on
both modules) and 80-98 % of every tensor's entries live for the post-Adam check.

Bars: (1) the logits, north_star's "within 1e-4 on logits": s_r, t_r and out (the reference's
sigmoid outputs, src/main.py:105-106,126) within 1e-4 of the float64 oracle's, and the student's
pre-sigmoid logits within 1e-4 * max(1, |z|); (2) every loss term within 1e-4; (3) every gradient
within 2e-4 of its largest magnitude of the float64 oracle, or within 4x the error of the
reference's own fp32 arithmetic (the same oracle in float32) where that is larger; (4) after the
clip + Adam update every parameter whose clipped gradient is not vanishing equals the f64
oracle's within 1e-4 * lr (the rest move by at most lr: Adam's first step is lr * g / |g|).  The
oracles run on 16 host threads (about 70 s on the GPU box's share)."""
import time
import types

import pytest
import torch

import fullsize_check as FC

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_collab_fullsize_fp32_step_matches_oracle():
    import llp_data
    import llp_engine
    import models
    from oracle import llp_oracle as O
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.set_num_threads(16)
    t0 = time.time()
    data = llp_data.synthetic_collab(seed=0, with_eval=False)
    N, F_ = data.N, data.F
    H, L = 1024, 3
    B, P = 13_110, 65_536
    args = types.SimpleNamespace(rw_step=3, hops=3, ns_rate=3, ps_method="nb", dropout=0.0, margin=0.01,
                                 LLP_D=1.0, LLP_R=1.0, True_label=1.0, predictor="mlp", lr=0.001, KD_RM=0.0,
                                 KD_LM=0.0)
    C = args.rw_step * args.hops * (1 + args.ns_rate)
    assert (N, F_, C) == (235_868, 128, 36)
    g = torch.Generator().manual_seed(11)
    pairs = data.train_pairs
    x = data.x
    t_h = torch.randn(N, 256, generator=g)
    # injected draws: anchors (node_perm slice), contexts (walk nodes + negatives), link ids, randint negatives
    anchors = torch.randperm(N, generator=g)[:B]
    samples = torch.cat([anchors.view(B, 1), torch.randint(0, N, (B, C), generator=g)], 1)
    link = torch.randperm(pairs.size(0), generator=g)[:P]
    neg = torch.randint(0, N, (2, P), generator=g)

    torch.manual_seed(3)
    model = models.MLP(L, F_, H, H, 0.0).to(DEV)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(DEV)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(DEV)
    with torch.no_grad():          # a trained-like state (docstring): weights x4, teacher predictor x3
        for m, gain in ((model, 4.0), (pred, 4.0), (tpred, 3.0)):
            for p in m.parameters():
                if p.dim() == 2:
                    p.mul_(gain)
    for p in tpred.parameters():
        p.requires_grad = False
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=args.lr)
    ei = data.edge_index
    eng = llp_engine.DistillEngine(model, pred, tpred, x.to(DEV), t_h.to(DEV), ei[0].numpy(), ei[1].numpy(), N,
                                   args, opt, dtype="fp32", seed=5)
    assert eng._dedup_ok()
    params = list(model.parameters()) + list(pred.parameters())
    params0 = [p.detach().cpu().clone() for p in params]
    tpar = [p.detach().cpu().clone() for p in tpred.parameters()]
    eng.step_minibatch(anchors.to(torch.int32).to(DEV), link.to(torch.int32).to(DEV), pairs.to(torch.int32).to(DEV),
                       samples=samples.to(torch.int32).to(DEV), neg=neg.to(torch.int32).to(DEV))
    torch.cuda.synchronize()
    terms = eng.terms.cpu()
    lg = {k: v.detach().double().cpu() for k, v in eng.last_logits().items()}
    rows = eng.last_student_rows
    grads_gpu = [p.grad.detach().cpu().clone() for p in params]
    params1 = [p.detach().cpu().clone() for p in params]
    t1 = time.time()
    print(f"engine step done ({rows} unique student rows of {B * (C + 1) + 4 * P}); {t1 - t0:.1f} s", flush=True)
    assert 200_000 < rows < B * (C + 1) + 4 * P

    # ---- the oracle: the reference's arithmetic on the same draws (row-wise over x[this_target]),
    # in float64 (the truth) and in float32 (the reference's own arithmetic, torch on the CPU)
    def losses(sw, sb, pw, pb, d):
        tw, tb = [p.to(d) for p in tpar[0::2]], [p.to(d) for p in tpar[1::2]]
        return O.distill_losses_minibatch(x.to(d), t_h.to(d), samples, pairs[link].t(), neg, sw, sb, pw, pb, tw, tb,
                                          args)

    o64 = FC.oracle_step(O, losses, params0, L, args.lr, torch.float64)
    t2 = time.time()
    print(f"oracle step (f64) done; {t2 - t1:.1f} s", flush=True)
    o32 = FC.oracle_step(O, losses, params0, L, args.lr, torch.float32)
    print(f"oracle step (f32) done; {time.time() - t2:.1f} s", flush=True)
    FC.check(lg, terms, grads_gpu, params1, params0, o64, o32, args.lr, (B, C), 2 * P)
