"""Oracle parity at the headline configuration's full size (BASELINE configs[2], ogbl-collab:
N = 235,868, F = 128, H = 1024, L = 3, B = 13,110 anchors, C = 36 contexts, P = 65,536 positive
edges), fp32: ONE train_minibatch link batch (src/main.py:73-143) on the HIP engine against the
CPU oracle (oracle/llp_oracle.py distill_losses_minibatch + distill_step) on the same injected
samples and negatives.

The golden fixtures pin the oracle to the reference at small sizes; this test closes the gap to
the benchmarked size, where the engine's unique-node student (~225k of 747k rows), the
multi-block compaction scans, the persistent GEMMs' tile walks and the long-segment sorts all
run at their production shapes.  Bars (VERDICT r04 "next" item 2): every loss term within 1e-4,
every gradient within 2e-4 of its largest magnitude of the float64 oracle, or within 4x the error
of the reference's own fp32 arithmetic (the same oracle in float32) where that is larger, and after
the clip + Adam update every parameter whose gradient is not vanishing equals the f64 oracle's
within 1e-4 * lr (the rest move by at most lr: Adam's first step is lr * g / |g|).  The oracles
run on 16 host threads (about 70 s on the GPU box's share)."""
import time
import types

import numpy as np
import pytest
import torch

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
    args = types.SimpleNamespace(rw_step=3, hops=3, ns_rate=3, ps_method="nb", dropout=0.0, margin=0.1,
                                 LLP_D=1.0, LLP_R=1.0, True_label=0.1, predictor="mlp", lr=0.001, KD_RM=0.0,
                                 KD_LM=0.0)
    C = args.rw_step * args.hops * (1 + args.ns_rate)
    assert (N, F_, C) == (235_868, 128, 36)
    g = torch.Generator().manual_seed(11)
    pairs = data.train_pairs
    x = data.x
    t_h = torch.randn(N, 256, generator=g) * 0.3
    # injected draws: anchors (node_perm slice), contexts (walk nodes + negatives), link ids, randint negatives
    anchors = torch.randperm(N, generator=g)[:B]
    samples = torch.cat([anchors.view(B, 1), torch.randint(0, N, (B, C), generator=g)], 1)
    link = torch.randperm(pairs.size(0), generator=g)[:P]
    neg = torch.randint(0, N, (2, P), generator=g)

    torch.manual_seed(3)
    model = models.MLP(L, F_, H, H, 0.0).to(DEV)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(DEV)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(DEV)
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
    rows = eng.last_student_rows
    grads_gpu = [p.grad.detach().cpu().clone() for p in params]
    params1 = [p.detach().cpu().clone() for p in params]
    t1 = time.time()
    print(f"engine step done ({rows} unique student rows of {B * (C + 1) + 4 * P}); {t1 - t0:.1f} s", flush=True)
    assert 200_000 < rows < B * (C + 1) + 4 * P

    # ---- the oracle: the reference's arithmetic on the same draws (row-wise over x[this_target]),
    # in float64 (the truth) and in float32 (the reference's own arithmetic, torch on the CPU).  At
    # this size a weight gradient is a cancelling sum of up to 603k rows (|sum| << sum |term|), so
    # fp32 rounding of the order of the 2e-4 bar is inherent to the arithmetic: the bar per
    # gradient tensor is 2e-4 of its largest magnitude against the f64 truth, or no worse than
    # 4x what the fp32 reference arithmetic itself reaches on the same tensor.
    def oracle(d):
        leaves = [p.to(d).clone().requires_grad_() for p in params0]
        sw, sb = leaves[0:2 * L:2], leaves[1:2 * L:2]
        pw, pb = leaves[2 * L::2], leaves[2 * L + 1::2]
        tw, tb = [p.to(d) for p in tpar[0::2]], [p.to(d) for p in tpar[1::2]]
        prev = torch.get_default_dtype()
        torch.set_default_dtype(d)          # the oracle's label vector (torch.ones / zeros) in d too
        try:
            r = O.distill_losses_minibatch(x.to(d), t_h.to(d), samples, pairs[link].t(), neg, sw, sb, pw, pb, tw,
                                           tb, args)
            adam = O.AdamState(leaves, lr=args.lr)
            new, grads_clip, norms = O.distill_step(leaves[:2 * L], leaves[2 * L:], adam, r["loss"])
        finally:
            torch.set_default_dtype(prev)
        # the engine's .grad holds the unclipped gradient (the clip is applied inside its Adam launch);
        # distill_step returns clipped ones: undo each module's clip coefficient (clip_grad_norm_,
        # max_norm 1, src/main.py:134-135)
        raw, coefs = [], []
        for grp, total in ((slice(0, 2 * L), norms[0]), (slice(2 * L, len(params)), norms[1])):
            coef = min(1.0, 1.0 / (float(total) + 1e-6))
            raw += [gc.detach() / coef for gc in grads_clip[grp]]
            coefs += [coef] * len(grads_clip[grp])
        terms_o = {k: r[k].item() for k in ("loss", "label_loss", "llp_d", "llp_r")}
        return terms_o, raw, [p.detach() for p in new], coefs

    t64, g64, p64, coef64 = oracle(torch.float64)
    t2 = time.time()
    print(f"oracle step (f64) done; {t2 - t1:.1f} s", flush=True)
    t32, g32, _, _ = oracle(torch.float32)
    print(f"oracle step (f32) done; {time.time() - t2:.1f} s", flush=True)

    for i, k in ((0, "loss"), (1, "label_loss"), (2, "llp_d"), (3, "llp_r")):
        ref = t64[k]
        assert abs(terms[i].item() - ref) <= 1e-4 * max(1.0, abs(ref)), (k, terms[i].item(), ref)
    rows_err = []
    for a, b, c, p in zip(grads_gpu, g64, g32, params0):
        m = b.abs().max().item()
        e_hip = (a.double() - b).abs().max().item()
        e_ref = (c.double() - b).abs().max().item()
        rows_err.append((tuple(p.shape), m, e_hip, e_ref))
    print("gradient max |g|, then error / max |g| (HIP fp32 | reference fp32) per tensor:", flush=True)
    for shape, m, e_hip, e_ref in rows_err:
        print(f"  {str(shape):14s} {m:.3e}  {e_hip / m:.2e} | {e_ref / m:.2e}", flush=True)
    for shape, m, e_hip, e_ref in rows_err:
        assert e_hip <= max(2e-4 * m, 4.0 * e_ref), (shape, m, e_hip, e_ref)
    # parameters after clip + Adam: where coef * |g| >= 1e-5 (1000x Adam's eps, so the update
    # lr * g / (|g| + eps) is insensitive to the gradient's rounding) within 1e-4 * lr of the truth;
    # everywhere at most 2 lr apart (Adam's first step moves a weight by at most lr)
    lr = args.lr
    for a, b, gref, coef in zip(params1, p64, g64, coef64):
        d = (a.double() - b).abs()
        assert d.max().item() <= 2 * lr * (1 + 1e-3), d.max().item()
        live = coef * gref.abs() >= 1e-5
        if bool(live.any()):
            assert d[live].max().item() <= 1e-4 * lr + 1e-8, d[live].max().item()
    assert np.isfinite(terms.numpy()).all()
