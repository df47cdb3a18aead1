"""Pin the CPU oracle against golden vectors produced by the reference's own code
(tests/golden/gen_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

import golden_io as G
from oracle import llp_oracle as O


def test_kl_loss_matches_reference():
    z = G.load("kl_loss")
    i = 0
    while f"case{i}/s" in z.files:
        s = torch.from_numpy(z[f"case{i}/s"]); t = torch.from_numpy(z[f"case{i}/t"])
        T = float(z[f"case{i}/T"])
        assert torch.allclose(O.kl_loss(s, t, T), torch.from_numpy(z[f"case{i}/kl"]), rtol=1e-6, atol=1e-7)
        i += 1
    assert i == 3


def test_models_match_reference():
    z = G.load("models_fwd_bwd")
    ws = [torch.from_numpy(z[f"mlp/layers.{i}.weight"]).requires_grad_() for i in range(3)]
    bs = [torch.from_numpy(z[f"mlp/layers.{i}.bias"]).requires_grad_() for i in range(3)]
    x = torch.from_numpy(z["mlp/x"]).requires_grad_()
    y = O.mlp_forward(x, ws, bs, 0.0)
    assert torch.allclose(y, torch.from_numpy(z["mlp/y"]), atol=1e-6)
    y.backward(torch.from_numpy(z["mlp/gy"]))
    assert torch.allclose(x.grad, torch.from_numpy(z["mlp/gx"]), atol=1e-5)
    for i in range(3):
        assert torch.allclose(ws[i].grad, torch.from_numpy(z[f"mlp/grad/layers.{i}.weight"]), atol=1e-5)
    for kind in ("mlp", "inner"):
        ws = [torch.from_numpy(z[f"lp_{kind}/lins.{i}.weight"]) for i in range(3)]
        bs = [torch.from_numpy(z[f"lp_{kind}/lins.{i}.bias"]) for i in range(3)]
        xi = torch.from_numpy(z[f"lp_{kind}/xi"]).requires_grad_()
        xj = torch.from_numpy(z[f"lp_{kind}/xj"]).requires_grad_()
        o = O.link_predictor_forward(xi, xj, ws, bs, kind, 0.0)
        assert torch.allclose(o, torch.from_numpy(z[f"lp_{kind}/out"]), atol=1e-6)
        o.backward(torch.from_numpy(z[f"lp_{kind}/gout"]))
        assert torch.allclose(xi.grad, torch.from_numpy(z[f"lp_{kind}/gxi"]), atol=1e-5)
        assert torch.allclose(xj.grad, torch.from_numpy(z[f"lp_{kind}/gxj"]), atol=1e-5)


def test_norm_models_match_reference():
    """norm_type 'layer' / 'batch' MLP (src/models.py:6-54) against the reference's own
    module: train-mode forward / backward, running statistics, eval-mode forward."""
    z = G.load("models_norm_fwd_bwd")
    for kind in ("layer", "batch"):
        pre = f"mlp_{kind}"
        ws = [torch.from_numpy(z[f"{pre}/layers.{i}.weight"]).requires_grad_() for i in range(3)]
        bs = [torch.from_numpy(z[f"{pre}/layers.{i}.bias"]).requires_grad_() for i in range(3)]
        nps = [torch.from_numpy(z[f"{pre}/norms.{i}.{w}"]).requires_grad_() for i in range(2) for w in ("weight", "bias")]
        bufs = None
        if kind == "batch":   # the recorded state is after the forward: restart from torch's initial statistics
            bufs = [t for i in range(2) for t in (torch.zeros(40), torch.ones(40), torch.tensor(0))]
        norms = O.make_norms(kind, nps, bufs)
        x = torch.from_numpy(z[f"{pre}/x"]).requires_grad_()
        y = O.mlp_forward(x, ws, bs, 0.0, norms=norms)
        assert torch.allclose(y, torch.from_numpy(z[f"{pre}/y"]), atol=1e-5)
        y.backward(torch.from_numpy(z[f"{pre}/gy"]))
        assert torch.allclose(x.grad, torch.from_numpy(z[f"{pre}/gx"]), atol=1e-5)
        for i in range(3):
            assert torch.allclose(ws[i].grad, torch.from_numpy(z[f"{pre}/grad/layers.{i}.weight"]), atol=1e-5)
        for i in range(2):
            for j, w in enumerate(("weight", "bias")):
                assert torch.allclose(nps[2 * i + j].grad, torch.from_numpy(z[f"{pre}/grad/norms.{i}.{w}"]),
                                      atol=1e-5)
            if kind == "batch":
                for w in ("running_mean", "running_var"):
                    assert torch.allclose(norms[i][w], torch.from_numpy(z[f"{pre}/norms.{i}.{w}"]), atol=1e-6)
        ye = O.mlp_forward(torch.from_numpy(z[f"{pre}/x_eval"]), ws, bs, 0.0, training=False, norms=norms)
        assert torch.allclose(ye, torch.from_numpy(z[f"{pre}/y_eval"]), atol=1e-5)


def _n_lin(case):
    return 2 * case.L


def oracle_norms(case, stu):
    """The oracle's norms for a norm_type case (None for 'none'), fresh running statistics."""
    if case.norm_type == "none":
        return None
    return O.make_norms(case.norm_type, stu[_n_lin(case):], case.stu_buf0)


def replay_oracle(case):
    a = case.args
    stu = [p.clone().requires_grad_() for p in case.stu0]
    pred = [p.clone().requires_grad_() for p in case.pred0]
    tw, tb = case.tpred[0::2], case.tpred[1::2]
    adam = O.AdamState(stu + pred, lr=float(a.lr))
    records = []
    norms = oracle_norms(case, stu)
    nl = _n_lin(case)
    for st in case.steps:
        sw, sb = stu[:nl][0::2], stu[:nl][1::2]
        pw, pb = pred[0::2], pred[1::2]
        if norms is not None:   # this step's gamma / beta, the running statistics carried over
            for i, nm in enumerate(norms):
                nm["weight"], nm["bias"] = stu[nl + 2 * i], stu[nl + 2 * i + 1]
        if case.full:
            r = O.distill_losses_fullbatch(case.x, case.t_h, st.samples, st.node_perm, st.edge, st.neg_edge,
                                           sw, sb, pw, pb, tw, tb, a, stu_norms=norms)
        else:
            r = O.distill_losses_minibatch(case.x, case.t_h, st.samples, st.edge, st.neg_edge,
                                           sw, sb, pw, pb, tw, tb, a, stu_norms=norms)
        new, grads, _ = O.distill_step(stu, pred, adam, r["loss"])
        records.append((r, grads))
        stu = [p.clone().requires_grad_() for p in new[:len(stu)]]
        pred = [p.clone().requires_grad_() for p in new[len(stu):]]
    replay_oracle.norms = norms
    return records, stu, pred


@pytest.mark.parametrize("name", G.MINIBATCH_CASES + G.FULLBATCH_CASES)
def test_oracle_replays_reference_steps(name):
    case = G.load_case(name)
    records, stu, pred = replay_oracle(case)
    for st, (r, grads) in zip(case.steps, records):
        for k in ("llp_d", "llp_r"):
            if getattr(st, k) is not None:
                assert abs(float(r[k]) - getattr(st, k)) <= 1e-6 * max(1.0, abs(getattr(st, k))), k
        # (norm cases: BatchNorm / LayerNorm statistics are thread-count dependent sums in torch: 1e-5)
        assert abs(float(r["label_loss"]) - st.bce) <= (1e-6 if case.norm_type == "none" else 1e-5)
        for g, ref in zip(grads, st.grads):
            assert torch.allclose(g, ref, rtol=1e-4, atol=1e-6), (name, (g - ref).abs().max())
    # (BatchNorm: a Linear bias that feeds a BatchNorm has a zero gradient in exact arithmetic, so its
    # recorded gradients are rounding noise and Adam moves it by up to +-lr per step either way)
    free = {2 * l + 1 for l in range(case.L - 1)} if case.norm_type == "batch" else set()
    bound = 2 * float(case.args.lr) * len(case.steps)
    for i, (p, ref) in enumerate(zip(stu + pred, case.stu_final + case.pred_final)):
        d = (p.detach() - ref).abs()
        if i in free:
            assert d.max() <= bound, (name, i)
        elif case.norm_type != "none":
            # (norm cases: torch's statistics sums depend on the thread count, and Adam turns a ~0
            # gradient's rounding into a +-lr step: the GPU tests' criterion)
            assert (d <= 1e-4).float().mean() > 0.99 and d.max() <= bound, (name, i, d.max())
        else:
            assert torch.allclose(p.detach(), ref, rtol=1e-4, atol=1e-5), (name, d.max())
    norms = replay_oracle.norms
    if case.norm_type == "batch":   # running statistics after every step's forward
        # (the running mean follows the free biases above: momentum x their bound)
        shift = 0.1 * 2 * float(case.args.lr) * len(case.steps)
        for i, nm in enumerate(norms):
            for j, w in enumerate(("running_mean", "running_var")):
                assert torch.allclose(nm[w], case.stu_buf_final[3 * i + j], rtol=1e-5,
                                      atol=1e-6 + (shift if j == 0 else 0.0)), (name, w)
    if case.h_eval is not None:
        # eval-mode student (BatchNorm: running statistics) on the reference's final state, so the free
        # biases' drift above does not enter
        nl = _n_lin(case)
        fin = case.stu_final
        en = O.make_norms(case.norm_type, fin[nl:], case.stu_buf_final)
        he = O.mlp_forward(case.x, fin[:nl][0::2], fin[:nl][1::2], 0.0, training=False, norms=en)
        assert torch.allclose(he, case.h_eval, rtol=1e-4, atol=1e-5), (name, (he - case.h_eval).abs().max())
    # epoch loss (main.py:141-144) — weighted mean over steps of loss.item()
    n = 0
    tot = 0.0
    ep = 0
    steps_per_epoch = len(case.steps) // len(case.epoch_losses)
    for i, (st, (r, _)) in enumerate(zip(case.steps, records)):
        tot += float(r["loss"]) * st.edge.size(1)
        n += st.edge.size(1)
        if (i + 1) % steps_per_epoch == 0:
            assert abs(tot / n - case.epoch_losses[ep]) < 1e-5
            tot, n, ep = 0.0, 0, ep + 1


def _oracle_encoder(c, enc, training, norms=None):
    if c.encoder == "gcn":   # per conv: bias, lin.weight (PyG GCNConv parameter order)
        convs = [(enc[2 * i + 1], enc[2 * i]) for i in range(c.L)]
        return O.gcn_forward(c.x, c.edge_index, convs, 0.0, training=training)
    convs = [tuple(enc[3 * i:3 * i + 3]) for i in range(c.L)]
    if norms is not None:   # the norms' gamma / beta follow the convs' parameters (model.parameters())
        for i, nm in enumerate(norms):
            nm["weight"], nm["bias"] = enc[3 * c.L + 2 * i], enc[3 * c.L + 2 * i + 1]
    return O.sage_forward(c.x, c.edge_index, convs, 0.0, training=training, updated=c.updated, norms=norms)


def _oracle_teacher_replay(c):
    """Oracle restatement of the teacher's train() on the recorded permutations
    and negatives: SAGE forward, LinkPredictor, BCE, clip per module, Adam."""
    enc = [p.clone().requires_grad_() for p in c.enc0]
    pred = [p.clone().requires_grad_() for p in c.pred0]
    adam = O.AdamState(enc + pred, lr=0.005)
    recs = []
    norms = None if c.norm_type == "none" else O.make_norms(c.norm_type, enc[3 * c.L:], c.enc_buf0)
    _oracle_teacher_replay.norms = norms
    for st in c.steps:
        h = _oracle_encoder(c, enc, True, norms)
        tr = torch.cat([st.edge, st.neg_edge], 1)
        out = O.link_predictor_forward(h[tr[0]], h[tr[1]], pred[0::2], pred[1::2]).squeeze(-1)
        label = torch.cat([torch.ones(st.edge.size(1)), torch.zeros(st.neg_edge.size(1))])
        loss = O.bce_loss(out, label)
        new, grads, _ = O.distill_step(enc, pred, adam, loss)
        recs.append((float(loss), grads))
        enc = [p.clone().requires_grad_() for p in new[:len(enc)]]
        pred = [p.clone().requires_grad_() for p in new[len(enc):]]
    return recs, enc, pred


@pytest.mark.parametrize("name", G.TEACHER_CASES)
def test_oracle_replays_reference_teacher(name):
    c = G.load_teacher_case(name)
    recs, enc, pred = _oracle_teacher_replay(c)
    for st, (loss, grads) in zip(c.steps, recs):
        assert abs(loss - st.bce) <= 1e-6
        for g, ref in zip(grads, st.grads):
            assert torch.allclose(g, ref, rtol=1e-4, atol=1e-6), (name, (g - ref).abs().max())
    # (BatchNorm: the bias of lin_l feeding a BatchNorm is free, as in the student's case above)
    free = {3 * l + 1 for l in range(c.L - 1)} if c.norm_type == "batch" else set()
    for i, (p, ref) in enumerate(zip(enc + pred, c.enc_final + c.pred_final)):
        if i in free:
            assert (p.detach() - ref).abs().max() <= 2 * 0.005 * len(c.steps), (name, i)
            continue
        assert torch.allclose(p.detach(), ref, rtol=1e-4, atol=1e-5), (name, (p - ref).abs().max())
    norms = _oracle_teacher_replay.norms
    if c.norm_type == "batch":
        for i, nm in enumerate(norms):
            for j, w in enumerate(("running_mean", "running_var")):
                shift = 0.1 * 2 * 0.005 * len(c.steps) if j == 0 else 0.0
                assert torch.allclose(nm[w], c.enc_buf_final[3 * i + j], rtol=1e-5, atol=1e-6 + shift), (name, w)
    if c.norm_type == "batch":   # eval on the reference's final state (free-bias drift, as above)
        enc = c.enc_final
        norms = O.make_norms("batch", enc[3 * c.L:], c.enc_buf_final)
    h = _oracle_encoder(c, [p.detach() for p in enc], False, norms)
    assert torch.allclose(h, c.h_eval, rtol=1e-4, atol=1e-5)
