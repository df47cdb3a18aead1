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


def replay_oracle(case):
    a = case.args
    stu = [p.clone().requires_grad_() for p in case.stu0]
    pred = [p.clone().requires_grad_() for p in case.pred0]
    tw, tb = case.tpred[0::2], case.tpred[1::2]
    adam = O.AdamState(stu + pred, lr=float(a.lr))
    records = []
    for st in case.steps:
        sw, sb = stu[0::2], stu[1::2]
        pw, pb = pred[0::2], pred[1::2]
        if case.full:
            r = O.distill_losses_fullbatch(case.x, case.t_h, st.samples, st.node_perm, st.edge, st.neg_edge,
                                           sw, sb, pw, pb, tw, tb, a)
        else:
            r = O.distill_losses_minibatch(case.x, case.t_h, st.samples, st.edge, st.neg_edge,
                                           sw, sb, pw, pb, tw, tb, a)
        new, grads, _ = O.distill_step(stu, pred, adam, r["loss"])
        records.append((r, grads))
        stu = [p.clone().requires_grad_() for p in new[:len(stu)]]
        pred = [p.clone().requires_grad_() for p in new[len(stu):]]
    return records, stu, pred


@pytest.mark.parametrize("name", G.MINIBATCH_CASES + G.FULLBATCH_CASES)
def test_oracle_replays_reference_steps(name):
    case = G.load_case(name)
    records, stu, pred = replay_oracle(case)
    for st, (r, grads) in zip(case.steps, records):
        for k in ("llp_d", "llp_r"):
            if getattr(st, k) is not None:
                assert abs(float(r[k]) - getattr(st, k)) <= 1e-6 * max(1.0, abs(getattr(st, k))), k
        assert abs(float(r["label_loss"]) - st.bce) <= 1e-6
        for g, ref in zip(grads, st.grads):
            assert torch.allclose(g, ref, rtol=1e-4, atol=1e-6), (name, (g - ref).abs().max())
    for p, ref in zip(stu + pred, case.stu_final + case.pred_final):
        assert torch.allclose(p.detach(), ref, rtol=1e-4, atol=1e-5), (name, (p - ref).abs().max())
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


def _oracle_encoder(c, enc, training):
    if c.encoder == "gcn":   # per conv: bias, lin.weight (PyG GCNConv parameter order)
        convs = [(enc[2 * i + 1], enc[2 * i]) for i in range(c.L)]
        return O.gcn_forward(c.x, c.edge_index, convs, 0.0, training=training)
    convs = [tuple(enc[3 * i:3 * i + 3]) for i in range(c.L)]
    return O.sage_forward(c.x, c.edge_index, convs, 0.0, training=training, updated=c.updated)


def _oracle_teacher_replay(c):
    """Oracle restatement of the teacher's train() on the recorded permutations
    and negatives: SAGE forward, LinkPredictor, BCE, clip per module, Adam."""
    enc = [p.clone().requires_grad_() for p in c.enc0]
    pred = [p.clone().requires_grad_() for p in c.pred0]
    adam = O.AdamState(enc + pred, lr=0.005)
    recs = []
    for st in c.steps:
        h = _oracle_encoder(c, enc, True)
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
    for p, ref in zip(enc + pred, c.enc_final + c.pred_final):
        assert torch.allclose(p.detach(), ref, rtol=1e-4, atol=1e-5), (name, (p - ref).abs().max())
    h = _oracle_encoder(c, [p.detach() for p in enc], False)
    assert torch.allclose(h, c.h_eval, rtol=1e-4, atol=1e-5)
