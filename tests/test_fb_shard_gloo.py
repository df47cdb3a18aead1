"""The node-sharded full-batch student (DistillEngine._fb_shard, default at several ranks),
checked on CPU over 2 and 3 gloo ranks with the oracle as the model: each rank runs the
student MLP on its slice of the nodes, the slices are all-gathered with the engine's
own `_all_gather_rows`, the rank's shard of the anchors / label edges gives d(loss)/dh
over all nodes, `_reduce_scatter_rows` sums it onto the owners' slices, and the slice
backward plus the SUM all-reduce of every gradient equals the single-rank gradient of
`train`'s loss (src/main.py:173-222, KD terms off).  The GPU engine's own 2-rank run of
the same path is tests/test_gpu_multirank.py (gated until measured)."""
import os
import socket
import sys
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    g = torch.Generator().manual_seed(0)
    N, F_, H, T = 301, 16, 32, 32      # T = H: the oracle also forms the (zero-weight) KD_RM term
    B, C1, P = 24, 7, 40
    x = torch.randn(N, F_, generator=g, dtype=torch.float64)
    t_h = torch.randn(N, T, generator=g, dtype=torch.float64)
    samples = torch.randint(0, N, (B, C1), generator=g)
    edge = torch.randint(0, N, (2, P), generator=g)
    neg = torch.randint(0, N, (2, P), generator=g)
    mk = lambda shp: [torch.randn(*s, generator=g, dtype=torch.float64) * 0.3 for s in shp]
    mkb = lambda shp: [torch.randn(s[0], generator=g, dtype=torch.float64) * 0.1 for s in shp]
    ss, sp, st = [(H, F_), (H, H)], [(H, H), (1, H)], [(T, T), (1, T)]
    params = (mk(ss), mkb(ss), mk(sp), mkb(sp), mk(st), mkb(st))
    args = types.SimpleNamespace(dropout=0.0, margin=0.05, predictor="mlp", True_label=0.5, LLP_D=1.0, LLP_R=1.0,
                                 KD_RM=0.0, KD_LM=0.0)
    return N, x, t_h, samples, edge, neg, params, args


def _shard_loss(O, h_leaf, rank, world, prob):
    """This rank's weighted share of the full-batch loss as a function of h (all nodes)."""
    N, x, t_h, samples, edge, neg, (sw, sb, pw, pb, tw, tb), args = prob
    B, P = samples.shape[0], edge.shape[1]
    b0, b1 = rank * B // world, (rank + 1) * B // world
    p0, p1 = rank * P // world, (rank + 1) * P // world
    lpw = [w.clone().requires_grad_() for w in pw]
    lpb = [b.clone().requires_grad_() for b in pb]
    real = O.mlp_forward
    O.mlp_forward = lambda *a, **k: h_leaf          # the student's output is given (sharded above)
    try:
        r = O.distill_losses_fullbatch(x, t_h, samples[b0:b1], samples[b0:b1, 0], edge[:, p0:p1], neg[:, p0:p1],
                                       sw, sb, lpw, lpb, tw, tb, args)
    finally:
        O.mlp_forward = real
    fb, fp = (b1 - b0) / B, (p1 - p0) / P
    loss = args.True_label * r["label_loss"] * fp + (args.LLP_D * r["llp_d"] + args.LLP_R * r["llp_r"]) * fb
    return loss, lpw + lpb


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
    from oracle import llp_oracle as O
    import llp_engine
    torch.set_default_dtype(torch.float64)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = _problem()
    N, x, t_h, samples, edge, neg, (sw, sb, pw, pb, tw, tb), args = prob
    fake = types.SimpleNamespace(world=world, rank=rank, group=None, N=N, emulate_shard=None, shard_student=True,
                                 _batch_norm=False)
    r0, n_rows, n_loc, s_world, s_rank = llp_engine.DistillEngine._fb_shard(fake, 0.0, True)
    assert (s_world, s_rank, n_loc) == (world, rank, -(-N // world))
    lw = [w.clone().requires_grad_() for w in sw]
    lb = [b.clone().requires_grad_() for b in sb]
    h_loc = O.mlp_forward(x[r0:r0 + n_rows], lw, lb)
    H = h_loc.shape[1]
    part = torch.zeros(n_loc, H)
    part[:n_rows] = h_loc.detach()
    full = torch.empty(world * n_loc, H)
    llp_engine.DistillEngine._all_gather_rows(fake, full, part, world, rank)
    h_leaf = full[:N].clone().requires_grad_()
    loss, pleaves = _shard_loss(O, h_leaf, rank, world, prob)
    grads = torch.autograd.grad(loss, [h_leaf] + pleaves)
    dh_full = torch.zeros(world * n_loc, H)
    dh_full[:N] = grads[0]
    dh = torch.empty(n_loc, H)
    llp_engine.DistillEngine._reduce_scatter_rows(fake, dh, dh_full, world, rank)
    sgrads = torch.autograd.grad(h_loc, lw + lb, dh[:n_rows])
    flat = torch.cat([g.reshape(-1) for g in list(sgrads) + list(grads[1:])])
    tot = torch.tensor([float(loss.detach())])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put((flat.numpy().copy(), float(tot.item())))
    dist.barrier()
    dist.destroy_process_group()


def _single():
    from oracle import llp_oracle as O
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        prob = _problem()
        N, x, t_h, samples, edge, neg, (sw, sb, pw, pb, tw, tb), args = prob
        lw = [w.clone().requires_grad_() for w in sw]
        lb = [b.clone().requires_grad_() for b in sb]
        h = O.mlp_forward(x, lw, lb)
        loss, pleaves = _shard_loss(O, h, 0, 1, prob)
        g = torch.autograd.grad(loss, lw + lb + pleaves)
    finally:
        torch.set_default_dtype(old)
    return torch.cat([t.reshape(-1) for t in g]).numpy(), float(loss.detach())


@pytest.mark.parametrize("world", [2, 3, 4])   # 4: the physics config's rank count (configs[3])
def test_node_sharded_student_sums_to_the_batch_gradient(world):
    full, full_loss = _single()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    flat, loss = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(loss - full_loss) <= 1e-12 * max(1.0, abs(full_loss)), (loss, full_loss)
    np.testing.assert_allclose(flat, full, rtol=1e-10, atol=1e-13)


def test_fb_shard_gating():
    """_fb_shard is on (shard_student, default) with several (or emulated) ranks, no dropout
    and no KD_RM; slices cover the nodes with ceil(N / world) rows, the last one ragged."""
    sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
    import llp_engine
    f = llp_engine.DistillEngine._fb_shard
    ns = lambda **kw: types.SimpleNamespace(**{"emulate_shard": None, "shard_student": True, "_batch_norm": False,
                                               **kw})
    eng = ns(world=4, rank=3, N=10)
    assert f(eng, 0.0, True) == (9, 1, 3, 4, 3)
    assert f(ns(world=4, rank=3, N=10, _batch_norm=True), 0.0, True) is None   # BatchNorm: replicated student
    eng.shard_student = False
    assert f(eng, 0.0, True) is None
    eng.shard_student = True
    assert f(eng, 0.5, True) is None and f(eng, 0.0, False) is None
    one = ns(world=1, rank=0, N=10)
    assert f(one, 0.0, True) is None
    one.emulate_shard = (1, 4)
    assert f(one, 0.0, True) == (3, 3, 3, 4, 1)
    for r in range(4):   # N=7 over 4 ranks: 2, 2, 2, 1 rows; N=6: rank 3 would have none -> off on every rank
        assert f(ns(world=4, rank=r, N=7), 0.0, True)[1] == (1 if r == 3 else 2)
        assert f(ns(world=4, rank=r, N=6), 0.0, True) is None
