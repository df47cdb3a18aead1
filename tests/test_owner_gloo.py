"""The owner decomposition of the minibatch step (DistillEngine.minibatch_owner),
checked on CPU with the oracle over 2, 3 and 8 gloo ranks.

Every rank holds the whole batch (samples, label edges, negatives).  Each predictor pair goes
to one rank (oracle pair_owner_assign: context pairs by the owner of the context node, label
pairs by the owner of their source, balanced).  A rank runs the student MLP only on the unique
end nodes of its pairs, the predictor on its pairs and the frozen teacher on its context pairs;
the context logits and teacher probabilities are placed into the [B, C] grid and SUM
all-reduced, every rank evaluates KL / rank over all anchors on that grid (gradient only into
its own pairs' logits) and the BCE of its own label pairs with the global normaliser.  The SUM
all-reduce of the ranks' gradients must equal the whole-batch gradient of train_minibatch's
loss (src/main.py:86-132), and the ranks' reported terms (KL / rank of the anchors of their
slice, their labels' BCE) must sum to the whole-batch loss.  The oracle is the checker; the GPU
engine's own 2-, 4- and 8-rank runs are in test_gpu_multirank.py."""
import os
import socket
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
    N, F_, H, T = 300, 16, 32, 16
    B, C1, P = 24, 7, 40
    x = torch.randn(N, F_, generator=g, dtype=torch.float64)
    t_h = torch.randn(N, T, generator=g, dtype=torch.float64)
    samples = torch.randint(0, N, (B, C1), generator=g)
    samples[:, 1:4] = torch.randint(0, N // 4, (B, 3), generator=g)   # skew: the first owner overflows
    edge = torch.randint(0, N, (2, P), generator=g)
    neg = torch.randint(0, N, (2, P), generator=g)
    shapes_s = [(H, F_), (H, H)]
    shapes_p = [(H, H), (1, H)]
    shapes_t = [(T, T), (1, T)]
    mk = lambda shp: [torch.randn(*s, generator=g, dtype=torch.float64) * 0.3 for s in shp]
    mkb = lambda shp: [torch.randn(s[0], generator=g, dtype=torch.float64) * 0.1 for s in shp]
    params = (mk(shapes_s), mkb(shapes_s), mk(shapes_p), mkb(shapes_p), mk(shapes_t), mkb(shapes_t))
    args = types.SimpleNamespace(dropout=0.0, margin=0.05, predictor="mlp", True_label=0.5, LLP_D=1.0, LLP_R=1.0)
    return N, x, t_h, samples, edge, neg, params, args


def _leaves(params):
    sw, sb, pw, pb, tw, tb = params
    leaves = [t.clone().requires_grad_() for t in sw + sb + pw + pb]
    ns, npd = len(sw), len(pw)
    return leaves, leaves[:ns], leaves[ns:2 * ns], leaves[2 * ns:2 * ns + npd], leaves[2 * ns + npd:], tw, tb


def _whole_batch():
    import sys
    sys.path.insert(0, REPO)
    from oracle import llp_oracle as O
    N, x, t_h, samples, edge, neg, params, args = _problem()
    leaves, lw, lb, lpw, lpb, tw, tb = _leaves(params)
    r = O.distill_losses_minibatch(x, t_h, samples, edge, neg, lw, lb, lpw, lpb, tw, tb, args)
    return [g.detach() for g in torch.autograd.grad(r["loss"], leaves)], float(r["loss"])


def _rank_part(rank, world, allreduce):
    """This rank's gradient and reported loss terms under the owner decomposition."""
    import sys
    sys.path.insert(0, REPO)
    from oracle import llp_oracle as O
    import torch.nn.functional as F
    N, x, t_h, samples, edge, neg, params, args = _problem()
    leaves, lw, lb, lpw, lpb, tw, tb = _leaves(params)
    B, C1 = samples.shape
    C = C1 - 1
    P = edge.shape[1]
    cs, ps, ns = (torch.from_numpy(a) for a in O.pair_owner_rank_items(samples.numpy(), edge.numpy(), neg.numpy(), N,
                                                                      world, rank))
    b_of, c_of = cs // C, cs % C
    ia = torch.cat([samples[b_of, 0], edge[0, ps], neg[0, ns]])
    ib = torch.cat([samples[b_of, 1 + c_of], edge[1, ps], neg[1, ns]])
    nodes, inv = torch.unique(torch.cat([ia, ib]), return_inverse=True)
    h = O.mlp_forward(x[nodes], lw, lb, 0.0)                      # the student on the unique ends only
    ra, rb = inv[:ia.numel()], inv[ia.numel():]
    out = O.link_predictor_forward(h[ra], h[rb], lpw, lpb, args.predictor).squeeze(-1)
    nc = cs.numel()
    s_loc = out[:nc]
    with torch.no_grad():
        t_loc = O.link_predictor_forward(t_h[samples[b_of, 0]], t_h[samples[b_of, 1 + c_of]], tw, tb,
                                         args.predictor).squeeze(-1)
    grid = torch.zeros(2, B * C, dtype=torch.float64)
    grid[0, cs] = s_loc.detach()
    grid[1, cs] = t_loc
    tot = allreduce(grid.clone())
    s_full = tot[0].clone()
    s_full = s_full.index_put((cs,), torch.zeros(nc, dtype=torch.float64)) + torch.zeros(B * C, dtype=torch.float64
                                                                                         ).index_put((cs,), s_loc)
    s_grid, t_grid = s_full.view(B, C), tot[1].view(B, C)
    kl = O.kl_loss(s_grid, t_grid, 1)
    rk = O.rank_loss(s_grid, t_grid, args.margin)
    lab_out = out[nc:]
    lab = torch.cat([torch.ones(ps.numel()), torch.zeros(ns.numel())]).double()
    bce = F.binary_cross_entropy(lab_out, lab, reduction="sum") / (2 * P)
    loss = args.True_label * bce + args.LLP_D * kl + args.LLP_R * rk
    grads = torch.autograd.grad(loss, leaves)
    b0, b1 = rank * B // world, (rank + 1) * B // world
    with torch.no_grad():
        f = (b1 - b0) / B
        kl_r = O.kl_loss(s_grid[b0:b1], t_grid[b0:b1], 1) * f if b1 > b0 else 0.0
        rk_r = O.rank_loss(s_grid[b0:b1], t_grid[b0:b1], args.margin) * f if b1 > b0 else 0.0
        rep = args.True_label * bce + args.LLP_D * kl_r + args.LLP_R * rk_r
    return [g.detach() for g in grads], float(rep), nodes.numel()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t
    grads, rep, n_nodes = _rank_part(rank, world, allreduce)
    flat = torch.cat([g.reshape(-1) for g in grads])
    tot = torch.tensor([rep], dtype=torch.float64)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put((flat.numpy().copy(), float(tot.item()), n_nodes))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_owner_decomposition_sums_to_the_batch_gradient(world):
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        full, full_loss = _whole_batch()
    finally:
        torch.set_default_dtype(old)
    full = torch.cat([g.reshape(-1) for g in full]).numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    flat, loss, n_nodes = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(loss - full_loss) <= 1e-12 * max(1.0, abs(full_loss)), (loss, full_loss)
    np.testing.assert_allclose(flat, full, rtol=1e-10, atol=1e-13)
    assert n_nodes > 0


def test_owner_assignment_properties():
    """Every pair on exactly one rank, cap_r pairs per rank, owned pairs first in item order."""
    import sys
    sys.path.insert(0, REPO)
    from oracle import llp_oracle as O
    g = np.random.default_rng(1)
    for N, n, W in ((235_868, 50_000, 8), (100, 37, 3), (10, 5, 8), (7, 0, 4)):
        key = np.minimum(g.integers(0, N // 2 + 1, n), N - 1)
        sel, off = O.pair_owner_assign(key, N, W)
        assert sorted(sel.tolist()) == list(range(n))
        assert np.array_equal(np.diff(off), [(r + 1) * n // W - r * n // W for r in range(W)])
        own = O.node_owner(key, N, W)
        for r in range(W):
            mine = sel[off[r]:off[r + 1]]
            kept = mine[own[mine] == r]
            assert np.array_equal(kept, np.sort(kept))                  # owned ones in item order
            k = kept.size
            assert np.array_equal(mine[:k], kept)                        # ...before the overflow
            cnt = int((own == r).sum())
            assert k == min(cnt, off[r + 1] - off[r])                    # an owner keeps up to its cap
