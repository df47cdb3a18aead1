"""The data-parallel decomposition the engines implement, checked
on CPU with the oracle over 2, 3 and 8 gloo ranks: each rank takes a contiguous slice of
the anchors (`node_perm`) and of the positive / negative label edges, weights
its loss terms by global normalisers (KL and margin-rank by B_shard / B_total,
BCE by 2 P_shard / 2 P_total), and a SUM all-reduce of the gradients equals the
whole-batch gradient of `train_minibatch`'s loss (src/main.py:86-132).  The
oracle is the checker here; the GPU engines' own 2-rank runs are in
test_gpu_multirank.py."""
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
    edge = torch.randint(0, N, (2, P), generator=g)
    neg = torch.randint(0, N, (2, P), generator=g)
    shapes_s = [(H, F_), (H, H)]
    shapes_p = [(H, H), (1, H)]
    shapes_t = [(T, T), (1, T)]
    mk = lambda shp: [torch.randn(*s, generator=g, dtype=torch.float64) * 0.3 for s in shp]
    mkb = lambda shp: [torch.randn(s[0], generator=g, dtype=torch.float64) * 0.1 for s in shp]
    params = (mk(shapes_s), mkb(shapes_s), mk(shapes_p), mkb(shapes_p), mk(shapes_t), mkb(shapes_t))
    args = types.SimpleNamespace(dropout=0.0, margin=0.05, predictor="mlp", True_label=0.5, LLP_D=1.0, LLP_R=1.0)
    return x, t_h, samples, edge, neg, params, args


def _grads(rank, world):
    import sys
    sys.path.insert(0, REPO)
    from oracle import llp_oracle as O
    torch.set_default_dtype(torch.float64)     # the oracle's BCE labels follow the default dtype
    x, t_h, samples, edge, neg, (sw, sb, pw, pb, tw, tb), args = _problem()
    B, P = samples.shape[0], edge.shape[1]
    b0, b1 = rank * B // world, (rank + 1) * B // world
    p0, p1 = rank * P // world, (rank + 1) * P // world
    leaves = [t.clone().requires_grad_() for t in sw + sb + pw + pb]
    ns, npd = len(sw), len(pw)
    lw, lb = leaves[:ns], leaves[ns:2 * ns]
    lpw, lpb = leaves[2 * ns:2 * ns + npd], leaves[2 * ns + npd:]
    r = O.distill_losses_minibatch(x, t_h, samples[b0:b1], edge[:, p0:p1], neg[:, p0:p1], lw, lb, lpw, lpb, tw, tb,
                                   args)
    fb, fp = (b1 - b0) / B, (p1 - p0) / P
    loss = args.True_label * r["label_loss"] * fp + (args.LLP_D * r["llp_d"] + args.LLP_R * r["llp_r"]) * fb
    grads = torch.autograd.grad(loss, leaves)
    return [g.detach() for g in grads], float(loss)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grads, loss = _grads(rank, world)
    flat = torch.cat([g.reshape(-1) for g in grads])
    tot = torch.tensor([loss], dtype=torch.float64)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put((flat.numpy().copy(), float(tot.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_rank_shards_sum_to_the_batch_gradient(world):
    """2 ranks, 3 (uneven slices of the 40 label edges) and 8 (the driver's largest
    data-parallel run: 3 anchors and 5 label edges per rank)."""
    old = torch.get_default_dtype()
    try:
        full, full_loss = _grads(0, 1)
    finally:
        torch.set_default_dtype(old)
    full = torch.cat([g.reshape(-1) for g in full]).numpy()
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
