"""a look-back timeout recorded on ONE rank must make EVERY rank raise and
reset at end_epoch, instead of only the failing rank (the others would carry on into the next
epoch's collectives and hang).  EngineBase.end_epoch all-reduces the error flag in the same
buffer as the epoch's loss sum.  Checked on CPU over 2 and 3 gloo ranks with the engine's own
end_epoch / check_device_errors / reset_device_state on a stand-in workspace (no device
kernels run: the error word is a tensor the test sets, as a timed-out scan would)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Ws:
    """Stand-in for a dedup / dense-negative workspace: its control block's error word."""

    def __init__(self, bad):
        self.buf = torch.tensor([7 if bad else 0], dtype=torch.int32)

    def error_word(self):
        return self.buf[0]

    def reset(self):
        self.buf.zero_()


def _engine(rank, world, bad):
    import llp_engine
    e = llp_engine.EngineBase.__new__(llp_engine.EngineBase)
    e.dev = torch.device("cpu")
    e.world, e.rank, e.group = world, rank, None
    e.loss_sum = torch.tensor([1.5 * (rank + 1)], dtype=torch.float64)
    e.loss_ticket = torch.ones(8, dtype=torch.int32)
    e.sumsq_ticket = torch.ones(8, dtype=torch.int32)
    e._dedup_wss = {"mb": _Ws(bad)}
    e._neg_wss = {}
    e.adam_step = torch.tensor([3], dtype=torch.int64)
    e.all_params = []
    e.optimizer = None
    return e


def _worker(rank, world, port, bad_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    e = _engine(rank, world, rank == bad_rank)
    out = {}
    try:
        out["loss"] = e.end_epoch(10)
        out["raised"] = False
    except RuntimeError as ex:
        out["raised"] = "look-back" in str(ex)
    out["reset"] = int(e.loss_ticket.abs().sum()) == 0 and int(e._dedup_wss["mb"].error_word()) == 0
    # after the reset the next epoch ends normally on every rank (the collectives stay matched)
    out["next"] = e.end_epoch(10)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bad_rank", [(2, 1), (3, 0), (3, -1)])
def test_end_epoch_error_flag_is_collective(world, bad_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bad_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = sum(1.5 * (r + 1) for r in range(world)) / 10
    for r in range(world):
        o = res[r]
        assert o["raised"] == (bad_rank >= 0), (r, o)
        if bad_rank < 0:
            assert abs(o["loss"] - total) < 1e-12
        else:
            assert o["reset"], (r, o)
        assert abs(o["next"] - total) < 1e-12
