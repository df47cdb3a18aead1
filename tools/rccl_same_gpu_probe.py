"""Probe: can two ranks share one GPU over the nccl (= RCCL) backend on this box?

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/rccl_same_gpu_probe.py

Each rank puts a tensor on cuda:0 and runs an all_reduce, a reduce_scatter_tensor and an
all_gather_into_tensor; rank 0 prints one JSON line with the results (or the error).  RCCL may
refuse duplicate devices; the answer decides whether the multi-rank GPU tests can run their
RCCL path on a one-GPU box.
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    out = {"world": world}
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        t = torch.full((4,), float(rank + 1), device="cuda:0")
        dist.all_reduce(t)
        out["all_reduce"] = t.tolist()
        full = torch.arange(4 * world, dtype=torch.float32, device="cuda:0") * (rank + 1)
        part = torch.empty(4, device="cuda:0")
        dist.reduce_scatter_tensor(part, full)
        out["reduce_scatter"] = part.tolist()
        g = torch.empty(4 * world, device="cuda:0")
        dist.all_gather_into_tensor(g, torch.full((4,), float(rank), device="cuda:0"))
        out["all_gather"] = g.tolist()
        torch.cuda.synchronize()
        out["ok"] = True
    except Exception as e:   # the probe's answer, not a failure of the probe
        out["ok"] = False
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
