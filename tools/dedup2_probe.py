"""llp_dedup_rows2 in isolation, 20 calls per case, for rocprofv3 --kernel-trace:
  physics   N = 31,044 nodes, R = 206k endpoint rows (rank 0 of 4's Hadamard backward grouping),
            with and without the absent-node zero fill of an f32 [N, 256] row buffer
  collab    N = 235,868, R = 93,402 (the 8-rank shard's unique-node student)
Cases run in that order, each preceded by a marker launch of llp_zero on 4 bytes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev)
g.manual_seed(0)
marker = torch.zeros(1, device=dev)
for name, N, R, zfill in (("physics", 31_044, 206_000, True), ("physics-nofill", 31_044, 206_000, False),
                          ("collab", 235_868, 93_402, False)):
    target = torch.randint(0, N, (R,), device=dev, dtype=torch.int32, generator=g)
    uniq = torch.empty(R, dtype=torch.int32, device=dev)
    pos = torch.empty(R, dtype=torch.int32, device=dev)
    nu = torch.empty(1, dtype=torch.int32, device=dev)
    segp = torch.empty(R + 1, dtype=torch.int32, device=dev)
    segr = torch.empty(R, dtype=torch.int32, device=dev)
    out = torch.empty(N, 256, device=dev) if zfill else None
    ws = K.DedupWorkspace(N, R, dev)
    K.zero_(marker)
    for _ in range(20):
        K.dedup_rows2(N, R, target, uniq, pos, nu, segp, segr, ws, zero_rows=out)
    torch.cuda.synchronize()
    print(name, "unique", int(nu.item()), "error", int(ws.error_word().item()), flush=True)
