"""dedup_rows at the collab sizes (R = 747,214 rows and the 8-rank shard's 93,4xx) on
collab-like targets, 20 calls each: run under rocprofv3 --kernel-trace to time the passes;
prints a checksum of the outputs (two environments must agree)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402

dev = "cuda"
N = 235_868
g = torch.Generator(device=dev)
g.manual_seed(0)
for R in (747_214, 93_402):
    target = torch.randint(0, N, (R,), device=dev, dtype=torch.int32, generator=g)
    target[: R // 4] = torch.randint(0, 2000, (R // 4,), device=dev, dtype=torch.int32, generator=g)   # repeats
    uniq = torch.empty(R, dtype=torch.int32, device=dev)
    pos = torch.empty(R, dtype=torch.int32, device=dev)
    nu = torch.empty(1, dtype=torch.int32, device=dev)
    segp = torch.empty(R + 1, dtype=torch.int32, device=dev)
    segr = torch.empty(R, dtype=torch.int32, device=dev)
    ws = torch.empty(K.dedup_ws_bytes(N, R) // 4 + 16, device=dev)
    for _ in range(20):
        K.dedup_rows(N, R, target, uniq, pos, nu, segp, segr, ws)
    torch.cuda.synchronize()
    U = int(nu.item())
    cs = [int(t[:n].to(torch.int64).mul(torch.arange(n, device=dev) % 9973 + 1).sum().item())
          for t, n in ((uniq, U), (pos, R), (segp, U + 1), (segr, R))]
    print(R, U, cs, flush=True)
