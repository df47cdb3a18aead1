"""dedup_rows on the real collab step's target rows (rank 0's shard of an R-rank job:
--ranks 1 or 8), 20 calls, under rocprofv3 --kernel-trace; also prints the largest
per-node multiplicities (atomic contention) of that target array."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import llp_data  # noqa: E402
import llp_engine  # noqa: E402
import llp_hip as K  # noqa: E402
import models  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
opt = ap.parse_args()
dev = torch.device("cuda", 0)
a = bench.collab_args()
data = llp_data.synthetic_collab(seed=0, with_eval=False)
N, F, H, L = data.N, data.F, a.hidden_channels, a.num_layers
E_train = data.train_pairs.shape[0]
P_full = a.link_batch_size
B_full = int(N / (E_train / P_full))
torch.manual_seed(1)
model = models.MLP(L, F, H, H, a.dropout).to(dev)
pred = models.LinkPredictor("mlp", H, H, 1, L, a.dropout).to(dev)
tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, a.dropout).to(dev)
t_h = torch.randn(N, 256) * 0.3
optim = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(dev), t_h.to(dev), data.edge_index[0].numpy(),
                               data.edge_index[1].numpy(), N, a, optim, dtype="bf16", seed=123)
pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
g = torch.Generator(device=dev)
g.manual_seed(2)
link_perm = torch.randperm(E_train, generator=g, device=dev).to(torch.int32)
node_perm = torch.randperm(N, generator=g, device=dev).to(torch.int32)
b1, p1 = B_full // opt.ranks, P_full // opt.ranks
eng.step_minibatch(node_perm[:b1], link_perm[:p1], pairs, b_offset=0, p_offset=0, B_total=B_full, P_total=P_full)
torch.cuda.synchronize()
target = eng._bufs["target"].clone()
R = target.numel()
cnt = torch.bincount(target.long(), minlength=N)
top = torch.topk(cnt, 10).values.tolist()
print(f"ranks {opt.ranks}: R {R}, unique {int((cnt > 0).sum())}, top multiplicities {top}", flush=True)
uniq = torch.empty(R, dtype=torch.int32, device=dev)
pos = torch.empty(R, dtype=torch.int32, device=dev)
nu = torch.empty(1, dtype=torch.int32, device=dev)
segp = torch.empty(R + 1, dtype=torch.int32, device=dev)
segr = torch.empty(R, dtype=torch.int32, device=dev)
ws = torch.empty(K.dedup_ws_bytes(N, R) // 4 + 16, device=dev)
for _ in range(20):
    K.dedup_rows(N, R, target, uniq, pos, nu, segp, segr, ws)
torch.cuda.synchronize()
