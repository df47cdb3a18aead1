"""How the unique-node student's work grows with the rank count (CPU, oracle sampler
on the synthetic collab graph, one global batch): rows and unique nodes per rank's
shard, the global unique count, and for an owner-computes split (every unique node's
student rows computed on one rank, h rows exchanged) the rows each rank would fetch.

    python tools/rank_overlap.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import llp_data  # noqa: E402
from oracle import llp_oracle as O  # noqa: E402

data = llp_data.synthetic_collab(seed=0, with_eval=False)
N = data.N
ei = data.edge_index.numpy()
rowptr, col = O.build_rowptr(ei[0], ei[1], N)
E_train = data.train_pairs.shape[0]
P, B = 65_536, int(N / (E_train / 65_536))
rng = np.random.default_rng(2)
anchors = rng.permutation(N)[:B]
links = rng.permutation(E_train)[:P]
pairs = data.train_pairs.numpy()
pos_s, neg_s = O.neighbor_samplers(rowptr, col, anchors, N, 3, "nb", 3, 3, seed=123, stream_base=0)
samples = np.concatenate([pos_s, neg_s], 1)                                                        # [B, 1 + 36]
neg = O.randint_edges(N, P, seed=123, stream=O.RANDINT_STREAM)                                                   # [2, P]


def target_rows(b0, b1, p0, p1):
    """student rows of one shard: samples.flat | src | dst (src/main.py:95)"""
    s = samples[b0:b1].reshape(-1)
    pos = pairs[links[p0:p1]]
    src = np.concatenate([pos[:, 0], neg[0, p0:p1]])
    dst = np.concatenate([pos[:, 1], neg[1, p0:p1]])
    return np.concatenate([s, src, dst])


glob = np.unique(target_rows(0, B, 0, P))
print(f"B={B} P={P}: rows {B * 37 + 4 * P}, global unique nodes {glob.size}")
for R in (1, 2, 4, 8):
    per, fetch = [], []
    owner = np.empty(N, dtype=np.int64)
    owner[glob] = np.arange(glob.size) * R // glob.size   # contiguous slot ranges of the global unique list
    for r in range(R):
        t = np.unique(target_rows(r * B // R, (r + 1) * B // R, r * P // R, (r + 1) * P // R))
        per.append(t.size)
        fetch.append(int((owner[t] != r).sum()))
    print(f"R={R}: unique per rank {np.mean(per):9.0f} (max {max(per)}), sum over ranks {sum(per):8d} "
          f"= {sum(per) / glob.size:.2f}x global; owner-computes: {glob.size / R:8.0f} rows per rank, "
          f"remote h rows fetched per rank {np.mean(fetch):8.0f} ({np.mean(fetch) * 2048 / 1e6:.0f} MB bf16 H=1024)")

# the owner decomposition (DistillEngine owner mode): context pairs to the owner of the context
# node, label pairs to the owner of their source (balanced, O.pair_owner_assign), anchors where
# their pairs are; the student runs on the unique endpoints of the rank's pairs
C = samples.shape[1] - 1
pos_all = pairs[links].T
print("owner decomposition (student rows = unique endpoints of the rank's pairs):")
for R in (2, 4, 8):
    per = []
    for r in range(R):
        cs, ps, ns = O.pair_owner_rank_items(samples, pos_all, neg, N, R, r)
        b, c = cs // C, cs % C
        ends = np.concatenate([samples[b, 0], samples[b, 1 + c], pos_all[0, ps], pos_all[1, ps], neg[0, ns],
                               neg[1, ns]])
        per.append(np.unique(ends).size)
    print(f"R={R}: unique per rank {np.mean(per):9.0f} (max {max(per)}, min {min(per)}); "
          f"pairs per rank {(B * C + 2 * P) / R:9.0f}")

# the same with node ownership by a locality order (DistillEngine owner_locality: label propagation)
import llp_sage  # noqa: E402
_, pi = llp_sage.locality_order(ei, N)
print("owner decomposition, ownership by the locality order:")
for R in (2, 4, 8):
    tab = (pi * R) // N
    per = []
    for r in range(R):
        cs, ps, ns = O.pair_owner_rank_items(samples, pos_all, neg, N, R, r, owner_tab=tab)
        b, c = cs // C, cs % C
        ends = np.concatenate([samples[b, 0], samples[b, 1 + c], pos_all[0, ps], pos_all[1, ps], neg[0, ns],
                               neg[1, ns]])
        per.append(np.unique(ends).size)
    print(f"R={R}: unique per rank {np.mean(per):9.0f} (max {max(per)}, min {min(per)})")
