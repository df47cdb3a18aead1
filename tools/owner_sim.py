"""Student rows per rank under owner rules for the 8-rank collab step (CPU, oracle sampler on the
synthetic collab graph, ownership by the locality order as DistillEngine uses it).  Answers the
round-4 verdict's "two-choice endpoint ownership" ask with numbers:

  * how local the context pairs are: the fraction of (anchor, context) pairs, walk contexts and
    negative contexts separately, whose two ends share an owner;
  * rows per rank with context pairs keyed by the context (the shipped rule) or by the anchor;
  * rows per rank when the label pairs may also go to the owner of their OTHER end whenever that
    end is already resident there (two-choice; balance ignored, so an upper bound on the gain).

    python tools/owner_sim.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import llp_data  # noqa: E402
import llp_sage  # noqa: E402
from oracle import llp_oracle as O  # noqa: E402


def main(R=8):
    data = llp_data.synthetic_collab(seed=0, with_eval=False)
    N = data.N
    ei = data.edge_index.numpy()
    rowptr, col = O.build_rowptr(ei[0], ei[1], N)
    P, B = 65_536, 13_110
    rng = np.random.default_rng(2)
    anchors = rng.permutation(N)[:B]
    links = rng.permutation(data.train_pairs.shape[0])[:P]
    pos_s, neg_s = O.neighbor_samplers(rowptr, col, anchors, N, 3, "nb", 3, 3, seed=123, stream_base=0)
    samples = np.concatenate([pos_s, neg_s], 1)
    C = samples.shape[1] - 1
    n_walk = pos_s.shape[1] - 1
    neg = O.randint_edges(N, P, seed=123, stream=O.RANDINT_STREAM)
    pos = data.train_pairs.numpy()[links].T
    _, pi = llp_sage.locality_order(ei, N)
    tab = (pi * R) // N
    a = np.repeat(samples[:, 0], C)
    c = samples[:, 1:].reshape(-1)
    walk = np.tile(np.arange(C) < n_walk, B)
    print(f"same-owner fraction: walk contexts {np.mean(tab[a[walk]] == tab[c[walk]]):.3f}, negative contexts "
          f"{np.mean(tab[a[~walk]] == tab[c[~walk]]):.3f}, positive label pairs {np.mean(tab[pos[0]] == tab[pos[1]]):.3f}, "
          f"negative label pairs {np.mean(tab[neg[0]] == tab[neg[1]]):.3f} (1/R = {1 / R:.3f})")

    def rows(oc, op, on):
        res = np.zeros((R, N), bool)
        res[oc, a] = True
        res[oc, c] = True
        res[op, pos[0]] = True
        res[op, pos[1]] = True
        res[on, neg[0]] = True
        res[on, neg[1]] = True
        return res.sum(1)

    shipped = rows(tab[c], tab[pos[0]], tab[neg[0]])
    by_anchor = rows(tab[a], tab[pos[0]], tab[neg[0]])
    # two-choice for the label pairs: the owner of either end, whichever has the other end resident
    res = np.zeros((R, N), bool)
    res[tab[c], a] = True
    res[tab[c], c] = True
    o0, o1 = tab[pos[0]], tab[pos[1]]
    chp = np.where(res[o0, pos[1]] | (o0 == o1), o0, np.where(res[o1, pos[0]], o1, o0))
    res[chp, pos[0]] = True
    res[chp, pos[1]] = True
    u, v = neg
    chn = np.where(res[tab[u], v], tab[u], np.where(res[tab[v], u], tab[v], tab[u]))
    two = rows(tab[c], chp, chn)
    anchors_per_rank = np.mean([np.unique(a[tab[c] == r]).size for r in range(R)])
    print(f"R={R}: student rows per rank, mean (max): contexts by context owner {shipped.mean():.0f} ({shipped.max()}), "
          f"by anchor owner {by_anchor.mean():.0f} ({by_anchor.max()}), two-choice label pairs {two.mean():.0f} "
          f"({two.max()}); anchors present per rank {anchors_per_rank:.0f} of {B}")


if __name__ == "__main__":
    main()
