"""Synthetic datasets with the shapes of the reference's benchmarks (no
downloads: PygLinkPropPredDataset / Planetoid fetch from the network,
src/main.py:307, src/utils.py:47-48).

ogbl-collab shape: N=235,868 nodes, F=128 features,
1,179,052 undirected training pairs written OGB-style as interleaved
(u,v),(v,u) (E=2,358,104 directed edges: row NOT sorted) with ~5 %
duplicated pairs (multi-edges, Q2); valid/test positives + 100,000 uniform
negatives each.  Planted-partition graph: 1,000 communities, 90 % intra.
"""
from __future__ import annotations

import types

import numpy as np
import torch

COLLAB = dict(N=235_868, F=128, E_train=1_179_052, n_valid=60_084, n_test=46_329, n_neg=100_000)


def planted_pairs(N: int, n_pairs: int, n_comm: int, p_intra: float, dup_frac: float, rng, comm=None):
    """Undirected pairs, a fraction p_intra inside the planted community of u.
    ``comm`` (node -> community) is drawn when not given."""
    if comm is None:
        comm = rng.integers(0, n_comm, N)
    members = [np.flatnonzero(comm == c) for c in range(n_comm)]
    n_dup = int(n_pairs * dup_frac)
    n_base = n_pairs - n_dup
    u = rng.integers(0, N, n_base)
    intra = rng.random(n_base) < p_intra
    v = rng.integers(0, N, n_base)
    cu = comm[u[intra]]
    # a random member of u's community
    sizes = np.array([m.size for m in members])
    offs = (rng.random(cu.size) * sizes[cu]).astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    flat = np.concatenate(members)
    v[intra] = flat[starts[cu] + offs]
    same = u == v
    v[same] = (v[same] + 1) % N
    pairs = np.stack([u, v], 1)
    dup = pairs[rng.integers(0, n_base, n_dup)]
    pairs = np.concatenate([pairs, dup], 0)
    pairs = pairs[rng.permutation(pairs.shape[0])]
    planted_pairs.last_comm = comm
    return pairs


def interleave(pairs: np.ndarray) -> np.ndarray:
    """OGB add_inverse_edge layout: columns (u0,v0),(v0,u0),(u1,v1),..."""
    return np.stack([pairs, pairs[:, ::-1]], 1).reshape(-1, 2).T.copy()


def synthetic_collab(seed: int = 0, scale: float = 1.0, with_eval: bool = True, F: int = None, n_comm: int = None):
    """Returns a namespace with x (f32 [N,F]), edge_index (int64 [2,E]),
    train pairs (int64 [E_train,2]) and split_edge-style valid/test dicts.
    n_comm: planted communities (default 1,000 x scale, at least 10)."""
    rng = np.random.default_rng(seed)
    N = int(COLLAB["N"] * scale)
    Fd = COLLAB["F"] if F is None else F
    E = int(COLLAB["E_train"] * scale)
    n_comm = max(10, int(1000 * scale)) if n_comm is None else int(n_comm)
    pairs = planted_pairs(N, E, n_comm, 0.9, 0.05, rng)
    comm = planted_pairs.last_comm
    # features carry the planted community (centroid + noise), so the student
    # MLP can learn the link structure from x as it does from real features
    cent = rng.standard_normal((n_comm, Fd), dtype=np.float32)
    x = (0.07 * (cent[comm] + rng.standard_normal((N, Fd), dtype=np.float32))).astype(np.float32)
    d = types.SimpleNamespace(N=N, F=Fd, x=torch.from_numpy(x), train_pairs=torch.from_numpy(pairs),
                              edge_index=torch.from_numpy(interleave(pairs)))
    if with_eval:
        nv, nt, nn_ = (int(COLLAB[k] * scale) for k in ("n_valid", "n_test", "n_neg"))
        # held-out positives from the SAME planted communities as the training graph
        held = planted_pairs(N, nv + nt, n_comm, 0.9, 0.0, rng, comm=comm)
        d.split_edge = {
            "train": {"edge": d.train_pairs},
            "valid": {"edge": torch.from_numpy(held[:nv]),
                      "edge_neg": torch.from_numpy(rng.integers(0, N, (nn_, 2)))},
            "test": {"edge": torch.from_numpy(held[nv:]),
                     "edge_neg": torch.from_numpy(rng.integers(0, N, (nn_, 2)))},
        }
    return d
