"""Offline dataset access for the CLI drop-ins (main.py, train_teacher_gnn.py).

The reference downloads its graphs (PygLinkPropPredDataset / Planetoid /
Coauthor / Amazon, src/main.py:307, src/utils.py:31-53) and caches the SEAL
edge split as ``../data/<ds>.pkl`` (src/main.py:298-303).  No network here, so:

  1. ``<dataset_dir>/<ds>.pt`` — a torch.save'd dict {'x': f32 [N,F],
     'split_edge': {'train': {'edge'}, 'valid': {'edge','edge_neg'}, 'test': ...},
     optional 'edge_index': int64 [2,E] (collab's message-passing graph)},
     loaded with ``weights_only=True``; or
  2. ``--synthetic``: a seeded graph with the dataset's published shape
     (nodes, feature width, undirected edges), planted communities, features
     that carry the community, and the SEAL split ratios the reference uses
     (val 0.05 / test 0.10 of the undirected edges, src/utils.py:59-105;
     collab: llp_data.synthetic_collab).

``data.adj_t`` follows the reference: the training edges ``[2, E_train]`` (one
direction) for non-collab datasets (src/main.py:305-306), the full directed
``edge_index`` for collab (src/main.py:316).
"""
from __future__ import annotations

import os
import types

import numpy as np
import torch

import llp_data

# name: (nodes, features, undirected edges, communities, binary bag-of-words features)
SHAPES = {
    "cora": (2708, 1433, 5278, 7, True),
    "citeseer": (3327, 3703, 4552, 6, True),
    "pubmed": (19717, 500, 44324, 3, False),
    "coauthor-cs": (18333, 6805, 81894, 15, True),
    "coauthor-physics": (34493, 8415, 247962, 5, True),
    "amazon-computers": (13752, 767, 245861, 10, True),
    "amazon-photos": (7650, 745, 119081, 8, True),
}


def _sample_non_edges(N, n, edge_set, rng):
    out = []
    while len(out) < n:
        u = rng.integers(0, N, 2 * n)
        v = rng.integers(0, N, 2 * n)
        for a, b in zip(u.tolist(), v.tolist()):
            if a != b and (a, b) not in edge_set and (b, a) not in edge_set:
                out.append((a, b))
                if len(out) == n:
                    break
    return torch.tensor(out, dtype=torch.int64)


def synthetic_transductive(name: str, seed: int = 0):
    """(data, split_edge) with the shape of ``name``."""
    if name == "collab":
        d = llp_data.synthetic_collab(seed=seed)
        data = types.SimpleNamespace(x=d.x, edge_index=d.edge_index, adj_t=d.edge_index, num_nodes=d.N)
        return data, d.split_edge
    if name not in SHAPES:
        raise ValueError(f"unknown dataset {name!r}; known: collab, {', '.join(SHAPES)}")
    N, F, E, n_comm, binary = SHAPES[name]
    rng = np.random.default_rng(seed)
    pairs = llp_data.planted_pairs(N, E, n_comm, 0.85, 0.0, rng)
    comm = llp_data.planted_pairs.last_comm
    pairs = np.unique(np.sort(pairs, 1), axis=0)            # simple undirected graph
    pairs = pairs[rng.permutation(pairs.shape[0])]
    if binary:   # bag-of-words: a community vocabulary + background words
        p = np.full((n_comm, F), 0.002, np.float32)
        for c in range(n_comm):
            p[c, rng.choice(F, max(1, F // (2 * n_comm)), replace=False)] = 0.03
        x = (rng.random((N, F), dtype=np.float32) < p[comm]).astype(np.float32)
    else:
        cent = rng.standard_normal((n_comm, F), dtype=np.float32)
        x = (0.1 * (cent[comm] + rng.standard_normal((N, F), dtype=np.float32))).astype(np.float32)
    n_v = int(np.floor(0.05 * pairs.shape[0]))
    n_t = int(np.floor(0.10 * pairs.shape[0]))
    valid, test, train = pairs[:n_v], pairs[n_v:n_v + n_t], pairs[n_v + n_t:]
    es = set(map(tuple, pairs.tolist()))
    split_edge = {
        "train": {"edge": torch.from_numpy(train)},
        "valid": {"edge": torch.from_numpy(valid), "edge_neg": _sample_non_edges(N, n_v, es, rng)},
        "test": {"edge": torch.from_numpy(test), "edge_neg": _sample_non_edges(N, n_t, es, rng)},
    }
    full = np.concatenate([pairs, pairs[:, ::-1]], 0).T.copy()
    data = types.SimpleNamespace(x=torch.from_numpy(x), edge_index=torch.from_numpy(full),
                                 adj_t=split_edge["train"]["edge"].t().contiguous(), num_nodes=N)
    return data, split_edge


def _coalesce(edge_index: torch.Tensor, N: int) -> torch.Tensor:
    """Sorted by (row, col), duplicates removed — the layout PyG datasets ship."""
    key = torch.unique(edge_index[0].long() * N + edge_index[1].long())
    return torch.stack([key // N, key % N], 0)


def load_graph(name: str, dataset_dir: str, synthetic: bool, seed: int = 0):
    """The whole graph (``get_dataset(...)[0]`` of src/utils.py:31-53) as a
    llp_split.GraphData(x, edge_index) with both directions of every edge —
    the input of the production split.  From ``<dataset_dir>/<ds>.pt``
    ('edge_index', else train+valid+test edges) or ``--synthetic``."""
    import llp_split
    path = os.path.join(dataset_dir, name + ".pt")
    if os.path.exists(path):
        b = torch.load(path, weights_only=True)
        x = b["x"].float()
        if "edge_index" in b:
            ei = b["edge_index"].long()
        else:
            se = b["split_edge"]
            und = torch.cat([se[s]["edge"] for s in ("train", "valid", "test")], 0).long().t()
            ei = torch.cat([und, und.flip([0])], -1)
    elif synthetic:
        data, _ = synthetic_transductive(name, seed)
        x, ei = data.x, data.edge_index.long()
    else:
        raise FileNotFoundError(f"{path} not found (or pass --synthetic)")
    return llp_split.GraphData(x, _coalesce(ei, x.size(0)))


def load_transductive(name: str, dataset_dir: str, synthetic: bool, seed: int = 0):
    path = os.path.join(dataset_dir, name + ".pt")
    if os.path.exists(path):
        b = torch.load(path, weights_only=True)
        split_edge = b["split_edge"]
        x = b["x"].float()
        if name == "collab" and "edge_index" in b:
            ei = b["edge_index"]
        else:
            ei = split_edge["train"]["edge"].t().contiguous()
        data = types.SimpleNamespace(x=x, edge_index=b.get("edge_index", ei), adj_t=ei, num_nodes=x.size(0))
        return data, split_edge
    if synthetic:
        return synthetic_transductive(name, seed)
    raise FileNotFoundError(
        f"{path} not found: save {{'x', 'split_edge'[, 'edge_index']}} there with torch.save, or pass "
        f"--synthetic for a seeded graph of the {name} shape (no network: the reference's downloaders cannot run)")
