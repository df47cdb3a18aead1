"""Offline dataset access for the CLI drop-ins (main.py, train_teacher_gnn.py).

The reference downloads its graphs (PygLinkPropPredDataset / Planetoid /
Coauthor / Amazon, src/main.py:307, src/utils.py:30-50) and caches the SEAL
edge split of non-collab datasets as ``../data/<ds>.pkl`` (src/main.py:292-301,
src/train_teacher_gnn.py:306-315).  There is no network here; a graph comes
from, in order:

  1. ``<dataset_dir>/<ds>.pt`` — a torch.save'd dict {'x': f32 [N,F],
     'split_edge': {'train': {'edge'}, 'valid': {'edge','edge_neg'}, 'test': ...},
     optional 'edge_index': int64 [2,E]} (``weights_only=True``);
  2. the raw files the reference's loaders download, read without unpickling:
       coauthor-cs / coauthor-physics  <dataset_dir>/{CS,Physics}/raw/ms_academic_{cs,phy}.npz
       amazon-computers / -photos      <dataset_dir>/{Computers,Photo}/raw/amazon_electronics_*.npz
       collab                          {dataset,<dataset_dir>}/ogbl_collab/raw/{edge,node-feat}.csv.gz
                                       + split/time/{train,valid,test}.pt
     (Planetoid's raw files are Python pickles of scipy objects: not read —
     use form 1 for cora / citeseer / pubmed);
  3. ``--synthetic``: a seeded graph with the dataset's published shape
     (nodes, feature width, undirected edges), planted communities and
     features that carry them (collab: llp_data.synthetic_collab).

The transductive split of a non-collab graph is the reference's own:
``../data/<ds>.pkl`` when it exists (a dict of tensors: read with
``weights_only=True``), else llp_split.do_edge_split (src/utils.py:62-105,
same random streams) written back to that path in the same format.
Synthetic graphs cache their split as ``<dataset_dir>/<ds>_synthetic_split.pt``
so they never overwrite a real dataset's cache.

``data.adj_t`` follows the reference: the training edges ``[2, E_train]`` for
non-collab datasets (both directions, as train_test_split_edges returns them,
src/main.py:305-306), the full directed ``edge_index`` for collab
(src/main.py:316).
"""
from __future__ import annotations

import os
import types

import numpy as np
import torch

import llp_data
import llp_split

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

# PyG Coauthor / Amazon raw layout: dataset dir -> file
NPZ_FILES = {
    "coauthor-cs": ("CS", "ms_academic_cs.npz"),
    "coauthor-physics": ("Physics", "ms_academic_phy.npz"),
    "amazon-computers": ("Computers", "amazon_electronics_computers.npz"),
    "amazon-photos": ("Photo", "amazon_electronics_photo.npz"),
}


def _safe_load(path):
    """torch.load with weights_only=True; numpy arrays (OGB's split files hold
    them) are admitted through the array-reconstruction allowlist only."""
    allow = [np.ndarray, np.dtype]
    rec = getattr(getattr(np, "_core", np.core), "multiarray")._reconstruct
    allow.append(rec)
    allow += [getattr(np.dtypes, n) for n in dir(np.dtypes) if n.endswith("DType")]
    with torch.serialization.safe_globals(allow):
        return torch.load(path, weights_only=True, map_location="cpu")


def _as_tensor(v):
    return torch.from_numpy(v) if isinstance(v, np.ndarray) else v


# ----------------------------------------------------------------------------- raw readers

def read_npz_graph(path: str) -> llp_split.GraphData:
    """torch_geometric.io.read_npz (PyG 2.2.0): binarised CSR attributes, the
    adjacency without self-loops, made undirected and coalesced."""
    import scipy.sparse as sp
    with np.load(path, allow_pickle=False) as f:
        x = sp.csr_matrix((f["attr_data"], f["attr_indices"], f["attr_indptr"]), tuple(f["attr_shape"])).todense()
        adj = sp.csr_matrix((f["adj_data"], f["adj_indices"], f["adj_indptr"]), tuple(f["adj_shape"])).tocoo()
    x = torch.from_numpy(np.asarray(x)).to(torch.float)
    x[x > 0] = 1
    ei = torch.stack([torch.from_numpy(adj.row).long(), torch.from_numpy(adj.col).long()])
    ei = ei[:, ei[0] != ei[1]]
    return llp_split.GraphData(x, llp_split.to_undirected(ei, x.size(0)))


def _ogb_collab_dir(dataset_dir: str):
    for root in ("dataset", dataset_dir):     # PygLinkPropPredDataset's default root is ./dataset
        d = os.path.join(root, "ogbl_collab")
        if os.path.exists(os.path.join(d, "raw", "edge.csv.gz")):
            return d
    return None


def read_ogb_collab(d: str):
    """ogbl-collab from its raw CSVs (OGB read_csv_graph_raw, add_inverse_edge:
    interleaved (u,v),(v,u)) and split/time/*.pt (get_edge_split)."""
    import pandas as pd
    edge = pd.read_csv(os.path.join(d, "raw", "edge.csv.gz"), compression="gzip", header=None).values.T
    x = pd.read_csv(os.path.join(d, "raw", "node-feat.csv.gz"), compression="gzip", header=None).values
    x = torch.from_numpy(x.astype(np.float32))
    split_edge = {}
    for s in ("train", "valid", "test"):
        raw = _safe_load(os.path.join(d, "split", "time", s + ".pt"))
        split_edge[s] = {k: _as_tensor(v) for k, v in raw.items()}
    ei = torch.from_numpy(llp_data.interleave(edge.T.astype(np.int64)))
    return x, ei, split_edge


# ----------------------------------------------------------------------------- synthetic

def synthetic_graph(name: str, seed: int = 0) -> llp_split.GraphData:
    """A coalesced undirected graph (both directions) with the shape of ``name``."""
    if name not in SHAPES:
        raise ValueError(f"unknown dataset {name!r}; known: collab, {', '.join(SHAPES)}")
    N, F, E, n_comm, binary = SHAPES[name]
    rng = np.random.default_rng(seed)
    pairs = llp_data.planted_pairs(N, E, n_comm, 0.85, 0.0, rng)
    comm = llp_data.planted_pairs.last_comm
    if binary:   # bag-of-words: a community vocabulary + background words
        p = np.full((n_comm, F), 0.002, np.float32)
        for c in range(n_comm):
            p[c, rng.choice(F, max(1, F // (2 * n_comm)), replace=False)] = 0.03
        x = (rng.random((N, F), dtype=np.float32) < p[comm]).astype(np.float32)
    else:
        cent = rng.standard_normal((n_comm, F), dtype=np.float32)
        x = (0.1 * (cent[comm] + rng.standard_normal((N, F), dtype=np.float32))).astype(np.float32)
    ei = torch.from_numpy(pairs.T.copy())
    return llp_split.GraphData(torch.from_numpy(x), llp_split.to_undirected(ei[:, ei[0] != ei[1]], N))


def synthetic_transductive(name: str, seed: int = 0, dataset_dir: str | None = None):
    """(data, split_edge) with the shape of ``name``; non-collab graphs split
    by the reference's do_edge_split."""
    if name == "collab":
        d = llp_data.synthetic_collab(seed=seed)
        data = types.SimpleNamespace(x=d.x, edge_index=d.edge_index, adj_t=d.edge_index, num_nodes=d.N)
        return data, d.split_edge
    g = synthetic_graph(name, seed)
    cache = os.path.join(dataset_dir, f"{name}_synthetic_split.pt") if dataset_dir else None
    if cache and os.path.exists(cache):
        split_edge = torch.load(cache, weights_only=True)
    else:
        split_edge = llp_split.do_edge_split(g)
        if cache:
            os.makedirs(dataset_dir, exist_ok=True)
            torch.save(split_edge, cache)
    return _transductive_data(g.x, g.edge_index, split_edge), split_edge


# ----------------------------------------------------------------------------- public loaders

def _transductive_data(x, edge_index, split_edge):
    adj = split_edge["train"]["edge"].t().contiguous()       # src/main.py:305-306
    return types.SimpleNamespace(x=x, edge_index=edge_index, adj_t=adj, num_nodes=x.size(0))


def load_graph(name: str, dataset_dir: str, synthetic: bool, seed: int = 0) -> llp_split.GraphData:
    """The whole graph (``get_dataset(...)[0]``, src/utils.py:30-50) with both
    directions of every edge, coalesced — the input of both splits."""
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
        return llp_split.GraphData(x, llp_split.coalesce(ei, x.size(0)))
    if name in NPZ_FILES:
        sub, fname = NPZ_FILES[name]
        p = os.path.join(dataset_dir, sub, "raw", fname)
        if os.path.exists(p):
            return read_npz_graph(p)
    if synthetic:
        return synthetic_graph(name, seed)
    raise FileNotFoundError(f"{path} not found and no raw files for {name!r} under {dataset_dir} "
                            f"(or pass --synthetic; no network: the reference's downloaders cannot run)")


def load_transductive(name: str, dataset_dir: str, synthetic: bool, seed: int = 0):
    """(data, split_edge) for the transductive setting (src/main.py:290-320)."""
    path = os.path.join(dataset_dir, name + ".pt")
    if os.path.exists(path):
        b = torch.load(path, weights_only=True)
        split_edge = b["split_edge"]
        x = b["x"].float()
        if name == "collab" and "edge_index" in b:
            ei = b["edge_index"]
            return types.SimpleNamespace(x=x, edge_index=ei, adj_t=ei, num_nodes=x.size(0)), split_edge
        return _transductive_data(x, b.get("edge_index", split_edge["train"]["edge"].t()), split_edge), split_edge
    if name == "collab":
        d = _ogb_collab_dir(dataset_dir)
        if d is not None:
            x, ei, split_edge = read_ogb_collab(d)
            return types.SimpleNamespace(x=x, edge_index=ei, adj_t=ei, num_nodes=x.size(0)), split_edge
        if synthetic:
            return synthetic_transductive(name, seed)
        raise FileNotFoundError("ogbl_collab raw files not found under ./dataset or " + dataset_dir +
                                " (or pass --synthetic)")
    real = (name in NPZ_FILES and os.path.exists(os.path.join(dataset_dir, *NPZ_FILES[name][:1], "raw",
                                                              NPZ_FILES[name][1])))
    if not real:
        if synthetic:
            return synthetic_transductive(name, seed, dataset_dir)
        raise FileNotFoundError(f"{path} not found and no raw files for {name!r} (or pass --synthetic)")
    g = load_graph(name, dataset_dir, False)
    cache = "../data/" + name + ".pkl"                       # the reference's own split cache
    if os.path.exists(cache):
        split_edge = torch.load(cache, weights_only=True)
    else:
        split_edge = llp_split.do_edge_split(g)
        os.makedirs("../data", exist_ok=True)
        torch.save(split_edge, cache)
    return _transductive_data(g.x, g.edge_index, split_edge), split_edge
