"""Edge splits of the reference, restated on its own random streams:

  do_edge_split              src/utils.py:62-105 (the SEAL transductive split,
                             cached by the reference as ``../data/<ds>.pkl``,
                             src/main.py:296-301, src/train_teacher_gnn.py:310-315)
  do_production_edge_split   src/generate_production_split.py:32-95 (the
                             inductive split, cached as ``<ds>_production.pkl``,
                             src/train_teacher_gnn.py:341-365, src/main.py:338)

The reference builds the split from torch_geometric 2.2.0 pieces; those are
restated here on the SAME random streams the reference draws from, so a given
graph and seed split into the same node / edge sets:

  train_test_split_edges(data, val, test)   ``torch.randperm`` over row<col edges,
                                            train edges made undirected, negatives
                                            from a dense N x N upper-triangle mask
  negative_sampling(..., method='sparse')   Python ``random.sample`` over the
                                            edge-vector population, ``np.isin``
                                            filtering, <= 3 rounds
  RandomNodeSplit(num_val, num_test)        ``torch.randperm(N)``, 'train_rest'
  split_edges (the reference's own helper)  ``torch.randperm`` over row<=col edges
  RandomLinkSplit(num_val, num_test,        ``torch.randperm`` over row<=col edges,
                  is_undirected=True)       sparse negatives for train + test
  subgraph(mask, ei, relabel_nodes=True)    node relabelling, no RNG

This is one-off data preparation (the reference runs it on the CPU once and
caches the result), so it runs on the host with torch's CPU generator — the
only way to keep the reference's random streams; the per-step negative
sampler on the training path is the device kernel ``llp_neg_sample_dense``.

Cache format: the reference pickles PyG ``Data`` objects, which cannot be
loaded without torch_geometric (and never with a code-executing loader), so
the cache here is ``<dataset_dir>/<ds>_production.pt``: a dict of plain
tensors, read back with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import math
import os
import random

import numpy as np
import torch


class GraphData:
    """The fields of torch_geometric.data.Data the LLP path reads: ``x``,
    ``edge_index`` and, after a link split, ``edge_label`` /
    ``edge_label_index``.  ``to(device)`` moves in place and returns self,
    as PyG's ``Data.to`` does (the reference calls it without assignment,
    src/main.py:342-346)."""

    def __init__(self, x=None, edge_index=None, **fields):
        self.x = x
        self.edge_index = edge_index
        for k, v in fields.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    def to(self, device):
        for k, v in list(vars(self).items()):
            if torch.is_tensor(v):
                setattr(self, k, v.to(device))
        return self

    def tensors(self) -> dict:
        return {k: v for k, v in vars(self).items() if torch.is_tensor(v)}

    @classmethod
    def from_tensors(cls, d: dict) -> "GraphData":
        g = cls()
        for k, v in d.items():
            setattr(g, k, v)
        return g

    def __repr__(self):
        parts = [f"{k}={list(v.shape)}" for k, v in self.tensors().items()]
        return "GraphData(" + ", ".join(parts) + ")"


# --- torch_geometric.utils.negative_sampling (PyG 2.2.0, method='sparse') ---

def _edge_index_to_vector(edge_index: torch.Tensor, N: int, force_undirected: bool):
    row, col = edge_index[0], edge_index[1]
    if force_undirected:              # upper triangle only
        mask = row < col
        row, col = row[mask], col[mask]
        offset = torch.arange(1, N).cumsum(0)[row]
        return row * N + col - offset, (N * (N + 1)) // 2 - N
    mask = row != col                 # no self-loops
    row, col = row[mask], col[mask].clone()
    col[row < col] -= 1
    return row * (N - 1) + col, N * N - N


def _vector_to_edge_index(idx: torch.Tensor, N: int, force_undirected: bool) -> torch.Tensor:
    if force_undirected:
        offset = torch.arange(1, N).cumsum(0)
        end = torch.arange(N, N * N, N) - offset
        row = torch.bucketize(idx, end, right=True)
        col = (offset[row] + idx) % N
        return torch.stack([torch.cat([row, col]), torch.cat([col, row])], 0)
    row = idx.div(N - 1, rounding_mode="floor")
    col = idx % (N - 1)
    col[row <= col] += 1
    return torch.stack([row, col], 0)


def _sample(population: int, k: int) -> torch.Tensor:
    if population <= k:
        return torch.arange(population)
    return torch.tensor(random.sample(range(population), k))


def negative_sampling(edge_index: torch.Tensor, num_nodes: int, num_neg_samples: int | None = None,
                      force_undirected: bool = False) -> torch.Tensor:
    """Non-edges of ``edge_index`` (PyG's sparse method): oversample
    ``int(1.1 * n / p_negative)`` vector ids without replacement, drop existing
    edges and earlier picks, up to three rounds; may return fewer than asked.
    ``force_undirected`` samples the upper triangle and returns both
    directions of ``num_neg_samples // 2`` pairs."""
    edge_index = edge_index.cpu()
    N = int(num_nodes)
    idx, population = _edge_index_to_vector(edge_index, N, force_undirected)
    if idx.numel() >= population:
        return edge_index.new_empty((2, 0))
    if num_neg_samples is None:
        num_neg_samples = edge_index.size(1)
    if force_undirected:
        num_neg_samples = num_neg_samples // 2
    prob = 1.0 - idx.numel() / population
    sample_size = int(1.1 * num_neg_samples / prob)
    idx_np = idx.numpy()
    neg_idx = None
    for _ in range(3):
        rnd = _sample(population, sample_size)
        mask = np.isin(rnd.numpy(), idx_np)
        if neg_idx is not None:
            mask |= np.isin(rnd.numpy(), neg_idx.numpy())
        rnd = rnd[~torch.from_numpy(mask)]
        neg_idx = rnd if neg_idx is None else torch.cat([neg_idx, rnd])
        if neg_idx.numel() >= num_neg_samples:
            neg_idx = neg_idx[:num_neg_samples]
            break
    return _vector_to_edge_index(neg_idx, N, force_undirected)


# --- transductive (SEAL) split ---

def coalesce(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Sorted by (row, col), duplicates removed (torch_geometric.utils.coalesce)."""
    key = torch.unique(edge_index[0].long() * num_nodes + edge_index[1].long())
    return torch.stack([key.div(num_nodes, rounding_mode="floor"), key % num_nodes], 0)


def to_undirected(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    return coalesce(torch.cat([edge_index, edge_index.flip([0])], 1), num_nodes)


def add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    loops = torch.arange(num_nodes, dtype=edge_index.dtype).unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loops], 1)


def train_test_split_edges(edge_index: torch.Tensor, num_nodes: int, val_ratio: float = 0.05,
                           test_ratio: float = 0.1) -> dict:
    """PyG 2.2.0 train_test_split_edges: shuffled row<col edges cut into
    val / test / train (train returned in both directions, coalesced); val and
    test negatives drawn from the upper triangle minus every positive edge."""
    row, col = edge_index
    mask = row < col
    row, col = row[mask], col[mask]
    n_v = int(math.floor(val_ratio * row.size(0)))
    n_t = int(math.floor(test_ratio * row.size(0)))
    perm = torch.randperm(row.size(0))
    row, col = row[perm], col[perm]
    out = {"val_pos": torch.stack([row[:n_v], col[:n_v]]),
           "test_pos": torch.stack([row[n_v:n_v + n_t], col[n_v:n_v + n_t]]),
           "train_pos": to_undirected(torch.stack([row[n_v + n_t:], col[n_v + n_t:]]), num_nodes)}
    neg_mask = torch.ones(num_nodes, num_nodes, dtype=torch.uint8).triu(diagonal=1).to(torch.bool)
    neg_mask[row, col] = 0
    neg_row, neg_col = neg_mask.nonzero(as_tuple=False).t()
    del neg_mask
    sel = torch.randperm(neg_row.size(0))[:n_v + n_t]
    neg_row, neg_col = neg_row[sel], neg_col[sel]
    out["val_neg"] = torch.stack([neg_row[:n_v], neg_col[:n_v]])
    out["test_neg"] = torch.stack([neg_row[n_v:n_v + n_t], neg_col[n_v:n_v + n_t]])
    return out


def do_edge_split(data: GraphData, fast_split: bool = False, val_ratio: float = 0.05, test_ratio: float = 0.1,
                  split_seed: int = 234) -> dict:
    """src/utils.py:62-105 -> split_edge {'train','valid','test'} x {'edge','edge_neg'}
    with edges as [E, 2] int64 (the dict the reference torch.saves)."""
    random.seed(split_seed)
    torch.manual_seed(split_seed)
    ei = data.edge_index.cpu().long()
    N = data.num_nodes
    if not fast_split:
        s = train_test_split_edges(ei, N, val_ratio, test_ratio)
        s["train_neg"] = negative_sampling(add_self_loops(s["train_pos"], N), N,
                                           num_neg_samples=s["train_pos"].size(1))
    else:
        row, col = ei
        mask = row < col
        row, col = row[mask], col[mask]
        n_v = int(math.floor(val_ratio * row.size(0)))
        n_t = int(math.floor(test_ratio * row.size(0)))
        perm = torch.randperm(row.size(0))
        row, col = row[perm], col[perm]
        s = {"val_pos": torch.stack([row[:n_v], col[:n_v]]),
             "test_pos": torch.stack([row[n_v:n_v + n_t], col[n_v:n_v + n_t]]),
             "train_pos": torch.stack([row[n_v + n_t:], col[n_v + n_t:]])}
        neg = negative_sampling(ei, N, num_neg_samples=row.size(0))
        s["val_neg"], s["test_neg"], s["train_neg"] = neg[:, :n_v], neg[:, n_v:n_v + n_t], neg[:, n_v + n_t:]
    return {"train": {"edge": s["train_pos"].t(), "edge_neg": s["train_neg"].t()},
            "valid": {"edge": s["val_pos"].t(), "edge_neg": s["val_neg"].t()},
            "test": {"edge": s["test_pos"].t(), "edge_neg": s["test_neg"].t()}}


# --- transforms ---

def random_node_split(num_nodes: int, num_val, num_test):
    """RandomNodeSplit(split='train_rest') masks (train, val, test)."""
    nv = round(num_nodes * num_val) if isinstance(num_val, float) else int(num_val)
    nt = round(num_nodes * num_test) if isinstance(num_test, float) else int(num_test)
    train = torch.zeros(num_nodes, dtype=torch.bool)
    val = torch.zeros(num_nodes, dtype=torch.bool)
    test = torch.zeros(num_nodes, dtype=torch.bool)
    perm = torch.randperm(num_nodes)
    val[perm[:nv]] = True
    test[perm[nv:nv + nt]] = True
    train[perm[nv + nt:]] = True
    return train, val, test


def split_edges(edge_index: torch.Tensor, val_ratio: float, test_ratio: float):
    """The reference's helper (src/generate_production_split.py:14-30): shuffle
    the row<=col edges, cut (train, val, test); train and val are returned in
    both directions, test in one."""
    perm = (edge_index[0] <= edge_index[1]).nonzero(as_tuple=False).view(-1)
    perm = perm[torch.randperm(perm.size(0))]
    n_val = int(val_ratio * perm.numel())
    n_test = int(test_ratio * perm.numel())
    n_train = perm.numel() - n_val - n_test
    tr = edge_index[:, perm[:n_train]]
    va = edge_index[:, perm[n_train:n_train + n_val]]
    te = edge_index[:, perm[n_train + n_val:]]
    return torch.cat([tr, tr.flip([0])], -1), torch.cat([va, va.flip([0])], -1), te


def subgraph_relabel(node_mask: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
    """subgraph(mask, edge_index, relabel_nodes=True)[0]."""
    relabel = torch.zeros(node_mask.numel(), dtype=torch.long)
    relabel[node_mask] = torch.arange(int(node_mask.sum()))
    keep = node_mask[edge_index[0]] & node_mask[edge_index[1]]
    return relabel[edge_index[:, keep]]


def random_link_split(data: GraphData, num_val, num_test, neg_sampling_ratio: float = 1.0):
    """RandomLinkSplit(num_val, num_test, is_undirected=True) with its defaults
    (negative training samples added, ratio 1.0) -> (train, val, test)."""
    ei = data.edge_index
    perm = (ei[0] <= ei[1]).nonzero(as_tuple=False).view(-1)
    perm = perm[torch.randperm(perm.size(0))]
    nv = int(num_val * perm.numel()) if isinstance(num_val, float) else int(num_val)
    nt = int(num_test * perm.numel()) if isinstance(num_test, float) else int(num_test)
    ntr = perm.numel() - nv - nt
    if ntr <= 0:
        raise ValueError("insufficient number of edges for training")
    train_e, val_e, test_e = perm[:ntr], perm[ntr:ntr + nv], perm[ntr + nv:]
    trainval_e = perm[:ntr + nv]

    def both(index):
        e = ei[:, index]
        return torch.cat([e, e.flip([0])], -1)

    n_neg_tr = int(ntr * neg_sampling_ratio)
    n_neg_va = int(nv * neg_sampling_ratio)
    n_neg_te = int(nt * neg_sampling_ratio)
    n_neg = n_neg_tr + n_neg_va + n_neg_te
    neg = negative_sampling(ei, data.num_nodes, num_neg_samples=n_neg)
    if neg.size(1) < n_neg:        # fewer non-edges found: shrink every share alike
        ratio = neg.size(1) / n_neg
        n_neg_tr, n_neg_va, n_neg_te = int(n_neg_tr * ratio), int(n_neg_va * ratio), int(n_neg_te * ratio)

    def labelled(mp_index, index, neg_part):
        pos = ei[:, index]
        lab = torch.cat([torch.ones(index.numel()), torch.zeros(neg_part.size(1))])
        return GraphData(data.x, both(mp_index), edge_label=lab, edge_label_index=torch.cat([pos, neg_part], -1))

    train = labelled(train_e, train_e, neg[:, n_neg_va + n_neg_te:])
    val = labelled(train_e, val_e, neg[:, :n_neg_va])
    test = labelled(trainval_e, test_e, neg[:, n_neg_va:n_neg_va + n_neg_te])
    return train, val, test


def production_ratios(data_name: str):
    """(test_ratio, val_node_ratio, val_ratio, old_old_extra_ratio) of
    src/train_teacher_gnn.py:350-364: 0.3 for cora/citeseer, 0.1 otherwise."""
    r = 0.3 if data_name in ("cora", "citeseer") else 0.1
    return r, r, r, 0.1


def do_production_edge_split(data: GraphData, data_name: str, test_ratio: float, val_node_ratio: float,
                             val_ratio: float, old_old_extra_ratio: float, split_seed: int = 234):
    """src/generate_production_split.py:32-95 -> (training_data, val_data,
    inference_data, data, test_edge_bundle, negative_samples)."""
    random.seed(split_seed)
    torch.manual_seed(split_seed)
    ei = data.edge_index.cpu().long()
    x = data.x.cpu()
    N = int(x.size(0))
    # global negatives (both directions of round(test_ratio * E / 2) // 2 pairs)
    negative_samples = negative_sampling(ei, N, round(test_ratio * ei.size(1) / 2), force_undirected=True)
    # step 1: new nodes
    old, _, new = random_node_split(N, 0.0, val_node_ratio)
    rows, cols = ei
    # step 2: old-old edges -> training / extra inference / test
    oo_train, oo_val, oo_test = split_edges(ei[:, old[rows] & old[cols]], old_old_extra_ratio, test_ratio)
    # step 3-4: old-new and new-new edges -> inference / test
    on_train, _, on_test = split_edges(ei[:, (old[rows] & new[cols]) | (new[rows] & old[cols])], 0.0, test_ratio)
    nn_train, _, nn_test = split_edges(ei[:, new[rows] & new[cols]], 0.0, test_ratio)
    # step 5: test edges
    test_edge_index = torch.cat([oo_test, on_test, nn_test], -1)
    test_edge_bundle = (oo_test, on_test, nn_test, test_edge_index)
    # step 6-7: the old-node training graph and its validation link split
    given = GraphData(x[old], subgraph_relabel(old, oo_train))
    training_data, _, val_data = random_link_split(given, 0.0, val_ratio)
    # step 8: inference graph over all nodes
    inference_data = GraphData(x, torch.cat([oo_train, oo_val, on_train, nn_train], -1))

    print("Datasets Infomation:\t\n")
    print("Name:\t" + data_name + "\n")
    print("#Old Nodes:\t" + str(given.x.size(0)) + "\n")
    print("#New Nodes:\t" + str(x.size(0) - given.x.size(0)) + "\n")
    print("#Old-Old testing edges:\t" + str(oo_test.size(1)) + "\n")
    print("#Old-New testing edges:\t" + str(on_test.size(1)) + "\n")
    print("#New-New testing edges:\t" + str(nn_test.size(1)) + "\n")
    return training_data, val_data, inference_data, GraphData(x, ei), test_edge_bundle, negative_samples


# --- cache ---

def save_production_split(path: str, split) -> None:
    training_data, val_data, inference_data, data, bundle, neg = split
    torch.save({"training_data": training_data.tensors(), "val_data": val_data.tensors(),
                "inference_data": inference_data.tensors(), "data": data.tensors(),
                "test_edge_bundle": list(bundle), "negative_samples": neg}, path)


def load_production_split(path: str):
    try:
        b = torch.load(path, weights_only=True, map_location="cpu")
    except Exception as e:  # e.g. a reference-written pickle of PyG Data objects
        raise RuntimeError(f"{path}: not a tensor-dict production split ({e}); delete it to re-split") from e
    return (GraphData.from_tensors(b["training_data"]), GraphData.from_tensors(b["val_data"]),
            GraphData.from_tensors(b["inference_data"]), GraphData.from_tensors(b["data"]),
            tuple(b["test_edge_bundle"]), b["negative_samples"])


def production_split(data_name: str, dataset_dir: str, synthetic: bool):
    """The reference's load-or-split step (src/train_teacher_gnn.py:341-365):
    ``<dataset_dir>/<ds>_production.pt`` when present, else split the full
    graph with the reference's ratios and seed 234 and cache it."""
    import llp_datasets
    path = os.path.join(dataset_dir, data_name + "_production.pt")
    if os.path.exists(path):
        return load_production_split(path)
    print("splitting the datasets now...")
    data = llp_datasets.load_graph(data_name, dataset_dir, synthetic)
    split = do_production_edge_split(data, data_name, *production_ratios(data_name))
    os.makedirs(dataset_dir, exist_ok=True)
    save_production_split(path, split)
    return split


__all__ = ["GraphData", "coalesce", "to_undirected", "add_self_loops", "train_test_split_edges", "do_edge_split",
           "negative_sampling", "random_node_split", "split_edges", "subgraph_relabel",
           "random_link_split", "production_ratios", "do_production_edge_split", "save_production_split",
           "load_production_split", "production_split"]
