"""GraphSAGE teacher pieces on MI355X: the CSR graph layout and the SAGEConv
layers used by the reference's SAGE encoder (src/models.py:82-119).

  SAGEConv          — torch_geometric 2.2.0 SAGEConv(aggr='mean') semantics
                      (restated, the package is not installed): mean over
                      incoming edges, then lin_l (bias) + lin_r (no bias) on the
                      root (used at src/train_teacher_gnn.py:381-383).
  SAGEConv_updated  — src/sageconv_updated.py:9-93: lin_l FIRST, then the
                      mean, then + lin_r(x) (used for coauthor-physics).
  GCNConv           — torch_geometric 2.2.0 GCNConv(cached=True) (restated):
                      lin (no bias), symmetric-normalised propagation over the
                      graph with one self-loop per node, + bias (the GCN
                      encoder, src/models.py:56-80).

State-dict keys (``lin_l.weight``, ``lin_l.bias``, ``lin_r.weight``; GCN:
``bias``, ``lin.weight``) match PyG's, so the reference's saved teacher
weights load here.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

import llp_ops as ops


class Graph:
    """edge_index (2, E) as CSR by destination (PyG flow source_to_target):
    row i lists the sources of the edges into i, duplicates kept.
    Also the transposed CSR (by source) and 1/deg for the backward.

    ``gcn=True``: the graph GCNConv propagates over (PyG 2.2.0 gcn_norm with
    add_remaining_self_loops): input self-loops dropped, one loop per node
    added; ``dinv`` = deg^-1/2 with deg counted at the destination."""

    def __init__(self, edge_index, num_nodes: int, device, gcn: bool = False):
        ei = edge_index.cpu().numpy() if torch.is_tensor(edge_index) else np.asarray(edge_index)
        src = ei[0].astype(np.int64)
        dst = ei[1].astype(np.int64)
        N = int(num_nodes)
        if gcn:
            keep = src != dst
            loops = np.arange(N, dtype=np.int64)
            src = np.concatenate([src[keep], loops])
            dst = np.concatenate([dst[keep], loops])
        assert src.size < 2 ** 31
        order = np.argsort(dst, kind="stable")
        deg = np.bincount(dst, minlength=N)
        rowptr = np.zeros(N + 1, np.int64)
        np.cumsum(deg, out=rowptr[1:])
        order_t = np.argsort(src, kind="stable")
        deg_t = np.bincount(src, minlength=N)
        rowptr_t = np.zeros(N + 1, np.int64)
        np.cumsum(deg_t, out=rowptr_t[1:])
        dev = torch.device(device)
        self.num_dst = N
        self.num_edges = int(src.size)
        self.rowptr = torch.from_numpy(rowptr.astype(np.int32)).to(dev)
        self.col = torch.from_numpy(src[order].astype(np.int32)).to(dev)
        self.rowptr_t = torch.from_numpy(rowptr_t.astype(np.int32)).to(dev)
        self.col_t = torch.from_numpy(dst[order_t].astype(np.int32)).to(dev)
        self.inv_deg = torch.from_numpy((1.0 / np.maximum(deg, 1)).astype(np.float32)).to(dev)
        self.gcn = gcn
        if gcn:
            self.dinv = torch.from_numpy((1.0 / np.sqrt(deg.astype(np.float64))).astype(np.float32)).to(dev)


def locality_order(edge_index, num_nodes: int, iters: int = 10):
    """A node order that puts each node's neighbours near it, for the CSR aggregate's L2 reuse
    (SAGE / GCN teacher, src/models.py:110-119): synchronous label propagation over the
    (symmetric) graph -- every node takes the most frequent label of its in-neighbours,
    ties to the smallest label, starting from its own id -- for up to ``iters`` rounds, then
    nodes sorted by (label, id).  Deterministic host numpy, O(E log E) per round.

    Returns (order, pi): new id i holds node order[i]; pi[v] = new id of node v."""
    ei = edge_index.cpu().numpy() if torch.is_tensor(edge_index) else np.asarray(edge_index)
    N = int(num_nodes)
    src, dst = ei[0].astype(np.int64), ei[1].astype(np.int64)
    lab = np.arange(N, dtype=np.int64)
    for _ in range(iters):
        key = dst * N + lab[src]
        key.sort()
        b = np.flatnonzero(np.diff(key)) + 1
        starts = np.concatenate([[0], b]) if key.size else np.zeros(0, np.int64)
        ends = np.concatenate([b, [key.size]]) if key.size else np.zeros(0, np.int64)
        rk, cnt = key[starts], ends - starts
        v, lb = rk // N, rk % N
        o = np.lexsort((lb, -cnt, v))            # per node: the largest count, then the smallest label
        vo = v[o]
        first = np.ones(vo.size, bool)
        first[1:] = vo[1:] != vo[:-1]
        new = lab.copy()
        new[vo[first]] = lb[o][first]
        if np.array_equal(new, lab):
            break
        lab = new
    order = np.lexsort((np.arange(N), lab))
    pi = np.empty(N, np.int64)
    pi[order] = np.arange(N)
    return order, pi


_GRAPH_CACHE = {}


def as_graph(edge_index, num_nodes, device, gcn=False):
    """Cache the CSR per edge_index tensor (the reference re-passes the same
    data.adj_t every step, src/train_teacher_gnn.py:43; GCNConv(cached=True)
    caches its normalised graph likewise)."""
    if isinstance(edge_index, Graph):
        return edge_index
    key = (id(edge_index), int(num_nodes), str(device), bool(gcn))
    g = _GRAPH_CACHE.get(key)
    if g is None or g[0] is not edge_index:
        g = (edge_index, Graph(edge_index, num_nodes, device, gcn=gcn))
        _GRAPH_CACHE[key] = g
    return g[1]


class SAGEConv(nn.Module):
    def __init__(self, in_channels, out_channels, normalize=False, root_weight=True, bias=True, **kwargs):
        super().__init__()
        if normalize:
            raise NotImplementedError("SAGEConv(normalize=True) is not used by the reference")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.root_weight = root_weight
        self.lin_l = nn.Linear(in_channels, out_channels, bias=bias)
        if root_weight:
            self.lin_r = nn.Linear(in_channels, out_channels, bias=False)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin_l.reset_parameters()
        if self.root_weight:
            self.lin_r.reset_parameters()

    def forward(self, x, edge_index):
        g = as_graph(edge_index, x.shape[0], x.device)
        out = ops.linear(ops.mean_aggregate(x, g), self.lin_l.weight, self.lin_l.bias)
        if self.root_weight:
            out = out + ops.linear(x, self.lin_r.weight, None)
        return out

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, aggr=mean)"


class SAGEConv_updated(SAGEConv):
    """src/sageconv_updated.py:65-81: out = mean_j(W_l x_j + b) + W_r x_i."""

    def forward(self, x, edge_index):
        g = as_graph(edge_index, x.shape[0], x.device)
        out = ops.mean_aggregate(ops.linear(x, self.lin_l.weight, self.lin_l.bias), g)
        if self.root_weight:
            out = out + ops.linear(x, self.lin_r.weight, None)
        return out


class GCNConv(nn.Module):
    """GCNConv(in, out, cached=True) with PyG 2.2.0 defaults (normalize,
    add_self_loops, improved=False, bias): out = D^-1/2 (A - loops + I) D^-1/2 (x W^T) + b."""

    def __init__(self, in_channels, out_channels, cached=False, bias=True, improved=False, add_self_loops=True,
                 normalize=True, **kwargs):
        super().__init__()
        if improved or not add_self_loops or not normalize:
            raise NotImplementedError("GCNConv options other than the reference's (src/models.py:60-64)")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.cached = cached
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.lin.weight)       # PyG 'glorot'
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x, edge_index):
        g = as_graph(edge_index, x.shape[0], x.device, gcn=True)
        return ops.gcn_aggregate(ops.linear(x, self.lin.weight, None), g, self.bias)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"
