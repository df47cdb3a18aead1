"""Offline dataset layer (llp_datasets): raw-file readers that need no
unpickling, the reference's split cache ``../data/<ds>.pkl`` (read and written
as the same dict of tensors), and synthetic graphs split by the reference's
do_edge_split (train edges in both directions, src/utils.py:62-105)."""
import gzip
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import llp_datasets
import llp_split


@pytest.fixture()
def workdir(tmp_path):
    w = tmp_path / "src"
    w.mkdir()
    old = os.getcwd()
    os.chdir(w)
    yield tmp_path
    os.chdir(old)


def _write_coauthor_npz(path, N=60, F=30, E=150, seed=0):
    rng = np.random.default_rng(seed)
    attr = sp.random(N, F, density=0.1, format="csr", random_state=seed, dtype=np.float32) * 3
    u, v = rng.integers(0, N, E), rng.integers(0, N, E)
    u[:3] = v[:3]                                       # self-loops: dropped by the reader
    adj = sp.csr_matrix((np.ones(E, np.float32), (u, v)), shape=(N, N))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez(path, attr_data=attr.data, attr_indices=attr.indices, attr_indptr=attr.indptr,
             attr_shape=np.array(attr.shape), adj_data=adj.data, adj_indices=adj.indices, adj_indptr=adj.indptr,
             adj_shape=np.array(adj.shape), labels=rng.integers(0, 5, N))
    return attr, u, v


def test_npz_reader_and_reference_split_cache(workdir):
    ddir = str(workdir / "data")
    attr, u, v = _write_coauthor_npz(os.path.join(ddir, "CS", "raw", "ms_academic_cs.npz"))
    g = llp_datasets.load_graph("coauthor-cs", ddir, synthetic=False)
    assert torch.equal(g.x, torch.from_numpy((attr.toarray() > 0).astype(np.float32)))
    keep = u != v
    want = set(zip(u[keep].tolist(), v[keep].tolist())) | set(zip(v[keep].tolist(), u[keep].tolist()))
    assert set(map(tuple, g.edge_index.t().tolist())) == want
    key = g.edge_index[0] * g.num_nodes + g.edge_index[1]
    assert bool((key[1:] > key[:-1]).all())                       # coalesced
    # first call splits and writes the reference's cache, second call reads it
    data, se = llp_datasets.load_transductive("coauthor-cs", ddir, synthetic=False)
    assert os.path.exists(workdir / "data" / "coauthor-cs.pkl")
    cached = torch.load(workdir / "data" / "coauthor-cs.pkl", weights_only=True)
    ref = llp_split.do_edge_split(g)
    for s in ("train", "valid", "test"):
        for k in ("edge", "edge_neg"):
            assert torch.equal(cached[s][k], ref[s][k]) and torch.equal(se[s][k], ref[s][k])
    data2, se2 = llp_datasets.load_transductive("coauthor-cs", ddir, synthetic=False)
    assert torch.equal(data2.adj_t, se["train"]["edge"].t())


def test_ogb_collab_raw_reader(workdir):
    d = workdir / "src" / "dataset" / "ogbl_collab"
    (d / "raw").mkdir(parents=True)
    (d / "split" / "time").mkdir(parents=True)
    rng = np.random.default_rng(1)
    N, E = 40, 90
    edges = rng.integers(0, N, (E, 2))
    feats = rng.standard_normal((N, 8)).astype(np.float32)
    with gzip.open(d / "raw" / "edge.csv.gz", "wt") as f:
        f.write("\n".join(f"{a},{b}" for a, b in edges) + "\n")
    with gzip.open(d / "raw" / "node-feat.csv.gz", "wt") as f:
        f.write("\n".join(",".join(repr(float(t)) for t in row) for row in feats) + "\n")
    torch.save({"edge": edges, "weight": np.ones(E), "year": np.full(E, 2010)}, d / "split" / "time" / "train.pt")
    for s in ("valid", "test"):     # OGB's split files hold numpy arrays
        torch.save({"edge": edges[:10], "edge_neg": rng.integers(0, N, (20, 2))}, d / "split" / "time" / (s + ".pt"))
    data, se = llp_datasets.load_transductive("collab", str(workdir / "data"), synthetic=False)
    assert torch.allclose(data.x, torch.from_numpy(feats))
    assert torch.equal(se["train"]["edge"], torch.from_numpy(edges))
    assert se["valid"]["edge_neg"].shape == (20, 2)
    # interleaved (u,v),(v,u) layout of add_inverse_edge
    assert torch.equal(data.edge_index[:, 0::2], torch.from_numpy(edges.T))
    assert torch.equal(data.edge_index[:, 1::2], torch.from_numpy(edges.T[::-1].copy()))


def test_synthetic_split_is_reference_layout(workdir):
    ddir = str(workdir / "data")
    data, se = llp_datasets.load_transductive("cora", ddir, synthetic=True)
    tr = se["train"]["edge"]
    assert set(map(tuple, tr.tolist())) == set(map(tuple, tr.flip(1).tolist()))   # both directions
    n_und = tr.shape[0] // 2 + se["valid"]["edge"].shape[0] + se["test"]["edge"].shape[0]
    assert se["valid"]["edge"].shape[0] == int(np.floor(0.05 * n_und))
    assert se["test"]["edge"].shape[0] == int(np.floor(0.10 * n_und))
    assert os.path.exists(os.path.join(ddir, "cora_synthetic_split.pt"))
    assert not os.path.exists(workdir / "data" / "cora.pkl")       # never the reference's cache
    _, se2 = llp_datasets.load_transductive("cora", ddir, synthetic=True)
    assert torch.equal(se2["train"]["edge"], tr)


def test_synthetic_collab_matches_the_benchmark_spec():
    """The bench's synthetic ogbl-collab: full-size counts,
    OGB-interleaved unsorted edges (Q1), ~5 % duplicate pairs (Q2), ~90 % of the
    non-duplicate pairs inside a planted community, no self loops, features of F=128."""
    import llp_data
    d = llp_data.synthetic_collab(seed=0, scale=1.0, with_eval=True)
    C = llp_data.COLLAB
    assert (d.N, d.F) == (C["N"], C["F"]) == (235_868, 128)
    assert tuple(d.train_pairs.shape) == (C["E_train"], 2)
    assert d.edge_index.shape[1] == 2 * C["E_train"] == 2_358_104
    ei = d.edge_index.numpy()
    assert np.array_equal(ei[:, 0::2], d.train_pairs.numpy().T)          # (u,v), (v,u), ...
    assert np.array_equal(ei[:, 1::2], d.train_pairs.numpy().T[::-1])
    assert (np.diff(ei[0]) < 0).any()                                    # row NOT sorted
    p = d.train_pairs.numpy()
    assert (p[:, 0] != p[:, 1]).all()
    key = p[:, 0].astype(np.int64) * d.N + p[:, 1]
    dup = 1.0 - np.unique(key).size / key.size
    assert 0.05 < dup < 0.065       # 5 % drawn as copies + chance repeats inside ~236-node communities
    comm = llp_data.planted_pairs.last_comm                              # the held-out draw reuses it
    intra = (comm[p[:, 0]] == comm[p[:, 1]]).mean()
    assert 0.88 < intra < 0.92
    for s, n in (("valid", C["n_valid"]), ("test", C["n_test"])):
        assert tuple(d.split_edge[s]["edge"].shape) == (n, 2)
        assert tuple(d.split_edge[s]["edge_neg"].shape) == (C["n_neg"], 2)
    assert d.x.dtype == torch.float32 and tuple(d.x.shape) == (d.N, 128)


def test_locality_order_is_a_permutation_that_groups_communities():
    """locality_order on a planted-partition graph: a permutation, and most edges end up
    between nearby rows (the L2 reuse the aggregate relies on)."""
    import numpy as np
    import llp_data
    import llp_sage
    d = llp_data.synthetic_collab(seed=3, scale=0.05, with_eval=False)
    ei = d.edge_index.numpy()
    order, pi = llp_sage.locality_order(ei, d.N)
    assert np.array_equal(np.sort(order), np.arange(d.N)) and np.array_equal(pi[order], np.arange(d.N))
    near = float((np.abs(pi[ei[0]] - pi[ei[1]]) < 1024).mean())
    near_id = float((np.abs(ei[0] - ei[1]) < 1024).mean())
    assert near > 0.6 and near > 4 * near_id, (near, near_id)
