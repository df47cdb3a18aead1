"""Production (inductive) split: llp_split.do_production_edge_split reproduces
the reference's do_production_edge_split (src/generate_production_split.py:32-95)
bit for bit on the golden graphs (tests/golden/production_split_*.npz, made by
gen_golden.run_production_split_case from the reference's own function; the
torch_geometric pieces it calls are restated there — parity with PyG itself is
unpinned), plus the split's structural invariants."""
import contextlib
import io
import os

import numpy as np
import pytest
import torch

import llp_split

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ("production_split_cora_small", "production_split_small")


def _run(case):
    g = np.load(os.path.join(HERE, "golden", case + ".npz"))
    data = llp_split.GraphData(torch.from_numpy(g["x"]), torch.from_numpy(g["edge_index"]))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = llp_split.do_production_edge_split(data, case, *[float(r) for r in g["ratios"]])
    return g, out, buf.getvalue()


@pytest.mark.parametrize("case", CASES)
def test_matches_reference_split(case):
    g, (tr, va, inf, data, bundle, neg), stdout = _run(case)
    eq = np.testing.assert_array_equal
    eq(tr.x.numpy(), g["train_x"])
    eq(tr.edge_index.numpy(), g["train_edge_index"])
    eq(tr.edge_label.numpy(), g["train_edge_label"])
    eq(tr.edge_label_index.numpy(), g["train_edge_label_index"])
    eq(va.edge_index.numpy(), g["val_edge_index"])
    eq(va.edge_label.numpy(), g["val_edge_label"])
    eq(va.edge_label_index.numpy(), g["val_edge_label_index"])
    eq(inf.edge_index.numpy(), g["inference_edge_index"])
    for i, k in enumerate(("old_old", "old_new", "new_new", "test")):
        eq(bundle[i].numpy(), g[k])
    eq(neg.numpy(), g["negative_samples"])
    assert stdout == bytes(g["stdout"]).decode()        # the reference's printed summary


@pytest.mark.parametrize("case", CASES)
def test_split_invariants(case):
    g, (tr, va, inf, data, bundle, neg), _ = _run(case)
    N = int(g["N"])
    ei = torch.from_numpy(g["edge_index"])
    edges = set(map(tuple, ei.t().tolist()))
    und = lambda e: set(map(tuple, torch.sort(e, 0)[0].t().tolist()))   # noqa: E731
    # test edges never appear in the inference graph
    assert not (und(bundle[3]) & und(inf.edge_index))
    # global negatives are non-edges, both directions present
    for a, b in neg.t().tolist():
        assert (a, b) not in edges and a != b
    assert und(neg) == und(neg.flip([0]))
    # old-node training graph: relabelled, within [0, N_old), symmetric
    n_old = tr.x.size(0)
    assert int(tr.edge_index.max()) < n_old
    assert und(tr.edge_index) == und(tr.edge_index.flip([0]))
    # validation labels: positives first, as many negatives
    lab = va.edge_label
    assert lab.sum() * 2 == lab.numel() and bool((lab[: int(lab.sum())] == 1).all())
    # test bundle = old_old | old_new | new_new
    assert bundle[3].size(1) == sum(bundle[i].size(1) for i in range(3))
    assert data.edge_index.size(1) == ei.size(1) and N == data.x.size(0)


def test_cache_round_trip(tmp_path):
    g, out, _ = _run(CASES[0])
    p = str(tmp_path / "x_production.pt")
    llp_split.save_production_split(p, out)
    back = llp_split.load_production_split(p)
    for a, b in zip(out[:4], back[:4]):
        for k, v in a.tensors().items():
            assert torch.equal(v, getattr(b, k))
    for a, b in zip(out[4], back[4]):
        assert torch.equal(a, b)
    assert torch.equal(out[5], back[5])


def test_undirected_vector_round_trip():
    """force_undirected edge <-> vector id maps are inverse (PyG layout)."""
    N = 37
    r, c = torch.triu_indices(N, N, 1)
    idx, pop = llp_split._edge_index_to_vector(torch.stack([r, c]), N, True)
    assert pop == N * (N - 1) // 2 and torch.equal(idx, torch.arange(pop))
    back = llp_split._vector_to_edge_index(idx, N, True)
    assert torch.equal(back[:, :pop], torch.stack([r, c]))
    idx2, pop2 = llp_split._edge_index_to_vector(back[:, :pop].flip([0]), N, False)
    back2 = llp_split._vector_to_edge_index(idx2, N, False)
    assert torch.equal(back2, back[:, :pop].flip([0]))


@pytest.mark.parametrize("case", ["edge_split_small", "edge_split_fast_small"])
def test_edge_split_matches_reference(case):
    """do_edge_split (src/utils.py:62-105, the transductive SEAL split the
    reference caches as ../data/<ds>.pkl): same edges, same order."""
    g = np.load(os.path.join(HERE, "golden", case + ".npz"))
    data = llp_split.GraphData(torch.from_numpy(g["x"]), torch.from_numpy(g["edge_index"]))
    se = llp_split.do_edge_split(data, fast_split=bool(int(g["fast_split"])))
    for s in ("train", "valid", "test"):
        for k in ("edge", "edge_neg"):
            np.testing.assert_array_equal(se[s][k].numpy(), g[f"{s}/{k}"], err_msg=f"{s}/{k}")
    if not int(g["fast_split"]):
        # train positives come back in both directions (to_undirected), the others once
        tr = se["train"]["edge"]
        assert set(map(tuple, tr.tolist())) == set(map(tuple, tr.flip(1).tolist()))
        assert bool((se["valid"]["edge"][:, 0] < se["valid"]["edge"][:, 1]).all())
