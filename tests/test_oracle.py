"""Known-answer tests of the oracle's restatements of third-party code the
reference calls but does not ship (torch_cluster 1.6.0 random_walk, PyG 2.2.0
mean aggregation / gcn_norm / dense negative_sampling, ogb 1.3.6 hits@K,
sklearn roc_auc_score) and of its own Philox stream.  None of those packages
is importable here, so these hand-computed answers (and the published
Random123 vectors) are what pins them.  CPU only."""
import itertools
import math

import numpy as np
import pytest
import torch

from oracle import llp_oracle as O


# ---------------------------------------------------------------- Philox4x32-10
@pytest.mark.parametrize("ctr,key,want", [
    # Random123 kat_vectors, philox4x32 R=10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, want):
    out = O.philox4x32(*[np.array([c], np.uint32) for c in ctr], *key)
    assert tuple(int(o[0]) for o in out) == want


def test_philox_stream_layout():
    """Draw #idx of (seed, stream) is word idx & 3 of the block at counter
    (idx >> 2, 0, stream_lo, stream_hi), key (seed_lo, seed_hi)."""
    seed, stream = 0x0123456789ABCDEF, (7 << 32) | 5
    idx = np.arange(12, dtype=np.uint64)
    got = O.philox_u32(seed, stream, idx)
    for i in range(12):
        blk = O.philox4x32(np.array([i >> 2], np.uint32), np.array([0], np.uint32), np.array([5], np.uint32),
                           np.array([7], np.uint32), seed & 0xFFFFFFFF, seed >> 32)
        assert int(got[i]) == int(blk[i & 3][0])


def test_dropout_code_and_keep_layout():
    """dropout_keep (the device's drop_keep): 8-bit draws when p * 256 is an integer, else
    16-bit with thr = ceil(p * 65536); element -> (block, word, byte/half) as documented,
    checked element by element against philox4x32 for both widths; keep rates near 1 - p."""
    assert O.dropout_code(0.5) == 0x80000000 | 128
    assert O.dropout_code(0.25) == 0x80000000 | 64
    assert O.dropout_code(0.3) == math.ceil(float(np.float32(0.3)) * 65536)
    seed, stream, rows, n = 0xABCDEF12345, 3 * O.STREAMS_PER_STEP + 2, 3, 200
    for p in (0.5, 0.3):
        keep = O.dropout_keep(seed, stream, rows, n, p)
        code = O.dropout_code(p)
        thr = code & 0x7FFFFFFF
        ng = (n + 63) // 64
        for r in range(rows):
            for c in range(0, n, 7):
                grp = (r * ng + c // 64) * 4 + ((c >> 2) & 3)
                if code >> 31:
                    blk, word, sh, mk = grp, (c >> 4) & 3, 8 * (c & 3), 0xFF
                else:
                    blk, word, sh, mk = 2 * grp + ((c >> 5) & 1), ((c >> 4) & 1) * 2 + ((c >> 1) & 1), 16 * (c & 1), 0xFFFF
                out = O.philox4x32(np.array([blk & 0xFFFFFFFF], np.uint32), np.array([blk >> 32], np.uint32),
                                   np.array([stream & 0xFFFFFFFF], np.uint32), np.array([stream >> 32], np.uint32),
                                   seed & 0xFFFFFFFF, seed >> 32)
                assert bool(keep[r, c]) == (((int(out[word][0]) >> sh) & mk) >= thr)
        big = O.dropout_keep(seed, stream, 512, 256, p)
        assert abs(big.mean() - (1 - p)) < 0.01
        assert np.array_equal(big, O.dropout_keep(seed, stream, 512, 256, p))


def test_uniform_and_randint_index_are_exact():
    rng = np.random.default_rng(0)
    x = rng.integers(0, 2 ** 32, 20_000, dtype=np.uint64).astype(np.uint32)
    for n in (1, 2, 3, 7, 1000, 235_868, (1 << 29) - 3):
        u = (x >> np.uint32(8)).astype(np.float64) / 2.0 ** 24          # exact in f64
        assert np.array_equal(O.uniform_index(x, n), np.floor(u * n).astype(np.int64))
        r = O.randint_index(x, n)
        assert r.min() >= 0 and r.max() < n
        assert np.array_equal(r, (x.astype(object) * n >> 32).astype(np.int64))


# ---------------------------------------------------------------- random walk
def test_rowptr_keeps_unsorted_col_order():
    """torch_cluster random_walk(coalesced=False): rowptr from degree counts, col
    NOT reordered (with an unsorted edge list the 'neighbours' of n are
    col[rowptr[n]:rowptr[n+1]] of the given array)."""
    row = np.array([0, 1, 0, 0, 0]); col = np.array([2, 0, 1, 2, 3])
    rowptr, c = O.build_rowptr(row, col, 4)
    assert rowptr.tolist() == [0, 4, 5, 5, 5]
    assert c.tolist() == [2, 0, 1, 2, 3]
    rowptr_s, c_s = O.build_rowptr(row, col, 4, coalesced=True)
    assert rowptr_s.tolist() == [0, 4, 5, 5, 5] and c_s.tolist() == [1, 2, 2, 3, 0]


def test_random_walk_step_law_and_dead_ends():
    row = np.array([0, 1, 0, 0, 0]); col = np.array([2, 0, 1, 2, 3])
    rowptr, c = O.build_rowptr(row, col, 4)
    n = 40_000
    w = O.random_walk(rowptr, c, np.zeros(n, np.int64), 1, seed=11, stream=3)
    assert (w[:, 0] == 0).all()
    # uniform over the 4 slots col[0:4] = [2, 0, 1, 2]: P(2) = 1/2, P(0) = P(1) = 1/4, P(3) = 0
    cnt = np.bincount(w[:, 1], minlength=4)
    assert cnt[3] == 0
    exp = np.array([0.25, 0.25, 0.5]) * n
    chi2 = float((((cnt[:3] - exp) ** 2) / exp).sum())
    assert chi2 < 13.8                       # 2 dof, p = 0.001
    # nodes without out-edges stay where they are
    w2 = O.random_walk(rowptr, c, np.array([2, 3, 3]), 3, seed=1, stream=0)
    assert w2.tolist() == [[2, 2, 2, 2], [3, 3, 3, 3], [3, 3, 3, 3]]
    # one walk: each step is col[rowptr[cur] + floor(u * deg(cur))] of its own draw
    w3 = O.random_walk(rowptr, c, np.array([0, 1]), 2, seed=5, stream=9)
    d = O.philox_u32(5, 9, np.arange(4, dtype=np.uint64)).reshape(2, 2)
    for b in range(2):
        cur = w3[b, 0]
        for l in range(2):
            deg = rowptr[cur + 1] - rowptr[cur]
            nxt = c[rowptr[cur] + int(O.uniform_index(d[b, l:l + 1], deg)[0])] if deg else cur
            assert w3[b, l + 1] == nxt
            cur = nxt


def test_neighbor_samplers_shapes_and_streams():
    """src/main.py:33-50: 'nb' concatenates `step` walks of `hops` (stream base + i),
    the negatives are step*hops*ns_rate uniform ids from stream base + step."""
    rng = np.random.default_rng(1)
    N = 50
    row = rng.integers(0, N, 300); col = rng.integers(0, N, 300)
    rowptr, c = O.build_rowptr(row, col, N)
    sample = np.arange(10)
    pos, neg = O.neighbor_samplers(rowptr, c, sample, N, step=3, ps_method="nb", ns_rate=2, hops=2, seed=4,
                                   stream_base=100)
    assert pos.shape == (10, 1 + 3 * 2) and neg.shape == (10, 3 * 2 * 2)
    w1 = O.random_walk(rowptr, c, sample, 2, 4, 101)
    assert np.array_equal(pos[:, 3:5], w1[:, 1:])
    assert (pos[:, 0] == sample).all()
    pos_rw, _ = O.neighbor_samplers(rowptr, c, sample, N, step=3, ps_method="rw", ns_rate=2, hops=2, seed=4,
                                    stream_base=100)
    assert np.array_equal(pos_rw, O.random_walk(rowptr, c, sample, 6, 4, 100))
    assert neg.min() >= 0 and neg.max() < N


# ---------------------------------------------------------------- PyG restatements
def test_sage_mean_counts_duplicates_and_empty_is_zero():
    x = torch.tensor([[1.0, 0.0], [0.0, 2.0], [4.0, 4.0]])
    src = torch.tensor([0, 1, 1, 2]); dst = torch.tensor([2, 2, 2, 0])
    out = O.sage_mean_aggregate(x, src, dst, 3)
    assert torch.allclose(out, torch.tensor([[4.0, 4.0], [0.0, 0.0], [1 / 3, 4 / 3]]))


def test_gcn_norm_replaces_self_loops():
    ei = torch.tensor([[0, 1, 1, 2, 0], [1, 0, 2, 1, 0]])   # path 0-1-2 and a loop on 0
    src, dst, w = O.gcn_norm(ei, 3)
    # the existing loop is dropped and one loop per node added: in-degrees 2, 3, 2
    assert src.tolist() == [0, 1, 1, 2, 0, 1, 2] and dst.tolist() == [1, 0, 2, 1, 0, 1, 2]
    dinv = [1 / math.sqrt(2), 1 / math.sqrt(3), 1 / math.sqrt(2)]
    want = [dinv[s] * dinv[d] for s, d in zip(src.tolist(), dst.tolist())]
    assert torch.allclose(w, torch.tensor(want, dtype=torch.float64))


def test_negative_sampling_dense_small_population_is_exact():
    """Population <= sample size: PyG takes range(population), drops the existing
    edges and decodes in order (no randomness)."""
    ei = torch.tensor([[0, 1], [1, 2]])                     # 0->1, 1->2; N = 3, population 6
    neg = O.negative_sampling_dense(ei, 3, 4)
    assert neg.tolist() == [[0, 1, 2, 2], [2, 0, 0, 1]]
    negp = O.negative_sampling_dense_philox(ei.numpy(), 3, 4, seed=0, stream=0)
    assert negp.tolist() == neg.tolist()
    assert O.dense_neg_sample_size(2, 3, 4) == 6


def test_negative_sampling_dense_properties():
    import random
    rng = np.random.default_rng(2)
    N = 40
    ei = torch.from_numpy(rng.integers(0, N, (2, 200)))
    existing = set(map(tuple, ei.t().tolist()))
    for neg in (O.negative_sampling_dense(ei, N, 150, rng=random.Random(3)),
                torch.from_numpy(O.negative_sampling_dense_philox(ei.numpy(), N, 150, seed=9, stream=1))):
        pairs = list(map(tuple, neg.t().tolist()))
        assert 0 < len(pairs) <= 150
        assert len(set(pairs)) == len(pairs)                # without replacement
        assert all(r != c for r, c in pairs)                # no self loops
        assert not (set(pairs) & existing)                  # no existing edge
        assert all(0 <= r < N and 0 <= c < N for r, c in pairs)


def test_dense_key_encoding_round_trip():
    N = 7
    r, c = np.meshgrid(np.arange(N), np.arange(N), indexing="ij")
    m = r != c
    ei = np.stack([r[m], c[m]])
    keys, n = O.dense_neg_keys(ei, N)
    assert n == N * (N - 1) and keys.tolist() == list(range(N * (N - 1)))


# ---------------------------------------------------------------- eval metrics
def test_hits_at_k_known_answers():
    pos = torch.tensor([0.9, 0.5, 0.3]); neg = torch.tensor([0.8, 0.4, 0.1])
    assert O.hits_at_k(pos, neg, 1) == pytest.approx(1 / 3)
    assert O.hits_at_k(pos, neg, 2) == pytest.approx(2 / 3)
    assert O.hits_at_k(pos, neg, 3) == pytest.approx(1.0)
    assert O.hits_at_k(pos, neg, 4) == 1.0                  # fewer negatives than K
    assert O.hits_at_k(torch.tensor([0.8]), torch.tensor([0.8, 0.2]), 1) == 0.0   # ties lose (strict >)


def test_auc_known_answers():
    assert O.auc(torch.tensor([0.9, 0.4]), torch.tensor([0.5, 0.1])) == pytest.approx(0.75)
    assert O.auc(torch.tensor([0.5]), torch.tensor([0.5])) == pytest.approx(0.5)     # a tie counts half
    rng = np.random.default_rng(3)
    p = torch.from_numpy(rng.normal(1, 1, 300)); n = torch.from_numpy(rng.normal(0, 1, 500))
    mw = float(((p[:, None] > n[None, :]).double() + 0.5 * (p[:, None] == n[None, :]).double()).mean())
    assert O.auc(p, n) == pytest.approx(mw, abs=1e-12)


# ---------------------------------------------------------------- losses and step tail
def test_pair_index_is_combinations_order():
    for C in (2, 5, 36):
        i, j = O.pair_index(C)
        assert list(zip(i.tolist(), j.tolist())) == list(itertools.combinations(range(C), 2))


def test_rank_loss_known_answer():
    s = torch.tensor([[0.9, 0.2, 0.5]]); t = torch.tensor([[0.8, 0.1, 0.45]])
    # pairs (0,1): t0 > t1 + m -> y = +1; (0,2): |dt| = 0.35 > m -> +1; (1,2): t1 < t2 - m -> -1
    m = 0.1
    want = (max(0, -(0.9 - 0.2) + m) + max(0, -(0.9 - 0.5) + m) + max(0, (0.2 - 0.5) + m)) / 3
    assert float(O.rank_loss(s, t, m)) == pytest.approx(want)
    # |t_i - t_j| <= margin: y = 0, the pair costs max(0, margin)
    assert float(O.rank_loss(torch.tensor([[3.0, -1.0]]), torch.tensor([[0.5, 0.55]]), 0.1)) == pytest.approx(0.1)


def test_kl_loss_zero_on_equal_and_sign():
    s = torch.randn(4, 6, generator=torch.Generator().manual_seed(0))
    assert float(O.kl_loss(s, s.clone())) == pytest.approx(0.0, abs=1e-7)
    assert float(O.kl_loss(s, s.flip(-1))) > 0


def test_clip_and_adam_match_torch():
    g = torch.Generator().manual_seed(5)
    params = [torch.randn(4, 3, generator=g), torch.randn(3, generator=g)]
    grads = [torch.randn(4, 3, generator=g) * 3, torch.randn(3, generator=g) * 3]
    clipped, total = O.clip_grad_norm(grads, 1.0)
    ref = [p.clone().requires_grad_() for p in params]
    for r, gr in zip(ref, grads):
        r.grad = gr.clone()
    tot_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    assert float(total) == pytest.approx(float(tot_ref), rel=1e-6)
    for cg, r in zip(clipped, ref):
        assert torch.allclose(cg, r.grad, rtol=1e-6)
    opt = torch.optim.Adam(ref, lr=0.01)
    st = O.AdamState(params, lr=0.01)
    cur = [p.clone() for p in params]
    for _ in range(3):
        opt.step()
        cur = st.step(cur, clipped)
    for c_, r in zip(cur, ref):
        assert torch.allclose(c_, r.detach(), rtol=1e-6, atol=1e-7)
