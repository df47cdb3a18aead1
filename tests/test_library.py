"""CPU-only checks of the C-ABI boundary: the library loads without a GPU and
exports every entry point include/llp_hip.h declares (no compute calls)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "llp_hip.h")
LIB = os.path.join(REPO, "linkless-link-prediction_amd", "libllp_hip.so")


def declared_symbols():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(llp_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import __graft_entry__  # noqa: F401  (repo root on sys.path via conftest)
        __graft_entry__.build()
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert len(syms) >= 30
    for must in ("llp_gemm_nt", "llp_gemm_tn", "llp_llp_loss", "llp_context_sampler", "llp_csr_aggregate",
                 "llp_adam_step", "llp_head_fwd", "llp_hadamard_bwd_blocks"):
        assert must in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_error_string(lib):
    lib.llp_version.restype = ctypes.c_int
    assert lib.llp_version() == 1
    lib.llp_last_error.restype = ctypes.c_char_p
    assert isinstance(lib.llp_last_error(), bytes)


def test_python_binding_signatures_cover_header():
    import llp_hip
    assert set(declared_symbols()) == set(llp_hip._SIGS), set(declared_symbols()) ^ set(llp_hip._SIGS)


def test_binding_loads_without_gpu():
    import llp_hip
    L = llp_hip.load()
    assert L.llp_version() == 1
    # argument validation happens before any device call
    assert L.llp_llp_loss_workspace_bytes(10, 20) > 0
    assert L.llp_gemm_tn_workspace_bytes(1, 1000, 64, 64) >= 64 * 64 * 4


def test_philox_stream_layout_agrees():
    """One stream layout per step in the kernels, the engine and the oracle, wide enough
    for the reference CLI's rw_step (any int; its scripts use up to 3) well past 14."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
    import llp_engine
    from oracle import llp_oracle as O
    txt = open(os.path.join(REPO, "linkless-link-prediction_amd", "csrc", "llp_common.h")).read()
    m = re.search(r"LLP_STREAMS_PER_STEP\s*=\s*(\d+)", txt)
    assert m and int(m.group(1)) == llp_engine.STREAMS_PER_STEP == O.STREAMS_PER_STEP
    assert llp_engine.RANDINT_STREAM == O.RANDINT_STREAM and llp_engine.DENSE_NEG_STREAM == O.DENSE_NEG_STREAM
    assert llp_engine.MAX_RW_STEP < llp_engine.DENSE_NEG_STREAM and llp_engine.MAX_RW_STEP >= 60   # negatives at rw_step


def test_splitk_plan_host_arithmetic():
    """llp_gemm_nt_splitk_plan (host only; 256 CUs without a device): split the first
    full-batch student layer at the coauthor-physics production shape (122 and, at 4
    ranks, 31 tiles over 132 K-tiles), never a launch that already fills the chip or has
    a short K, and the slab workspace is S*M*N floats."""
    import llp_hip
    plan = llp_hip.gemm_nt_splitk_plan
    assert plan(31_044, 256, 8_448) == 2
    assert plan(7_761, 256, 8_448) == 8
    assert plan(1_000, 512, 2_048) == 4
    assert plan(225_334, 1024, 1024) == 1       # thousands of tiles
    assert plan(31_044, 256, 256) == 1          # 4 K-tiles
    assert plan(1_000, 500, 2_048) == 1         # N not a multiple of 256
    assert plan(100, 256, 64 * 1000) == 16      # capped at 16 slabs
    assert llp_hip.gemm_nt_splitk_ws_bytes(7_761, 256, 8) == 8 * 7_761 * 256 * 4


def test_sparse_rows_host_layout():
    """llp_hip.SparseRows (the sparse first layer's host-side layout, built with torch on any
    device; here the CPU): CSR of x, per-slice CSC with local rows ascending in each column,
    the heavy-first feature order and heavy count llp_spmm_tn schedules by, and val = None
    exactly when every stored value is 1."""
    import numpy as np
    import torch
    import llp_hip
    g = torch.Generator().manual_seed(2)
    x = (torch.rand(90, 333, generator=g) < 0.03).float()
    x[:, 7] = 1.0                                   # a column with a nonzero in every row
    x[40] = 0.0                                     # an empty row
    xs = llp_hip.SparseRows(x)
    assert xs.val is None and xs.nnz == int((x != 0).sum())
    rp, ci = xs.rowptr.numpy(), xs.colidx.numpy()
    for r in range(90):
        assert np.array_equal(ci[rp[r]:rp[r + 1]], np.nonzero(x[r].numpy())[0])
    heavy = llp_hip.load().llp_spmm_heavy_nnz()
    for r0, n in [(0, 90), (13, 50)]:
        colptr, rowidx, val, perm, n_heavy = xs.csc(r0, n)
        cp, ri = colptr.numpy(), rowidx.numpy()
        cnt = np.diff(cp)
        for f in range(333):
            assert np.array_equal(ri[cp[f]:cp[f + 1]], np.nonzero(x[r0:r0 + n, f].numpy())[0])
        assert np.array_equal(perm.numpy(), np.argsort(-cnt, kind="stable"))
        assert n_heavy == int((cnt >= heavy).sum())
        assert val is None
    xv = x * 2.0
    assert torch.equal(llp_hip.SparseRows(xv).val, torch.full((xs.nnz,), 2.0))


def test_sparse_rows_values_rounded_like_the_dense_layer():
    """the sparse first layer's values are x rounded through bf16, as the dense
    first layer reads x (its bf16 copy), so both paths multiply the same numbers."""
    import torch
    import llp_hip
    x = torch.zeros(4, 300)
    x[0, 3] = 1.0 / 3.0
    x[2, 17] = 0.1
    x[3, 299] = 2.0
    xs = llp_hip.SparseRows(x)
    want = x[x != 0].to(torch.bfloat16).float()
    assert torch.equal(xs.val, want)
    assert not torch.equal(xs.val, x[x != 0])      # 1/3 and 0.1 are not exact in bf16


def test_loss_entry_points_keep_the_round3_signature():
    """llp_llp_loss has its round-3 argument list again (no term range); the term
    range lives in llp_llp_loss_range."""
    txt = open(HDR).read()
    import re as _re
    sig = _re.search(r"int llp_llp_loss\((.*?)\);", txt, _re.S).group(1)
    assert "term_b0" not in sig and sig.count(",") == 24
    rng = _re.search(r"int llp_llp_loss_range\((.*?)\);", txt, _re.S).group(1)
    assert "term_b0" in rng and rng.count(",") == 26
