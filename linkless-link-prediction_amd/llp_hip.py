"""ctypes binding of libllp_hip.so (the C ABI in include/llp_hip.h).

This is the only way the product reaches the GPU: every op below launches a
hand-written gfx950 kernel on torch's current HIP stream.  There is no CPU
fallback — if the library or a GPU is missing, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LLP_LIB", os.path.join(HERE, "libllp_hip.so"))   # LLP_LIB: an alternative build (A/B)

LLP_F32, LLP_BF16, LLP_MASK = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_RELU_BWD = 0, 1, 2
NORM_LAYER, NORM_BATCH = 1, 2

c_i64 = C.c_int64
c_int = C.c_int
c_f32 = C.c_float
c_f64 = C.c_double
c_vp = C.c_void_p
c_u64 = C.c_uint64


class Operand(C.Structure):
    _fields_ = [("ptr", c_vp), ("idx", c_vp), ("ptr2", c_vp), ("idx2", c_vp), ("ld", c_i64), ("ld2", c_i64),
                ("rows_dev", c_vp)]


class Dropout(C.Structure):
    _fields_ = [("p", c_f32), ("seed", c_u64), ("step_ctr", c_vp), ("stream_offset", c_i64)]


class HeadParts(C.Structure):
    """llp_head_parts: a gemm_nt_head's per-256-column partials [parts][ld] and the head bias."""
    _fields_ = [("part", c_vp), ("bias", c_vp), ("parts", c_i64), ("ld", c_i64)]


class TensorDesc(C.Structure):
    _fields_ = [("param", c_vp), ("grad", c_vp), ("exp_avg", c_vp), ("exp_avg_sq", c_vp), ("shadow", c_vp),
                ("shadow_t", c_vp), ("numel", c_i64), ("rows", c_i64), ("cols", c_i64), ("group", C.c_int32),
                ("shadow_dtype", C.c_int32), ("shadow_ld", c_i64), ("shadow_t_ld", c_i64)]


_SIGS = {
    "llp_version": (c_int, []),
    "llp_last_error": (C.c_char_p, []),
    "llp_last_gemm_kernel": (C.c_char_p, []),
    "llp_device_count": (c_int, []),
    "llp_gemm_nt": (c_int, [c_int, c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64, c_int,
                            c_vp, c_int, c_vp, c_i64, c_int, c_f32, C.POINTER(Dropout), c_vp]),
    "llp_gemm_nt_head_parts": (c_i64, [c_i64]),
    "llp_gemm_nt_head": (c_int, [c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64, c_vp, c_int,
                                 c_f32, C.POINTER(Dropout), c_vp, c_vp, c_vp]),
    "llp_head_finish": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_gemm_nt_splitk_plan": (c_int, [c_i64, c_i64, c_i64]),
    "llp_batch_slices": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp,
                                 c_i64, c_vp, c_vp, c_vp]),
    "llp_gemm_nt_splitk_ws_bytes": (c_i64, [c_i64, c_i64, c_int]),
    "llp_gemm_nt_splitk": (c_int, [c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64, c_vp,
                                   c_int, c_vp, c_i64, c_int, c_vp, c_i64, c_vp]),
    "llp_gemm_tn_workspace_bytes": (c_i64, [c_int, c_i64, c_i64, c_i64]),
    "llp_gemm_tn": (c_int, [c_int, c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64, c_int,
                            c_vp, c_vp, c_i64, c_vp]),
    "llp_gemm_tn_split": (c_int, [c_int, c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64,
                                  c_i64, c_vp, c_i64, c_int, c_vp, c_vp, c_i64, c_vp]),
    "llp_colsum_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_colsum": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_int, c_vp, c_i64, c_vp]),
    "llp_spmm_rows": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_i64, c_vp,
                              c_i64, c_vp]),
    "llp_spmm_tn": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, c_vp]),
    "llp_spmm_heavy_nnz": (c_int, []),
    "llp_gemm_nt_head_f32": (c_int, [c_i64, c_i64, c_i64, C.POINTER(Operand), C.POINTER(Operand), c_vp, c_i64, c_vp,
                                     c_vp, c_vp, c_vp]),
    "llp_spmm_rows_dt": (c_int, [c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_i64,
                                 c_vp, c_i64, c_vp]),
    "llp_spmm_tn_dt": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_int,
                               c_vp]),
    "llp_head_fwd": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_head_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_head_bwd": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_int, c_f32, c_vp, c_i64, c_vp, c_vp,
                             c_int, c_vp, c_i64, c_vp]),
    "llp_llp_loss_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_llp_loss": (c_int, [c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_f64, c_f64, c_f32, c_f32, c_f32, c_f32,
                             c_f32, c_f32, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_f64, c_vp, c_i64, c_vp]),
    "llp_llp_loss_range": (c_int, [c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_f64, c_f64, c_f32, c_f32, c_f32,
                                   c_f32, c_f32, c_f32, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_f64, c_i64, c_i64,
                                   c_vp, c_i64, c_vp]),
    "llp_llp_loss_heads": (c_int, [c_i64, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_f64, c_f64, c_f32, c_f32, c_f32,
                                   c_f32, c_f32, c_f32, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_f64, c_i64, c_i64,
                                   c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "llp_pair_owner_workspace_bytes": (c_i64, [c_i64, c_i64, c_i64, c_int]),
    "llp_pair_owner_assign": (c_int, [c_int, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                      c_vp]),
    "llp_pair_owner_scatter": (c_int, [c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_hadamard_bwd_blocks": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_dedup_rows_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_dedup_rows": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "llp_dedup_rows2_state_bytes": (c_i64, [c_i64]),
    "llp_dedup_rows2_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_dedup_rows2": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp,
                                c_i64, c_vp]),
    "llp_segment_sum_rows": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_int, c_vp, c_vp,
                                     c_vp]),
    "llp_hadamard_bwd_segments": (c_int, [c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                          c_vp, c_i64, c_int, c_vp, c_vp, c_vp]),
    "llp_gather_i32": (c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_gather_rows": (c_int, [c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "llp_minibatch_sample": (c_int, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int, c_u64, c_vp,
                                     c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp]),
    "llp_hadamard_bwd_scatter": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_context_sampler": (c_int, [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int, c_u64, c_vp,
                                    c_i64, c_vp, c_vp]),
    "llp_randint_pairs": (c_int, [c_i64, c_i64, c_i64, c_i64, c_u64, c_vp, c_i64, c_vp, c_vp]),
    "llp_build_targets": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp,
                                  c_vp]),
    "llp_pair_index_from_samples": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_neg_sample_dense_workspace_bytes": (c_i64, [c_i64]),
    "llp_neg_sample_dense2_state_bytes": (c_i64, [c_i64]),
    "llp_neg_sample_dense2_workspace_bytes": (c_i64, [c_i64]),
    "llp_neg_sample_dense2": (c_int, [c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_u64, c_vp, c_i64, c_vp,
                                      c_i64, c_vp, c_int, c_vp, c_i64, c_vp]),
    "llp_neg_sample_dense": (c_int, [c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_u64, c_vp, c_i64, c_vp,
                                     c_i64, c_vp, c_vp, c_i64, c_vp]),
    "llp_edge_table_size": (c_i64, [c_i64]),
    "llp_edge_table_build": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp]),
    "llp_fullbatch_pairs": (c_int, [c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp,
                                    c_vp]),
    "llp_kd_terms_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_kd_terms": (c_int, [c_int, c_i64, c_vp, c_vp, c_f64, c_f32, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp,
                             c_f64, c_f32, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "llp_hits_at_k": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_int, c_vp, c_vp]),
    "llp_auc_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_auc": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "llp_csr_aggregate": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_int, c_vp, c_i64, c_int, c_vp]),
    "llp_gcn_aggregate": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "llp_grad_sumsq_workspace_bytes": (c_i64, [c_int, c_i64]),
    "llp_grad_sumsq": (c_int, [c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_i64, c_vp]),
    "llp_adam_step": (c_int, [c_vp, c_int, c_i64, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "llp_grad_sumsq_t": (c_int, [c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "llp_adam_step_t": (c_int, [c_vp, c_int, c_i64, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "llp_refresh_shadows": (c_int, [c_vp, c_int, c_i64, c_vp]),
    "llp_grad_sumsq_work_items": (c_i64, [c_i64]),
    "llp_adam_work_items": (c_i64, [c_i64, c_i64, c_i64, c_int]),
    "llp_grad_sumsq_w": (c_int, [c_vp, c_int, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "llp_adam_step_w": (c_int, [c_vp, c_int, c_i64, c_i64, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp]),
    "llp_convert": (c_int, [c_int, c_int, c_i64, c_vp, c_vp, c_vp]),
    "llp_accumulate": (c_int, [c_i64, c_vp, c_f32, c_vp, c_vp]),
    "llp_increment": (c_int, [c_vp, c_vp]),
    "llp_step_end": (c_int, [c_vp, c_f32, c_vp, c_vp, c_vp]),
    "llp_step_end2": (c_int, [c_vp, c_f32, c_vp, c_vp, c_vp, c_vp]),
    "llp_zero": (c_int, [c_vp, c_i64, c_vp]),
    "llp_hadamard_rows": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_relu_bwd": (c_int, [c_int, c_i64, c_vp, c_vp, c_f32, c_vp, c_vp]),
    "llp_act_2d": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_int, C.POINTER(Dropout), c_vp]),
    "llp_relu_bwd_2d": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_f32, c_vp, c_i64, c_vp]),
    "llp_transpose": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "llp_mul": (c_int, [c_int, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_row_scale": (c_int, [c_int, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_sigmoid_bwd": (c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_mfma_probe": (c_int, [c_vp, c_i64, c_i64, c_vp, C.POINTER(c_f64), c_vp]),
    "llp_mfma_probe_out_floats": (c_i64, []),
    "llp_mfma_probe_f32": (c_int, [c_vp, c_i64, c_i64, c_vp, C.POINTER(c_f64), c_vp]),
    "llp_stage_probe": (c_int, [c_int, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "llp_gemm_nt_w4_probe": (c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_int, c_f32,
                                     c_vp, c_vp, c_i64, c_int, c_vp]),
    "llp_norm_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "llp_norm_colsums": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "llp_norm_fwd": (c_int, [c_int, c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_f32, c_int, c_vp, c_f64, c_f32,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_int, C.POINTER(Dropout), c_vp, c_i64, c_vp]),
    "llp_norm_bwd_sums": (c_int, [c_int, c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_f32, c_vp, c_i64, c_vp,
                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "llp_norm_bwd": (c_int, [c_int, c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_f32, c_vp, c_i64, c_vp, c_vp,
                             c_vp, c_f64, c_vp, c_vp, c_i64, c_vp]),
}

_lib = None


def load(path: str = LIB_PATH):
    """dlopen the library (works without a GPU: no compute call is made)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise RuntimeError(f"libllp_hip.so not found at {path}: run `python build_lib.py` (or "
                               f"__graft_entry__.build()) first — there is no CPU fallback")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def lib():
    """The library, for compute: requires a visible GPU."""
    L = load()
    if not torch.cuda.is_available():
        raise RuntimeError("libllp_hip: no HIP device visible — the LLP hot path runs only on MI355X (gfx950)")
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.llp_last_error().decode() if _lib else ""
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def last_gemm_kernel() -> str:
    """The NT GEMM kernel the last gemm_nt call on this thread launched (llp_last_gemm_kernel)."""
    return lib().llp_last_gemm_kernel().decode()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return LLP_F32
    if t == torch.bfloat16:
        return LLP_BF16
    raise TypeError(f"unsupported dtype {t}")


def operand(t, idx=None, t2=None, idx2=None, count=None) -> Operand:
    """Operand over the row-major 2-D tensor ``t`` (rows optionally gathered by
    int32 ``idx``), optionally times ``t2[idx2]`` elementwise.  ``count``: an
    int32 device scalar; the GEMM then runs on min(M, count) rows without a
    host read (llp_operand.rows_dev)."""
    assert t.dim() == 2 and t.stride(1) == 1
    if idx is not None:
        assert idx.dtype == torch.int32 and idx.is_contiguous()
    if count is not None:
        assert count.dtype == torch.int32 and count.device == t.device
    o = Operand(t.data_ptr(), ptr(idx), ptr(t2), ptr(idx2), t.stride(0), t2.stride(0) if t2 is not None else 0,
                ptr(count))
    o._keep = (t, idx, t2, idx2, count)   # the struct holds raw pointers: keep the tensors alive with it
    return o


# ------------------------------------------------------------------ op wrappers
def gemm_nt(A: Operand, B: Operand, M, N, K, C_out, dtype, bias=None, act=ACT_NONE, aux=None, alpha=1.0,
            dropout: Dropout | None = None):
    L = lib()
    # a uint8 aux is a ReLU bit mask [M, N/8]: written by act=RELU, read by act=RELU_BWD
    aux_code = 0 if aux is None else (LLP_MASK if aux.dtype == torch.uint8 else dtype_code(aux.dtype))
    check(L.llp_gemm_nt(dtype, M, N, K, C.byref(A), C.byref(B), C_out.data_ptr(), C_out.stride(0),
                        dtype_code(C_out.dtype), ptr(bias), act, ptr(aux), aux.stride(0) if aux is not None else 0,
                        aux_code, alpha,
                        C.byref(dropout) if dropout is not None else None, stream_ptr()), "llp_gemm_nt")


def head_parts(N):
    return load().llp_gemm_nt_head_parts(N)


def gemm_nt_splitk_plan(M, N, K):
    """Split count for llp_gemm_nt_splitk (1: the plain llp_gemm_nt is the better launch).
    Host arithmetic only (the CU count falls back to 256 without a device)."""
    return load().llp_gemm_nt_splitk_plan(M, N, K)


def gemm_nt_splitk_ws_bytes(M, N, splits):
    return load().llp_gemm_nt_splitk_ws_bytes(M, N, splits)


def gemm_nt_splitk(A: Operand, B: Operand, M, N, K, C_out, splits, ws, bias=None, act=ACT_NONE, mask=None):
    """bf16 split-K GEMM: C = act(A.B^T + bias) with an optional ReLU bit mask [M, N/8]."""
    L = lib()
    check(L.llp_gemm_nt_splitk(M, N, K, C.byref(A), C.byref(B), C_out.data_ptr(), C_out.stride(0), ptr(bias), act,
                               ptr(mask), mask.stride(0) if mask is not None else 0, splits, ws.data_ptr(),
                               ws.numel() * ws.element_size(), stream_ptr()), "llp_gemm_nt_splitk")


def gemm_nt_head(A: Operand, B: Operand, M, N, K, C_out, head_w, head_part, bias=None, act=ACT_RELU, alpha=1.0,
                 dropout: Dropout | None = None):
    """bf16 GEMM with the Linear(N,1) head fused (C_out may be None)."""
    L = lib()
    check(L.llp_gemm_nt_head(M, N, K, C.byref(A), C.byref(B), ptr(C_out), C_out.stride(0) if C_out is not None else 0,
                             ptr(bias), act, alpha, C.byref(dropout) if dropout is not None else None, head_w.data_ptr(),
                             head_part.data_ptr(), stream_ptr()), "llp_gemm_nt_head")


def gemm_nt_head_f32(A: Operand, B: Operand, M, N, K, C_out, head_w, head_part, bias=None):
    """f32 GEMM + ReLU with the Linear(N,1) head's per-256-column partials fused (llp_gemm_nt_head_f32)."""
    L = lib()
    check(L.llp_gemm_nt_head_f32(M, N, K, C.byref(A), C.byref(B), C_out.data_ptr(), C_out.stride(0), ptr(bias),
                                 head_w.data_ptr(), head_part.data_ptr(), stream_ptr()), "llp_gemm_nt_head_f32")


def head_finish(parts, M, head_part, b, logit=None, prob=None):
    L = lib()
    check(L.llp_head_finish(parts, M, head_part.data_ptr(), ptr(b), ptr(logit), ptr(prob), stream_ptr()),
          "llp_head_finish")


def gemm_tn_ws_bytes(dtype, M, P, Q):
    return load().llp_gemm_tn_workspace_bytes(dtype, M, P, Q)


def gemm_tn(A: Operand, B: Operand, M, P, Q, C_out, dtype, ws, accumulate=False, colsum_a=None, split=None):
    """C_out (+)= A^T B (f32).  split=(q, C2): columns [q, Q) go to C2 instead (llp_gemm_tn_split;
    C_out then holds the first q columns)."""
    L = lib()
    if split is not None:
        q, C2 = split
        check(L.llp_gemm_tn_split(dtype, M, P, Q, C.byref(A), C.byref(B), C_out.data_ptr(), C_out.stride(0), q,
                                  C2.data_ptr(), C2.stride(0), int(accumulate), ptr(colsum_a), ws.data_ptr(),
                                  ws.numel() * ws.element_size(), stream_ptr()), "llp_gemm_tn_split")
        return
    check(L.llp_gemm_tn(dtype, M, P, Q, C.byref(A), C.byref(B), C_out.data_ptr(), C_out.stride(0), int(accumulate),
                        ptr(colsum_a), ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()), "llp_gemm_tn")


def colsum_ws_bytes(M, N):
    return load().llp_colsum_workspace_bytes(M, N)


def colsum(Y, M, N, out, ws, accumulate=False):
    L = lib()
    check(L.llp_colsum(dtype_code(Y.dtype), M, N, Y.data_ptr(), Y.stride(0), out.data_ptr(), int(accumulate),
                       ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()), "llp_colsum")


class SparseRows:
    """A constant sparse matrix x [N, F] on the device for llp_spmm_rows / llp_spmm_tn: CSR
    (rowptr, colidx, val; val None when every stored value is 1) and, per row slice, its CSC
    (csc(r0, n): colptr, rowidx local to the slice, ascending within a column, val).  Built once
    from the dense x with torch (setup plumbing, not the step)."""

    def __init__(self, x, round_bf16=True):
        assert x.dim() == 2
        self.N, self.F = x.shape
        nz = torch.nonzero(x)                                   # row-major order: rows, then columns
        self.nnz = int(nz.shape[0])
        assert self.nnz < 2 ** 31
        counts = torch.bincount(nz[:, 0], minlength=self.N)
        self.rowptr = torch.zeros(self.N + 1, dtype=torch.int64, device=x.device)
        self.rowptr[1:] = torch.cumsum(counts, 0)
        self.rowptr_host = self.rowptr.cpu()
        self.rowptr = self.rowptr.to(torch.int32)
        self.colidx = nz[:, 1].to(torch.int32).contiguous()
        # rounded through bf16 as the dense first layer reads x (its bf16 copy): the sparse and the
        # dense path then multiply the same values for non-binary features too
        # (round_bf16=False: the fp32 engine, whose dense path reads x in f32)
        v = x[nz[:, 0], nz[:, 1]].float()
        v = (v.to(torch.bfloat16).float() if round_bf16 else v).contiguous()
        self.val = None if bool((v == 1).all()) else v
        self._csc = {}

    def csc(self, r0, n):
        key = (int(r0), int(n))
        c = self._csc.get(key)
        if c is None:
            k0, k1 = int(self.rowptr_host[r0]), int(self.rowptr_host[r0 + n])
            rows = torch.repeat_interleave(torch.arange(n, device=self.colidx.device, dtype=torch.int32),
                                           (self.rowptr[r0 + 1:r0 + n + 1] - self.rowptr[r0:r0 + n]).long())
            cols = self.colidx[k0:k1].long()
            order = torch.sort(cols, stable=True).indices        # ascending rows kept within a column
            cnt = torch.bincount(cols, minlength=self.F)
            colptr = torch.zeros(self.F + 1, dtype=torch.int64, device=cols.device)
            colptr[1:] = torch.cumsum(cnt, 0)
            # llp_spmm_tn's schedule: most nonzeros first (ties by feature), the heavy ones counted
            perm = torch.sort(-cnt, stable=True).indices
            n_heavy = int((cnt >= load().llp_spmm_heavy_nnz()).sum())
            c = (colptr.to(torch.int32), rows[order].contiguous(),
                 None if self.val is None else self.val[k0:k1][order].contiguous(), perm.to(torch.int32), n_heavy)
            self._csc[key] = c
        return c


def spmm_rows(xs, rows, row0, Wt, bias, Y, act=ACT_NONE, mask=None):
    """Y[:rows] = act(x[row0:row0+rows] @ Wt + bias) (llp_spmm_rows_dt); Wt [F, H] and Y bf16 or f32
    (the same dtype)."""
    L = lib()
    H = Wt.shape[1]
    assert Y.dtype == Wt.dtype
    check(L.llp_spmm_rows_dt(dtype_code(Wt.dtype), rows, row0, H, xs.rowptr.data_ptr(), xs.colidx.data_ptr(),
                             ptr(xs.val), Wt.data_ptr(), Wt.stride(0), ptr(bias), act, Y.data_ptr(), Y.stride(0),
                             ptr(mask), mask.stride(0) if mask is not None else 0, stream_ptr()), "llp_spmm_rows")


def spmm_tn(xs, r0, n, dY, dW, accumulate=False):
    """dW (+)= dY[:n]^T @ x[r0:r0+n] (llp_spmm_tn_dt); dY bf16 or f32, dW f32 [H, F] (row stride >= F)."""
    L = lib()
    colptr, rowidx, val, perm, n_heavy = xs.csc(r0, n)
    check(L.llp_spmm_tn_dt(dtype_code(dY.dtype), xs.F, dY.shape[1], colptr.data_ptr(), rowidx.data_ptr(), ptr(val),
                           perm.data_ptr(), n_heavy, dY.data_ptr(), dY.stride(0), dW.data_ptr(), dW.stride(0),
                           int(accumulate), stream_ptr()), "llp_spmm_tn")


def head_fwd(Z, R, H, w, b, logit=None, prob=None, Z2=None, iz=None, iz2=None):
    L = lib()
    check(L.llp_head_fwd(dtype_code(Z.dtype), R, H, Z.data_ptr(), Z.stride(0), ptr(Z2),
                         Z2.stride(0) if Z2 is not None else 0, ptr(iz), ptr(iz2), ptr(w), ptr(b), ptr(logit),
                         ptr(prob), stream_ptr()), "llp_head_fwd")


def head_bwd_ws_bytes(R, H):
    return load().llp_head_bwd_workspace_bytes(R, H)


def head_bwd(dlogit, Z, R, H, w, relu_mask, dZ, dw, db, ws, accumulate=False, alpha=1.0):
    L = lib()
    check(L.llp_head_bwd(dtype_code(Z.dtype), R, H, dlogit.data_ptr(), Z.data_ptr(), Z.stride(0), ptr(w),
                         int(relu_mask), alpha, ptr(dZ), dZ.stride(0) if dZ is not None else 0, ptr(dw), ptr(db),
                         int(accumulate), ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()),
          "llp_head_bwd")


def llp_loss_ws_bytes(B, n_lab):
    return load().llp_llp_loss_workspace_bytes(B, n_lab)


def head_in(part, parts, ld, bias):
    """HeadParts of a gemm_nt_head partial buffer (finished inside llp_loss)."""
    return HeadParts(part.data_ptr(), ptr(bias), int(parts), int(ld))


def llp_loss(B, Cc, s_logit, t_prob, n_lab, n_pos, out_logit, B_total, n_lab_total, margin, T, w_label, w_d, w_r,
             dlogit_ctx, dlogit_lab, terms, ws, accumulate=False, loss_scale=1.0, neg_count=None, neg_offset=0,
             pos_total=0.0, term_range=None, s_head=None, t_head=None, ticket=None):
    """neg_count: the dense negatives' int32 device count (label slots past it inert, the BCE
    mean over pos_total + count labels); n_lab_total is then unused.  term_range (b0, b1): the
    anchors whose KL / rank terms are reported (default all B; every gradient is written).
    s_head / t_head (HeadParts): the student / teacher logits finished inside the loss launch and
    written to s_logit + out_logit / t_prob; ticket (int32 device word, zero, left zero): the
    terms are finalised by the launch's last workgroup (one launch in all)."""
    L = lib()
    tb0, tb1 = (0, B) if term_range is None else term_range
    check(L.llp_llp_loss_heads(B, Cc, ptr(s_logit), ptr(t_prob), n_lab, n_pos, ptr(out_logit), float(B_total),
                               float(n_lab_total), margin, T, w_label, w_d, w_r, loss_scale, ptr(dlogit_ctx),
                               ptr(dlogit_lab), terms.data_ptr(), int(accumulate), ptr(neg_count), int(neg_offset),
                               float(pos_total), int(tb0), int(tb1),
                               C.byref(s_head) if s_head is not None else None,
                               C.byref(t_head) if t_head is not None else None, ptr(ticket),
                               ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()),
          "llp_llp_loss")


class OwnerCat(C.Structure):
    """llp_owner_cat: one category of pairs for llp_pair_owner_assign; end e of item i is
    e[(i // kc) * kld + koff + (i % kc) * kstep]."""
    _fields_ = [("a", c_vp), ("a_kc", c_i64), ("a_kld", c_i64), ("a_koff", c_i64), ("a_kstep", c_i64), ("b", c_vp),
                ("b_kc", c_i64), ("b_kld", c_i64), ("b_koff", c_i64), ("b_kstep", c_i64), ("key_b", C.c_int32),
                ("pad", C.c_int32), ("n", c_i64)]


def owner_cat(n, a, b, a_view=None, b_view=None, key_b=False):
    """a / b: int32 tensors of node ids; *_view = (kc, kld, koff, kstep) strided view (default
    contiguous: (1, 1, 0, 0))."""
    av = a_view or (1, 1, 0, 0)
    bv = b_view or (1, 1, 0, 0)
    c = OwnerCat(ptr(a), *av, ptr(b), *bv, int(bool(key_b)), 0, int(n))
    c._keep = (a, b)
    return c


def pair_owner_ws_bytes(ns, world):
    ns = list(ns) + [0] * (3 - len(ns))
    return load().llp_pair_owner_workspace_bytes(ns[0], ns[1], ns[2], int(world))


def pair_owner_assign(cats, num_nodes, world, rank, sel, ws, gpos=None, target=None, R2=0, owner_tab=None):
    """llp_pair_owner_assign over 1-3 OwnerCat categories: sel (int32[sum n]) holds rank r's items
    of each category at [cat base + r n / world, ...); gpos (int32[sum n], optional) item -> slot;
    target (int32[2 R2], optional) = this rank's pairs' [a ends | b ends] in its order;
    owner_tab (int32[N], optional): node -> owner rank (default node // ceil(N / world))."""
    arr = (OwnerCat * len(cats))(*cats)
    check(lib().llp_pair_owner_assign(len(cats), C.cast(arr, c_vp), int(num_nodes), int(world), int(rank),
                                      ptr(owner_tab), sel.data_ptr(), ptr(gpos), ptr(target), int(R2), ws.data_ptr(),
                                      ws.numel() * ws.element_size(), stream_ptr()),
          "llp_pair_owner_assign")


def pair_owner_scatter(n, gpos, lo, hi, s_loc, t_loc, s_full, t_full):
    """s_full[i] = s_loc[gpos[i] - lo] when lo <= gpos[i] < hi else 0 (t likewise; either may be None)."""
    check(lib().llp_pair_owner_scatter(int(n), gpos.data_ptr(), int(lo), int(hi), ptr(s_loc), ptr(t_loc),
                                       ptr(s_full), ptr(t_full), stream_ptr()), "llp_pair_owner_scatter")


def hadamard_bwd_blocks(B, Cc, L2, H, dZ, h, dh, drow=None, hidx=None):
    L = lib()
    check(L.llp_hadamard_bwd_blocks(dtype_code(h.dtype), B, Cc, L2, H, ptr(dZ), ptr(drow), h.data_ptr(), ptr(hidx),
                                    dh.data_ptr(), stream_ptr()), "llp_hadamard_bwd_blocks")


def dedup_ws_bytes(num_nodes, R):
    return load().llp_dedup_rows_workspace_bytes(num_nodes, R)


def dedup_rows(num_nodes, R, target, uniq, pos, n_unique, seg_ptr, seg_rows, ws):
    L = lib()
    check(L.llp_dedup_rows(num_nodes, R, target.data_ptr(), uniq.data_ptr(), pos.data_ptr(), n_unique.data_ptr(),
                           seg_ptr.data_ptr(), seg_rows.data_ptr(), ws.data_ptr(), ws.numel() * ws.element_size(),
                           stream_ptr()), "llp_dedup_rows")


class DedupWorkspace:
    """The workspace of llp_dedup_rows2 for one num_nodes, with the clean-state bookkeeping:
    the first call zeroes the persistent state, later calls vouch for it."""

    def __init__(self, num_nodes, R, device):
        import torch
        self.num_nodes = int(num_nodes)
        self.R = int(R)
        nbytes = load().llp_dedup_rows2_workspace_bytes(self.num_nodes, self.R)
        self.buf = torch.empty(nbytes // 4 + 16, dtype=torch.float32, device=device)
        self.clean = False

    def fits(self, num_nodes, R):
        return int(num_nodes) == self.num_nodes and int(R) <= self.R

    def _state_bytes(self):
        return load().llp_dedup_rows2_state_bytes(self.num_nodes)

    def error_word(self):
        """Word [2] of the control block (nonzero: a look-back timed out; that call's outputs are
        invalid, though every write stayed in bounds)."""
        off = self._state_bytes() - 256
        return self.buf.view(-1)[off // 4 + 2].view(torch.int32)

    def reset(self):
        """Zero the persistent state (counts, look-back flags, control words) in place: valid for
        calls already captured in a graph too (zero is the state every call starts from)."""
        self.buf[:self._state_bytes() // 4].zero_()


def dedup_rows2(num_nodes, R, target, uniq, pos, n_unique, seg_ptr, seg_rows, dws, zero_rows=None):
    """llp_dedup_rows2 (four launches, same outputs as dedup_rows) on a DedupWorkspace;
    zero_rows (2-D, may be None): rows of nodes absent from target are zeroed."""
    L = lib()
    zr = 0 if zero_rows is None else zero_rows.stride(0) * zero_rows.element_size()
    zb = 0 if zero_rows is None else zero_rows.shape[1] * zero_rows.element_size()
    check(L.llp_dedup_rows2(num_nodes, R, ptr(target), ptr(uniq), ptr(pos), ptr(n_unique), ptr(seg_ptr),
                            ptr(seg_rows), ptr(zero_rows), zr, zb, int(dws.clean), dws.buf.data_ptr(),
                            dws.buf.numel() * dws.buf.element_size(), stream_ptr()), "llp_dedup_rows2")
    dws.clean = True


def segment_sum_rows(U, seg_ptr, rows, src, out, count=None, out_rows=None):
    """out[u] (out[out_rows[u]] with ``out_rows``) = sum of src[rows[seg_ptr[u]:seg_ptr[u+1]]]
    for u < U (u < min(U, count) with an int32 device ``count``); ``out`` in src's dtype
    or f32 (unrounded sums)."""
    L = lib()
    check(L.llp_segment_sum_rows(dtype_code(src.dtype), U, src.shape[1], seg_ptr.data_ptr(), rows.data_ptr(),
                                 src.data_ptr(), src.stride(0), out.data_ptr(), out.stride(0), dtype_code(out.dtype),
                                 ptr(out_rows), ptr(count), stream_ptr()), "llp_segment_sum_rows")


def hadamard_bwd_segments(U, B, C, L2, H, seg_ptr, rows, pos, dZ, h, dh, anchor_rows, drow=None, count=None,
                          out_rows=None):
    """dh[u] (U x H; dh[out_rows[u]] with ``out_rows``) = per-node sum of the Hadamard-backward
    rows (llp_hadamard_bwd_segments), in dh's dtype (h's, or f32); anchor_rows: [B, H] scratch
    of h's dtype (None when B = 0)."""
    L = lib()
    t = dZ if dZ is not None else h
    check(L.llp_hadamard_bwd_segments(dtype_code(t.dtype), U, B, C, L2, H, seg_ptr.data_ptr(), rows.data_ptr(),
                                      pos.data_ptr(), ptr(dZ), ptr(drow), h.data_ptr(), ptr(anchor_rows),
                                      dh.data_ptr(), dh.stride(0), dtype_code(dh.dtype), ptr(out_rows), ptr(count),
                                      stream_ptr()),
          "llp_hadamard_bwd_segments")


def gather_i32(idx, src, out):
    L = lib()
    check(L.llp_gather_i32(idx.numel(), idx.data_ptr(), src.data_ptr(), out.data_ptr(), stream_ptr()),
          "llp_gather_i32")


def gather_rows(src, idx, out, count=None):
    """out[r] = src[idx[r]] for r < min(out rows, *count) (count: device int32[1] or None)."""
    L = lib()
    n = out.shape[0]
    rb = out.shape[1] * out.element_size()
    check(L.llp_gather_rows(n, rb, idx.data_ptr(), src.data_ptr(), src.stride(0) * src.element_size(),
                            out.data_ptr(), out.stride(0) * out.element_size(), ptr(count), stream_ptr()),
          "llp_gather_rows")


def hadamard_rows(a, ia, b, ib, out):
    L = lib()
    R, H = out.shape
    check(L.llp_hadamard_rows(dtype_code(a.dtype), R, H, a.data_ptr(), ptr(ia), b.data_ptr(), ptr(ib),
                              out.data_ptr(), stream_ptr()), "llp_hadamard_rows")


def hadamard_bwd_scatter(R, H, dZ, ia, ib, h, dh, drow=None):
    L = lib()
    check(L.llp_hadamard_bwd_scatter(dtype_code(h.dtype), R, H, ptr(dZ), ptr(drow), ia.data_ptr(), ib.data_ptr(),
                                     h.data_ptr(), dh.data_ptr(), stream_ptr()), "llp_hadamard_bwd_scatter")


def context_sampler(rowptr, col, num_nodes, start, B, ps_method, rw_step, hops, ns_rate, seed, step_ctr,
                    stream_offset, samples, b_offset=0):
    L = lib()
    check(L.llp_context_sampler(rowptr.data_ptr(), col.data_ptr(), num_nodes, start.data_ptr(), B, b_offset,
                                1 if ps_method == "nb" else 0, rw_step, hops, ns_rate, seed, step_ctr.data_ptr(),
                                stream_offset, samples.data_ptr(), stream_ptr()), "llp_context_sampler")


def minibatch_sample(rowptr, col, num_nodes, start, B, ps_method, rw_step, hops, ns_rate, seed, step_ctr,
                     stream_offset, pairs, perm, P, P_total, p_offset, neg_stream_offset, samples, neg, target, t_ia,
                     t_ib, b_offset=0):
    """context_sampler + randint_pairs + build_targets + pair_index_from_samples in one launch."""
    L = lib()
    check(L.llp_minibatch_sample(rowptr.data_ptr(), col.data_ptr(), num_nodes, start.data_ptr(), B, b_offset,
                                 1 if ps_method == "nb" else 0, rw_step, hops, ns_rate, seed, step_ctr.data_ptr(),
                                 stream_offset, pairs.data_ptr(), perm.data_ptr(), P, P_total, p_offset,
                                 neg_stream_offset, samples.data_ptr(), neg.data_ptr(), target.data_ptr(),
                                 ptr(t_ia), ptr(t_ib), stream_ptr()), "llp_minibatch_sample")


def randint_pairs(num_nodes, n, seed, step_ctr, stream_offset, out, n_total=None, offset=0):
    L = lib()
    n_total = n if n_total is None else n_total
    check(L.llp_randint_pairs(num_nodes, n, n_total, offset, seed, step_ctr.data_ptr(), stream_offset,
                              out.data_ptr(), stream_ptr()), "llp_randint_pairs")


def build_targets(B, C1, samples, pairs, perm, step_ctr, perm_stride, P, neg, target, n_neg=None):
    """neg: int32[2, ld] view whose first n_neg (default P) columns are used."""
    L = lib()
    n_neg = P if n_neg is None else int(n_neg)
    check(L.llp_build_targets(B, C1, samples.data_ptr(), pairs.data_ptr(), perm.data_ptr(), ptr(step_ctr),
                              perm_stride, P, ptr(neg), n_neg, neg.stride(0) if neg is not None else 0,
                              target.data_ptr(), stream_ptr()), "llp_build_targets")


def pair_index_from_samples(B, Cc, samples, ia, ib):
    L = lib()
    check(L.llp_pair_index_from_samples(B, Cc, samples.data_ptr(), ia.data_ptr(), ib.data_ptr(), stream_ptr()),
          "llp_pair_index_from_samples")


def neg_sample_ws_bytes(max_candidates):
    return load().llp_neg_sample_dense_workspace_bytes(max_candidates)


def neg_sample_dense(num_nodes, edge_keys, num_neg, sample_size, seed, step_ctr, stream_offset, out, count, ws,
                     rounds=3, edge_table=None):
    """out: int32[2, ld] (ld >= num_neg); count: int32[1] on the device; edge_table: the keys'
    set from edge_table_build (then used for the membership test)."""
    L = lib()
    check(L.llp_neg_sample_dense(num_nodes, ptr(edge_keys), 0 if edge_keys is None else edge_keys.numel(),
                                 ptr(edge_table), 0 if edge_table is None else edge_table.numel(), num_neg,
                                 sample_size, rounds, seed, step_ctr.data_ptr(), stream_offset, out.data_ptr(),
                                 out.stride(0), count.data_ptr(), ws.data_ptr(), ws.numel() * ws.element_size(),
                                 stream_ptr()), "llp_neg_sample_dense")


class StatefulWorkspace:
    """A workspace whose leading state persists between calls of one llp_* entry point (the
    two-launch dense sampler, ...): the first call clears it (state_clean = 0), later calls
    vouch for it."""

    def __init__(self, nbytes, key, device, state_bytes=None):
        """state_bytes: the leading state's size (its last 256 bytes the control block, word [2]
        the look-back error word), for error_word / reset; None: neither is available."""
        import torch
        self.key = key
        self.buf = torch.empty(int(nbytes) // 4 + 16, dtype=torch.float32, device=device)
        self.clean = False
        self.state_bytes = None if state_bytes is None else int(state_bytes)

    def error_word(self):
        """Word [2] of the control block (nonzero: a look-back of some call timed out), or None."""
        if self.state_bytes is None:
            return None
        return self.buf.view(-1)[(self.state_bytes - 256) // 4 + 2].view(torch.int32)

    def reset(self):
        """Zero the persistent state in place (valid for captured calls too)."""
        if self.state_bytes is not None:
            self.buf[:self.state_bytes // 4].zero_()
        else:
            self.clean = False


def neg_sample_dense2(num_nodes, edge_keys, num_neg, sample_size, seed, step_ctr, stream_offset, out, count, sws,
                      rounds=3, edge_table=None):
    """llp_neg_sample_dense2 (two launches, the same outputs as neg_sample_dense) on a
    StatefulWorkspace sized by neg_sample2_ws_bytes(max_candidates)."""
    L = lib()
    check(L.llp_neg_sample_dense2(num_nodes, ptr(edge_keys), 0 if edge_keys is None else edge_keys.numel(),
                                  ptr(edge_table), 0 if edge_table is None else edge_table.numel(), num_neg,
                                  sample_size, rounds, seed, step_ctr.data_ptr(), stream_offset, out.data_ptr(),
                                  out.stride(0), count.data_ptr(), int(sws.clean), sws.buf.data_ptr(),
                                  sws.buf.numel() * sws.buf.element_size(), stream_ptr()), "llp_neg_sample_dense2")
    sws.clean = True


def neg_sample2_ws_bytes(max_candidates):
    return load().llp_neg_sample_dense2_workspace_bytes(max_candidates)


def neg_sample2_state_bytes(max_candidates):
    return load().llp_neg_sample_dense2_state_bytes(max_candidates)


def edge_table_build(edge_keys):
    """The sorted int64 edge keys' open-addressing set (int64 [llp_edge_table_size] on their device)."""
    L = lib()
    n = edge_keys.numel()
    t = torch.empty(int(L.llp_edge_table_size(n)), dtype=torch.int64, device=edge_keys.device)
    check(L.llp_edge_table_build(ptr(edge_keys), n, t.data_ptr(), t.numel(), stream_ptr()), "llp_edge_table_build")
    return t


def batch_slices(perm_a, stride_a, off_a, out_a, perm_b, stride_b, off_b, out_b, n_batches, step_ctr,
                 ctr_offset=0):
    """llp_batch_slices: out_a = perm_a[j*stride_a + off_a :][:len(out_a)], out_b likewise, with
    j = (step_ctr + ctr_offset) mod n_batches read on the device (a hipGraph feeds itself)."""
    L = lib()
    check(L.llp_batch_slices(ptr(perm_a), int(stride_a), int(off_a), out_a.numel(), ptr(perm_b), int(stride_b),
                             int(off_b), out_b.numel(), int(n_batches), perm_a.numel(), perm_b.numel(),
                             step_ctr.data_ptr(), int(ctr_offset), ptr(out_a), ptr(out_b), stream_ptr()),
          "llp_batch_slices")


def fullbatch_pairs(B, C1, samples, pairs, perm, P, neg, n_neg, ia, ib, neg_count=None, neg_offset=0):
    L = lib()
    check(L.llp_fullbatch_pairs(B, C1, ptr(samples), ptr(pairs), ptr(perm), P, ptr(neg),
                                neg.stride(0) if neg is not None else 0, n_neg, ptr(neg_count), int(neg_offset),
                                ia.data_ptr(), ib.data_ptr(), stream_ptr()), "llp_fullbatch_pairs")


def kd_terms_ws_bytes(B_rm, n_lab):
    return load().llp_kd_terms_workspace_bytes(B_rm, n_lab)


def kd_terms(terms, ws, n_lab=0, out_logit=None, t_prob_lab=None, n_lab_total=1.0, w_lm=0.0, dlogit_lab=None,
             B_rm=0, h=None, t_h=None, idx_rm=None, B_rm_total=1.0, w_rm=0.0, dh=None, loss_scale=1.0):
    L = lib()
    dc = dtype_code(h.dtype) if h is not None else LLP_F32
    H = h.shape[1] if h is not None else 0
    check(L.llp_kd_terms(dc, n_lab, ptr(out_logit), ptr(t_prob_lab), float(n_lab_total), float(w_lm), B_rm, H, ptr(h),
                         h.stride(0) if h is not None else 0, ptr(t_h), t_h.stride(0) if t_h is not None else 0,
                         ptr(idx_rm), float(B_rm_total), float(w_rm), float(loss_scale), ptr(dlogit_lab), ptr(dh),
                         dh.stride(0) if dh is not None else 0, terms.data_ptr(), ws.data_ptr(),
                         ws.numel() * ws.element_size(), stream_ptr()), "llp_kd_terms")


def act_2d(x, y, act=ACT_RELU, dropout: Dropout | None = None):
    """y = dropout(act(x)) on (strided) 2-D views of equal shape."""
    L = lib()
    check(L.llp_act_2d(dtype_code(x.dtype), x.shape[0], x.shape[1], x.data_ptr(), x.stride(0), y.data_ptr(),
                       y.stride(0), act, C.byref(dropout) if dropout is not None else None, stream_ptr()),
          "llp_act_2d")


def relu_bwd_2d(gy, y, alpha, out):
    L = lib()
    check(L.llp_relu_bwd_2d(dtype_code(gy.dtype), gy.shape[0], gy.shape[1], gy.data_ptr(), gy.stride(0), y.data_ptr(),
                            y.stride(0), float(alpha), out.data_ptr(), out.stride(0), stream_ptr()), "llp_relu_bwd_2d")


def hits_at_k(pos, neg, Ks):
    """Hits@K for every K in ``Ks`` (device computation, one sync); list of floats."""
    L = lib()
    Ks = [int(k) for k in Ks]
    if any(k <= 0 for k in Ks):
        raise ValueError("K must be positive")
    kd = torch.tensor(Ks, dtype=torch.int32).to(pos.device)
    out = torch.empty(len(Ks), dtype=torch.float64, device=pos.device)
    pos = pos.float().contiguous()
    neg = neg.float().contiguous()
    check(L.llp_hits_at_k(pos.data_ptr(), pos.numel(), neg.data_ptr(), neg.numel(), kd.data_ptr(), len(Ks),
                          out.data_ptr(), stream_ptr()), "llp_hits_at_k")
    return out.tolist()


def auc(pos, neg):
    L = lib()
    pos = pos.float().contiguous()
    neg = neg.float().contiguous()
    ws = torch.empty(L.llp_auc_workspace_bytes(pos.numel(), neg.numel()), dtype=torch.uint8, device=pos.device)
    out = torch.empty(1, dtype=torch.float64, device=pos.device)
    check(L.llp_auc(pos.data_ptr(), pos.numel(), neg.data_ptr(), neg.numel(), out.data_ptr(), ws.data_ptr(),
                    ws.numel(), stream_ptr()), "llp_auc")
    return float(out.item())


def csr_aggregate(n_rows, F, rowptr, col, x, inv_deg, mode, out, accumulate=False):
    L = lib()
    check(L.llp_csr_aggregate(dtype_code(x.dtype), n_rows, F, rowptr.data_ptr(), col.data_ptr(), x.data_ptr(),
                              x.stride(0), ptr(inv_deg), mode, out.data_ptr(), out.stride(0), int(accumulate),
                              stream_ptr()), "llp_csr_aggregate")


def gcn_aggregate(n_rows, F, rowptr, col, x, dinv, out, bias=None, accumulate=False):
    """out[i] = dinv[i] * sum_j dinv[j] x[j] (+ bias) over the CSR rows (llp_gcn_aggregate)."""
    L = lib()
    check(L.llp_gcn_aggregate(dtype_code(x.dtype), n_rows, F, rowptr.data_ptr(), col.data_ptr(), x.data_ptr(),
                              x.stride(0), dinv.data_ptr(), ptr(bias), out.data_ptr(), out.stride(0),
                              int(accumulate), stream_ptr()), "llp_gcn_aggregate")


def grad_sumsq_ws_bytes(n, max_numel):
    return load().llp_grad_sumsq_workspace_bytes(n, max_numel)


TICKET_WORDS = 2080   # LLP_TICKET_WORDS (include/llp_hip.h)


def ticket_block(dev):
    """A ticket block for the one-launch loss / gradient norm: zero, left zero by every call."""
    return torch.zeros(TICKET_WORDS, dtype=torch.int32, device=dev)


def work_items(shapes):
    """(n_work of llp_grad_sumsq_w, n_work of llp_adam_step_w) for a descriptor table whose
    tensors have ``shapes`` = [(numel, rows, cols, has_transposed_shadow), ...]."""
    L = load()
    return (sum(int(L.llp_grad_sumsq_work_items(int(n))) for n, _, _, _ in shapes),
            sum(int(L.llp_adam_work_items(int(n), int(r), int(c), int(bool(t)))) for n, r, c, t in shapes))


def grad_sumsq(descs_dev, n, max_numel, n_groups, sumsq, ws, ticket=None, n_work=0):
    """ticket (a ticket_block): one launch (the finalize in its last workgroup); with n_work
    (work_items) on the compact grid (llp_grad_sumsq_w)."""
    L = lib()
    assert ticket is None or ticket.numel() >= TICKET_WORDS
    if n_work and ticket is not None:
        check(L.llp_grad_sumsq_w(descs_dev.data_ptr(), n, max_numel, int(n_work), n_groups, sumsq.data_ptr(),
                                 ticket.data_ptr(), ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()),
              "llp_grad_sumsq_w")
        return
    check(L.llp_grad_sumsq_t(descs_dev.data_ptr(), n, max_numel, n_groups, sumsq.data_ptr(), ptr(ticket),
                             ws.data_ptr(), ws.numel() * ws.element_size(), stream_ptr()), "llp_grad_sumsq")


def adam_step(descs_dev, n, max_numel, sumsq, max_norm, lr, beta1, beta2, eps, step, fused=False, n_work=0):
    """fused: one launch (both shadows in the Adam pass) that reads *step without advancing it
    (step_end(..., adam_step=step) advances it), on the compact grid with n_work (work_items);
    otherwise Adam + shadow pass, step advanced."""
    L = lib()
    if fused and n_work:
        check(L.llp_adam_step_w(descs_dev.data_ptr(), n, max_numel, int(n_work), ptr(sumsq), max_norm, lr, beta1, beta2, eps,
                                step.data_ptr(), stream_ptr()), "llp_adam_step_w")
        return
    if fused:
        check(L.llp_adam_step_t(descs_dev.data_ptr(), n, max_numel, ptr(sumsq), max_norm, lr, beta1, beta2, eps,
                                step.data_ptr(), stream_ptr()), "llp_adam_step_t")
    else:
        check(L.llp_adam_step(descs_dev.data_ptr(), n, max_numel, ptr(sumsq), max_norm, lr, beta1, beta2, eps,
                              step.data_ptr(), stream_ptr()), "llp_adam_step")


def refresh_shadows(descs_dev, n, max_numel):
    L = lib()
    check(L.llp_refresh_shadows(descs_dev.data_ptr(), n, max_numel, stream_ptr()), "llp_refresh_shadows")


def convert(src, dst):
    L = lib()
    assert src.numel() == dst.numel() and src.is_contiguous() and dst.is_contiguous()
    check(L.llp_convert(dtype_code(src.dtype), dtype_code(dst.dtype), src.numel(), src.data_ptr(), dst.data_ptr(),
                        stream_ptr()), "llp_convert")


def accumulate(src, weight, dst):
    L = lib()
    check(L.llp_accumulate(src.numel(), src.data_ptr(), weight, dst.data_ptr(), stream_ptr()), "llp_accumulate")


def zero_(t):
    L = lib()
    check(L.llp_zero(t.data_ptr(), t.numel() * t.element_size(), stream_ptr()), "llp_zero")


def step_end(loss, weight, loss_sum, ctr, adam_step=None):
    L = lib()
    if adam_step is not None:
        check(L.llp_step_end2(loss.data_ptr(), weight, loss_sum.data_ptr(), ctr.data_ptr(), adam_step.data_ptr(),
                              stream_ptr()), "llp_step_end2")
    else:
        check(L.llp_step_end(loss.data_ptr(), weight, loss_sum.data_ptr(), ctr.data_ptr(), stream_ptr()),
              "llp_step_end")


def increment(ctr):
    L = lib()
    check(L.llp_increment(ctr.data_ptr(), stream_ptr()), "llp_increment")


def descs_to_device(descs, device):
    """Pack a list of TensorDesc into a device byte tensor."""
    arr = (TensorDesc * len(descs))(*descs)
    raw = bytes(C.string_at(C.addressof(arr), C.sizeof(arr)))
    host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    return host.to(device)


def relu_bwd(gy, y, alpha, out):
    L = lib()
    check(L.llp_relu_bwd(dtype_code(gy.dtype), gy.numel(), gy.data_ptr(), ptr(y), alpha, out.data_ptr(),
                         stream_ptr()), "llp_relu_bwd")


def transpose(W):
    L = lib()
    rows, cols = W.shape
    out = torch.empty(cols, rows, dtype=W.dtype, device=W.device)
    check(L.llp_transpose(dtype_code(W.dtype), rows, cols, W.data_ptr(), out.data_ptr(), stream_ptr()),
          "llp_transpose")
    return out


def mul(a, b):
    L = lib()
    a, b = a.contiguous(), b.contiguous()
    out = torch.empty_like(a)
    check(L.llp_mul(dtype_code(a.dtype), a.numel(), a.data_ptr(), b.data_ptr(), out.data_ptr(), stream_ptr()),
          "llp_mul")
    return out


def row_scale(z, s):
    L = lib()
    z = z.contiguous()
    out = torch.empty_like(z)
    check(L.llp_row_scale(dtype_code(z.dtype), z.shape[0], z.shape[1], z.data_ptr(), s.data_ptr(), out.data_ptr(),
                          stream_ptr()), "llp_row_scale")
    return out


def sigmoid_bwd(gprob, prob, out):
    L = lib()
    check(L.llp_sigmoid_bwd(prob.numel(), gprob.data_ptr(), prob.data_ptr(), out.data_ptr(), stream_ptr()),
          "llp_sigmoid_bwd")


# ------------------------------------------------------------------ norm_type (src/models.py:27-37,50-51,90-101,114-115)
def _ld(t):
    assert t.dim() == 2 and t.stride(1) == 1
    return t.stride(0)


def norm_ws_bytes(M, H):
    return int(load().llp_norm_workspace_bytes(int(M), int(H)))


def norm_colsums(y, sums, ws, count=None):
    """sums (f64 [2, H]) = column sums of y and y*y (BatchNorm statistics)."""
    L = lib()
    check(L.llp_norm_colsums(dtype_code(y.dtype), y.shape[0], y.shape[1], y.data_ptr(), _ld(y), ptr(count),
                             sums.data_ptr(), ws.data_ptr(), stream_ptr()), "llp_norm_colsums")


def norm_fwd(kind, y, out, stats, gamma=None, beta=None, eps=1e-5, training=True, sums=None, count=0.0,
             momentum=0.1, running_mean=None, running_var=None, num_batches_tracked=None, relu=True,
             dropout: Dropout | None = None, rows=None):
    """out = dropout(relu(norm(y))); stats f32 [2, M] (layer) / [2, H] (batch)."""
    L = lib()
    check(L.llp_norm_fwd(int(kind), dtype_code(y.dtype), y.shape[0], y.shape[1], y.data_ptr(), _ld(y), ptr(gamma),
                         ptr(beta), float(eps), int(bool(training)), ptr(sums), float(count), float(momentum),
                         ptr(running_mean), ptr(running_var), ptr(num_batches_tracked), stats.data_ptr(), ptr(rows),
                         int(bool(relu)), C.byref(dropout) if dropout is not None else None, out.data_ptr(), _ld(out),
                         stream_ptr()), "llp_norm_fwd")


def norm_bwd_sums(kind, gout, out, alpha, y, stats, sums, ws, dgamma=None, dbeta=None, rows=None):
    """sums (f64 [2, H]) = column sums of g and g*xhat, g = alpha * gout * (out > 0);
    also written to dbeta / dgamma when given."""
    L = lib()
    check(L.llp_norm_bwd_sums(int(kind), dtype_code(y.dtype), y.shape[0], y.shape[1], gout.data_ptr(), _ld(gout),
                              ptr(out), _ld(out) if out is not None else 0, float(alpha), y.data_ptr(), _ld(y),
                              stats.data_ptr(), ptr(rows), sums.data_ptr(), ptr(dgamma), ptr(dbeta), ws.data_ptr(),
                              stream_ptr()), "llp_norm_bwd_sums")


def norm_bwd(kind, gout, out, alpha, y, stats, gy, gamma=None, sums=None, count=0.0, rows=None):
    """gy = d(loss)/dy through dropout(relu(norm(y)))."""
    L = lib()
    check(L.llp_norm_bwd(int(kind), dtype_code(y.dtype), y.shape[0], y.shape[1], gout.data_ptr(), _ld(gout), ptr(out),
                         _ld(out) if out is not None else 0, float(alpha), y.data_ptr(), _ld(y), ptr(gamma),
                         stats.data_ptr(), ptr(sums), float(count), ptr(rows), gy.data_ptr(), _ld(gy), stream_ptr()),
          "llp_norm_bwd")


# ------------------------------------------------------------------ diagnostics
def mfma_probe(data, iters, out):
    """Launch the bare-MFMA ceiling loop (llp_mfma_probe); returns its FLOP count."""
    L = lib()
    fl = c_f64(0.0)
    check(L.llp_mfma_probe(data.data_ptr(), data.numel() * data.element_size() // 16, int(iters), out.data_ptr(),
                           C.byref(fl), stream_ptr()), "llp_mfma_probe")
    return fl.value


def mfma_probe_f32(data, iters, out):
    """The f32-MFMA ceiling loop (llp_mfma_probe_f32) over the f32 tensor ``data``; returns its FLOP count."""
    L = lib()
    fl = c_f64(0.0)
    check(L.llp_mfma_probe_f32(data.data_ptr(), data.numel(), int(iters), out.data_ptr(), C.byref(fl), stream_ptr()),
          "llp_mfma_probe_f32")
    return fl.value


def mfma_probe_out_floats():
    return int(lib().llp_mfma_probe_out_floats())
