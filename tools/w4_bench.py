"""The one-wave-per-SIMD NT GEMM (csrc/gemm256_w4.hip, llp_gemm_nt_w4_probe) against the shipped
persistent ping-pong kernel (llp_gemm_nt -> gemm_nt_bf16_pp8p): numerics vs a torch fp32
reference on bf16 operands, ReLU-mask consistency, then event-timed launches at the collab
student's dominant shape (M x 1024 x 1024).  One JSON line per check."""
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import llp_hip as K  # noqa: E402

L = K.lib()
L.llp_gemm_nt_w4_probe.restype = C.c_int
L.llp_gemm_nt_w4_probe.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                   C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_float, C.c_void_p, C.c_void_p,
                                   C.c_int64, C.c_int, C.c_void_p]
dev = torch.device("cuda", 0)


def w4(A, W, M, N, Kd, Cout, bias=None, act=K.ACT_RELU, alpha=1.0, mask_out=None, mask_in=None, diag=0):
    ldm = (mask_out if mask_out is not None else mask_in).stride(0) if (mask_out is not None or mask_in is not None) else 0
    K.check(L.llp_gemm_nt_w4_probe(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), M, N, Kd, Cout.data_ptr(),
                                   Cout.stride(0), K.ptr(bias), act, alpha, K.ptr(mask_out), K.ptr(mask_in), ldm,
                                   diag, K.stream_ptr()), "llp_gemm_nt_w4_probe")


def bits_of(mask, N):
    return ((mask.unsqueeze(-1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1).reshape(mask.shape[0], N)


def check(M, N, Kd, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    W = (torch.randn(N, Kd, generator=g) * (1.0 / Kd ** 0.5)).to(torch.bfloat16).to(dev)
    b = (torch.randn(N, generator=g) * 0.1).to(dev)
    ref = A.float() @ W.float().t() + b
    C1 = torch.full((M, N), 7.0, dtype=torch.bfloat16, device=dev)
    m1 = torch.zeros(M, N // 8, dtype=torch.uint8, device=dev)
    w4(A, W, M, N, Kd, C1, bias=b, act=K.ACT_RELU, mask_out=m1)
    C0 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    m0 = torch.zeros(M, N // 8, dtype=torch.uint8, device=dev)
    K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C0, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=m0)
    torch.cuda.synchronize()
    relu = torch.relu(ref)
    err = (C1.float() - relu).abs().max().item()
    tol = 1e-2 * (1 + relu.abs().max().item())
    diff_pp8 = (C1.float() - C0.float()).abs().max().item()
    mask_ok = bool(torch.equal(bits_of(m1, N).bool(), C1 != 0))
    ulp_frac = (C1 != C0).float().mean().item()
    # plain (no act, no bias) and the ReLU backward through m1 (alpha 2)
    C2 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    w4(A, W, M, N, Kd, C2, act=K.ACT_NONE)
    C3 = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    w4(A, W, M, N, Kd, C3, act=K.ACT_RELU_BWD, alpha=2.0, mask_in=m1)
    torch.cuda.synchronize()
    ref2 = A.float() @ W.float().t()
    err2 = (C2.float() - ref2).abs().max().item()
    ref3 = torch.where(bits_of(m1, N).bool(), 2.0 * C2.float(), torch.zeros_like(ref2))
    err3 = (C3.float() - ref3).abs().max().item()
    ok = err <= tol and err2 <= tol and err3 <= 2 * tol and mask_ok
    print(json.dumps({"check": [M, N, Kd], "relu_err": err, "none_err": err2, "bwd_err_vs_2x_none": err3, "tol": tol,
                      "max_diff_vs_pp8p": diff_pp8, "frac_elems_differing_vs_pp8p": ulp_frac, "mask_ok": mask_ok,
                      "ok": ok}), flush=True)
    return ok


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for s, t in ev:
        s.record()
        fn()
        t.record()
    torch.cuda.synchronize()
    return sorted(s.elapsed_time(t) for s, t in ev)[n // 2]


def main():
    ok = all(check(M, N, Kd, i) for i, (M, N, Kd) in enumerate([(256, 256, 128), (1000, 512, 256), (70_001, 1024, 1024),
                                                                  (5_000, 256, 1024)]))
    if not ok:
        sys.exit(1)
    for M in (225_280,):
        N = Kd = 1024
        g = torch.Generator(device="cpu").manual_seed(3)
        A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
        W = (torch.randn(N, Kd, generator=g) * 0.03).to(torch.bfloat16).to(dev)
        b = torch.zeros(N, device=dev)
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        mk = torch.empty(M, N // 8, dtype=torch.uint8, device=dev)
        fl = 2.0 * M * N * Kd
        res = {"shape": [M, N, Kd], "random_operands": True}
        for name, fn in (("pp8p", lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, Cb, K.LLP_BF16, bias=b,
                                                   act=K.ACT_RELU, aux=mk)),
                         ("w4", lambda: w4(A, W, M, N, Kd, Cb, bias=b, act=K.ACT_RELU, mask_out=mk)),
                         ("w4_none", lambda: w4(A, W, M, N, Kd, Cb, act=K.ACT_NONE)),
                         ("w4_bwd", lambda: w4(A, W, M, N, Kd, Cb, act=K.ACT_RELU_BWD, mask_in=mk)),
                         *[(f"w4_diag{d}", (lambda d=d: w4(A, W, M, N, Kd, Cb, act=K.ACT_NONE, diag=d)))
                           for d in (16, 31)]):
            ms = timeit(fn)
            res[name] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
