"""Reference point: torch.mm (hipBLASLt) vs the hand-written NT/TN kernels at
the step's GEMM shapes, same random data, interleaved rounds.

    python tools/gemm_vs_blaslt.py [--dtype bf16|fp32] [--M 603032,225384]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402


def t(fn, it=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--M", default="603032,225384")
    opt = ap.parse_args()
    dev = "cuda"
    bf = torch.bfloat16 if opt.dtype == "bf16" else torch.float32
    torch.backends.cuda.matmul.allow_tf32 = False      # fp32 means fp32 (no reduced-precision MFMA)
    dc = K.dtype_code(bf)
    g = torch.Generator(device=dev).manual_seed(0)
    for M in (int(m) for m in opt.M.split(",")):
        A = torch.randn(M, 1024, device=dev, dtype=bf, generator=g)
        W = (torch.randn(1024, 1024, device=dev, generator=g) * 0.03).to(bf)
        out = torch.empty(M, 1024, device=dev, dtype=bf)
        Wt = W.t().contiguous()
        ws = torch.empty(K.gemm_tn_ws_bytes(dc, M, 1024, 1024) // 4 + 16, device=dev)
        gW = torch.empty(1024, 1024, device=dev)
        f = 2 * M * 1024 * 1024
        res = {}
        for r in range(3):
            for name, fn in (("ours NT", lambda: K.gemm_nt(K.operand(A), K.operand(W), M, 1024, 1024, out, dc)),
                             ("torch mm NT", lambda: torch.mm(A, Wt, out=out)),
                             ("ours TN", lambda: K.gemm_tn(K.operand(A), K.operand(A), M, 1024, 1024, gW, dc, ws)),
                             ("torch mm TN", lambda: torch.mm(A.t(), A))):
                res.setdefault(name, []).append(t(fn))
        for name, v in res.items():
            ms = sorted(v)[1]
            print(f"{opt.dtype} M={M:7d} {name:12s} {ms:.3f} ms {f / ms / 1e9:.0f} TF", flush=True)
        K.gemm_nt(K.operand(A), K.operand(W), M, 1024, 1024, out, dc)
        ref = torch.mm(A.float(), W.float().t())
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"{opt.dtype} M={M:7d} NT max rel error vs an f32 torch.mm: {err:.2e} ({K.last_gemm_kernel()})", flush=True)


if __name__ == "__main__":
    main()
