"""Split an NT GEMM's time into the K-proportional main loop and the per-tile
constant (prologue + epilogue): time(K) = a + b*K at fixed M, N, for each
main-loop variant in LLP_AB_VARIANTS (interleaved in one process)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402

VARIANTS = tuple(int(v) for v in os.environ.get("LLP_AB_VARIANTS", "6").split(","))
KS = tuple(int(v) for v in os.environ.get("LLP_KS", "1024,2048,4096").split(","))


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
    L = K.lib()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = int(os.environ.get("LLP_M", 225_334)), 1024
    out = torch.empty(M, N, device=dev, dtype=bf)
    bias = torch.randn(N, device=dev, generator=g)
    ops = {}
    for Kd in KS:
        A = torch.randn(M, Kd, device=dev, dtype=bf, generator=g)
        W = (torch.randn(N, Kd, device=dev, generator=g) * 0.03).to(bf)
        ops[Kd] = (A, W)
    res = {(v, Kd): [] for v in VARIANTS for Kd in KS}
    for rnd in range(5):
        for Kd in KS:
            A, W = ops[Kd]
            for v in VARIANTS:
                L.llp_set_gemm_variant(v)
                fn = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, out, 1, bias=bias, act=K.ACT_RELU)
                res[(v, Kd)].append(t(fn))
    for v in VARIANTS:
        pts = []
        for Kd in KS:
            ms = sorted(res[(v, Kd)])[2]
            pts.append((Kd, ms))
            print(f"variant {v} K={Kd:5d} {ms:.3f} ms {2 * M * N * Kd / ms / 1e9:.0f} TF", flush=True)
        (k1, t1), (k2, t2) = pts[0], pts[-1]
        b = (t2 - t1) / (k2 - k1)
        a = t1 - b * k1
        print(f"variant {v}: per-call constant {a:.3f} ms; main loop {2 * M * N / b / 1e9:.0f} TF marginal "
              f"(constant = {100 * a / (a + b * 1024):.0f} % at K=1024)", flush=True)


if __name__ == "__main__":
    main()
