"""Split an NT GEMM's time into the K-proportional main loop and the per-tile
constant (prologue + epilogue): time(K) = a + b*K at fixed M, N."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402


def t(fn, it=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = 225_334, 1024
    out = torch.empty(M, N, device=dev, dtype=bf)
    aux = torch.randn(M, N, device=dev, dtype=bf, generator=g)
    bias = torch.randn(N, device=dev, generator=g)
    for mode in ("plain", "bias+relu", "relu-bwd"):
        res = []
        for Kd in (256, 512, 1024, 2048):
            A = torch.randn(M, Kd, device=dev, dtype=bf, generator=g)
            W = (torch.randn(N, Kd, device=dev, generator=g) * 0.03).to(bf)
            if mode == "plain":
                fn = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, out, 1)
            elif mode == "bias+relu":
                fn = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, out, 1, bias=bias, act=K.ACT_RELU)
            else:
                fn = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, out, 1, act=K.ACT_RELU_BWD, aux=aux)
            ms = min(t(fn) for _ in range(3))
            res.append((Kd, ms))
            print(f"{mode:10s} K={Kd:5d} {ms:.3f} ms {2 * M * N * Kd / ms / 1e9:.0f} TF", flush=True)
        (k1, t1), (k2, t2) = res[1], res[3]
        b = (t2 - t1) / (k2 - k1)
        a = t1 - b * k1
        print(f"{mode:10s} per-call constant {a:.3f} ms; K=1024 main loop {b * 1024:.3f} ms "
              f"(constant = {100 * a / (a + b * 1024):.0f} % at K=1024)", flush=True)


if __name__ == "__main__":
    main()
