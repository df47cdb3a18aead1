"""Cost of each NT GEMM epilogue feature at the collab step shapes: the same
main loop with (a) bias only, (b) bias + ReLU, (c) bias + ReLU + bit-mask out,
(d) ReLU backward through a bit mask, (e) ReLU + fused Linear(N,1) head.
Interleaved rounds, median of rounds.

    python tools/epi_cost.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_hip as K  # noqa: E402


def timed(fn, it):
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    opt = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    H = 1024
    W = (torch.randn(H, H, device=dev, generator=g) * 0.03).to(bf)
    bias = torch.randn(H, device=dev, generator=g)
    hw = torch.randn(H, device=dev, generator=g)
    cases = {}
    for M in (225_334, 603_032):
        A = torch.randn(M, H, device=dev, dtype=bf, generator=g)
        out = torch.empty(M, H, device=dev, dtype=bf)
        mask = torch.zeros(M, H // 8, dtype=torch.uint8, device=dev)
        mask_in = torch.randint(0, 256, (M, H // 8), dtype=torch.uint8, device=dev, generator=g)
        hpart = torch.zeros(K.head_parts(H), M, device=dev)
        op, opw = K.operand(A), K.operand(W)
        cases[(M, "bias")] = lambda op=op, out=out, M=M: K.gemm_nt(op, opw, M, H, H, out, 1, bias=bias)
        cases[(M, "bias+relu")] = lambda op=op, out=out, M=M: K.gemm_nt(op, opw, M, H, H, out, 1, bias=bias,
                                                                        act=K.ACT_RELU)
        cases[(M, "bias+relu+mask")] = lambda op=op, out=out, M=M, mask=mask: K.gemm_nt(
            op, opw, M, H, H, out, 1, bias=bias, act=K.ACT_RELU, aux=mask)
        cases[(M, "relu-bwd mask_in")] = lambda op=op, out=out, M=M, mi=mask_in: K.gemm_nt(
            op, opw, M, H, H, out, 1, act=K.ACT_RELU_BWD, aux=mi)
        cases[(M, "head relu")] = lambda op=op, out=out, M=M, hp=hpart: K.gemm_nt_head(
            op, opw, M, H, H, out, hw, hp, bias=bias)
    res = {k: [] for k in cases}
    for _ in range(opt.rounds):
        for k, fn in cases.items():
            res[k].append(timed(fn, opt.iters))
    for (M, name), v in res.items():
        ms = sorted(v)[len(v) // 2]
        print(f"M={M:7d} {name:18s} {ms:.4f} ms  {2 * M * H * H / ms / 1e9:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
