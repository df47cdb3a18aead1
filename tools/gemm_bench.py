"""Micro-benchmark of the LLP GEMM kernels at the ogbl-collab step shapes.
Prints one line per shape: milliseconds per launch and TFLOP/s.
  python tools/gemm_bench.py [--iters 10]
(LLP_GEMM_V1=1 forces the general 128x128 kernel for an A/B.)"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_hip as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    opt = ap.parse_args()
    dev = "cuda"
    bf = torch.bfloat16
    R1, R2, RT, N0 = 747_214, 603_032, 471_960, 235_868
    x = torch.randn(N0, 128, device=dev, dtype=bf)
    idx = torch.randint(0, N0, (R1,), device=dev, dtype=torch.int32)
    h = torch.randn(R1, 1024, device=dev, dtype=bf)
    ia = torch.randint(0, R1, (R2,), device=dev, dtype=torch.int32)
    ib = torch.randint(0, R1, (R2,), device=dev, dtype=torch.int32)
    W = torch.randn(1024, 1024, device=dev, dtype=bf) * 0.03
    W1 = torch.randn(1024, 128, device=dev, dtype=bf) * 0.1
    th = torch.randn(N0, 256, device=dev, dtype=bf)
    tia = torch.randint(0, N0, (RT,), device=dev, dtype=torch.int32)
    Wt = torch.randn(256, 256, device=dev, dtype=bf) * 0.05
    bias = torch.zeros(1024, device=dev)
    out = torch.empty(R1, 1024, device=dev, dtype=bf)
    aux = torch.randn(R1, 1024, device=dev, dtype=bf)
    cases = [
        ("L1 fwd gather   747214x1024x128", lambda: K.gemm_nt(K.operand(x, idx), K.operand(W1), R1, 1024, 128, out, 1,
                                                            bias=bias, act=K.ACT_RELU), 2 * R1 * 1024 * 128),
        ("L2 fwd          747214x1024x1024", lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1,
                                                             bias=bias, act=K.ACT_RELU), 2 * R1 * 1024 * 1024),
        ("L2 dgrad relu   747214x1024x1024", lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1,
                                                             act=K.ACT_RELU_BWD, aux=aux), 2 * R1 * 1024 * 1024),
        ("P1 fwd hadamard 603032x1024x1024", lambda: K.gemm_nt(K.operand(h, ia, h, ib), K.operand(W), R2, 1024, 1024,
                                                             out, 1, bias=bias, act=K.ACT_RELU),
         2 * R2 * 1024 * 1024),
        ("T1 fwd hadamard 471960x256x256", lambda: K.gemm_nt(K.operand(th, tia, th, tia), K.operand(Wt), RT, 256, 256,
                                                           out, 1, act=K.ACT_RELU), 2 * RT * 256 * 256),
    ]
    gW = torch.empty(1024, 1024, device=dev)
    ws = torch.empty(K.gemm_tn_ws_bytes(1, R1, 1024, 1024) // 4 + 16, device=dev)
    gW1 = torch.empty(1024, 128, device=dev)
    ws1 = torch.empty(K.gemm_tn_ws_bytes(1, R1, 1024, 128) // 4 + 16, device=dev)
    cases += [
        ("L2 wgrad        1024x1024 over 747214", lambda: K.gemm_tn(K.operand(aux), K.operand(h), R1, 1024, 1024, gW,
                                                                   1, ws), 2 * R1 * 1024 * 1024),
        ("L1 wgrad gather 1024x128 over 747214", lambda: K.gemm_tn(K.operand(aux), K.operand(x, idx), R1, 1024, 128,
                                                                  gW1, 1, ws1), 2 * R1 * 1024 * 128),
        ("P1 wgrad hadam. 1024x1024 over 603032", lambda: K.gemm_tn(K.operand(aux), K.operand(h, ia, h, ib), R2, 1024,
                                                                   1024, gW, 1, ws), 2 * R2 * 1024 * 1024),
    ]
    for name, fn, flop in cases:
        ms = timeit(fn, opt.iters)
        print(f"{name:42s} {ms:8.3f} ms  {flop / ms / 1e9:8.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
