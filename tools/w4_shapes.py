"""Per-shape A/B of the NT GEMMs of the collab step: the shipped persistent ping-pong kernel
(llp_gemm_nt -> pp8p) against the one-wave-per-SIMD kernel (llp_gemm_nt_w4_probe), random bf16
operands, event-timed medians, both in one process.  One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import w4_bench as WB  # noqa: E402

K = WB.K
dev = WB.dev
shapes = [(225_280, 1024, 128, "relu"), (225_280, 1024, 1024, "relu"), (225_280, 1024, 1024, "none"),
          (225_280, 1024, 1024, "bwd"), (603_032, 1024, 1024, "relu"), (603_032, 1024, 1024, "none"),
          (603_032, 1024, 1024, "bwd")]
g = torch.Generator(device="cpu").manual_seed(1)
for M, N, Kd, mode in shapes:
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    W = (torch.randn(N, Kd, generator=g) * (1.0 / Kd ** 0.5)).to(torch.bfloat16).to(dev)
    b = (torch.randn(N, generator=g) * 0.1).to(dev)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    mk = torch.zeros(M, N // 8, dtype=torch.uint8, device=dev)
    # a realistic mask (about half the bits set) for the backward mode
    K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=mk)
    if mode == "relu":
        f0 = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=mk)
        f1 = lambda: WB.w4(A, W, M, N, Kd, C, bias=b, act=K.ACT_RELU, mask_out=mk)
    elif mode == "none":
        f0 = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C, K.LLP_BF16, bias=b)
        f1 = lambda: WB.w4(A, W, M, N, Kd, C, bias=b, act=K.ACT_NONE)
    else:
        f0 = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C, K.LLP_BF16, act=K.ACT_RELU_BWD, aux=mk)
        f1 = lambda: WB.w4(A, W, M, N, Kd, C, act=K.ACT_RELU_BWD, mask_in=mk)
    t = {}
    for rnd in range(2):
        for name, f in (("pp8p", f0), ("w4", f1)):
            t.setdefault(name, []).append(WB.timeit(f))
    fl = 2.0 * M * N * Kd
    print(json.dumps({"shape": [M, N, Kd], "mode": mode, "pp8p_ms": min(t["pp8p"]), "w4_ms": min(t["w4"]),
                      "w4_over_pp8p": round(min(t["w4"]) / min(t["pp8p"]), 3),
                      "w4_tflops": round(fl / min(t["w4"]) / 1e9, 1)}), flush=True)
    del A, W, C, mk
    torch.cuda.empty_cache()
