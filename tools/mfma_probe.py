"""Practical bf16 MFMA peak of this MI355X (llp_mfma_probe, bench.py practical_peak), three
repeats; with --gemm also the persistent NT GEMM on random bf16 operands at the dominant
shape, event-timed, for the fraction of that peak."""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import bench  # noqa: E402
import llp_hip as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gemm", type=int, default=225280, help="M of the M x 1024 x 1024 NT GEMM (0: skip)")
ap.add_argument("--a-one-row", action="store_true",
                help="diagnostic: every A row aliases row 0 (stride 0), so A is always an L2 hit")
opt = ap.parse_args()
dev = torch.device("cuda", 0)
res = {"practical_peak_tflops": [bench.practical_peak(dev) for _ in range(3)]}
if opt.gemm:
    M, N, Kd = opt.gemm, 1024, 1024
    g = torch.Generator(device="cpu").manual_seed(3)
    A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    if opt.a_one_row:
        A = A[:1].expand(M, Kd)
    W = (torch.randn(N, Kd, generator=g) * 0.03).to(torch.bfloat16).to(dev)
    b = torch.zeros(N, device=dev)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    mask = torch.empty(M, N // 8, dtype=torch.uint8, device=dev)
    run = lambda: K.gemm_nt(K.operand(A), K.operand(W), M, N, Kd, C, K.LLP_BF16, bias=b, act=K.ACT_RELU, aux=mask)
    for _ in range(5):
        run()
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for s, t in e:
        s.record()
        run()
        t.record()
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(t) for s, t in e)[len(e) // 2]
    res["gemm_random"] = {"shape": [M, N, Kd], "median_ms": ms, "tflops": 2.0 * M * N * Kd / ms / 1e9,
                          "a_one_row": bool(opt.a_one_row)}
print(json.dumps(res), flush=True)
