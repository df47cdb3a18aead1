"""Runs a few launches of chosen llp_gemm_nt_w4_probe variants (and the shipped pp8p kernel) at the
dominant shape, for rocprofv3 counter passes (tools/w4_bench.py is the timed A/B)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import w4_bench as WB  # noqa: E402

M = N = Kd = 1024
M = 225_280
g = torch.Generator(device="cpu").manual_seed(3)
A = (torch.randn(M, Kd, generator=g) * 0.5).to(torch.bfloat16).to(WB.dev)
W = (torch.randn(N, Kd, generator=g) * 0.03).to(torch.bfloat16).to(WB.dev)
Cb = torch.empty(M, N, dtype=torch.bfloat16, device=WB.dev)
mk = torch.empty(M, N // 8, dtype=torch.uint8, device=WB.dev)
b = torch.zeros(N, device=WB.dev)
diags = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"])]
for _ in range(3):
    for d in diags:
        if d < 0:
            WB.K.gemm_nt(WB.K.operand(A), WB.K.operand(W), M, N, Kd, Cb, WB.K.LLP_BF16, bias=b, act=WB.K.ACT_RELU,
                         aux=mk)
        else:
            WB.w4(A, W, M, N, Kd, Cb, act=WB.K.ACT_NONE, diag=d)
torch.cuda.synchronize()
print("done", flush=True)
