"""One bf16 weight-gradient GEMM shape, repeated (for rocprofv3 --pmc passes):
    python tools/tn_one.py VARIANT M P Q [iters]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402

import llp_hip as K  # noqa: E402

v, M, P, Q = (int(a) for a in sys.argv[1:5])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 5
K.lib().llp_set_gemm_tn_variant(v)
g = torch.Generator(device="cuda").manual_seed(0)
dz = torch.randn(M, P, device="cuda", dtype=torch.bfloat16, generator=g)
x = torch.relu(torch.randn(M, Q, device="cuda", dtype=torch.bfloat16, generator=g))
gw = torch.empty(P, Q, device="cuda")
gb = torch.empty(P, device="cuda")
ws = torch.empty(K.gemm_tn_ws_bytes(1, M, P, Q) // 4 + 16, device="cuda")
for _ in range(it):
    K.gemm_tn(K.operand(dz), K.operand(x), M, P, Q, gw, 1, ws, colsum_a=gb)
torch.cuda.synchronize()
print("ok")
