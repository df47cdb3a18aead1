"""Writes the weight-gradient GEMM's outputs at three step shapes (seeded inputs)
to gpurun_out/tn_<LLP_TN_STAG>.pt, so two main-loop variants can be compared
bit for bit across processes:  python tools/tn_dump.py; python tools/tn_dump.py --compare 0 2"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402


def main():
    out_dir = os.path.join(REPO, "gpurun_out")
    if len(sys.argv) > 1 and sys.argv[1] == "--compare":
        a = torch.load(os.path.join(out_dir, f"tn_{sys.argv[2]}.pt"), weights_only=True)
        b = torch.load(os.path.join(out_dir, f"tn_{sys.argv[3]}.pt"), weights_only=True)
        same = all(torch.equal(a[k], b[k]) for k in a)
        print(f"TN variants {sys.argv[2]} vs {sys.argv[3]} bit-identical: {same}")
        sys.exit(0 if same else 1)
    import llp_hip as K
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    res = {}
    for name, M, P, Q, gather in (("p", 603_032, 1024, 1024, False), ("u", 225_334, 1024, 1024, False),
                                  ("x", 225_334, 1024, 128, True)):
        dz = torch.randn(M, P, device=dev, dtype=bf, generator=g)
        if gather:
            x = torch.randn(235_868, Q, device=dev, dtype=bf, generator=g)
            idx = torch.randint(0, 235_868, (M,), device=dev, dtype=torch.int32, generator=g)
            B = K.operand(x, idx)
        else:
            B = K.operand(torch.relu(torch.randn(M, Q, device=dev, dtype=bf, generator=g)))
        gw = torch.empty(P, Q, device=dev)
        gb = torch.empty(P, device=dev)
        ws = torch.empty(K.gemm_tn_ws_bytes(1, M, P, Q) // 4 + 16, device=dev)
        K.gemm_tn(K.operand(dz), B, M, P, Q, gw, 1, ws, colsum_a=gb)
        torch.cuda.synchronize()
        res[name + "_w"], res[name + "_b"] = gw.cpu(), gb.cpu()
    os.makedirs(out_dir, exist_ok=True)
    torch.save(res, os.path.join(out_dir, f"tn_{os.environ.get('LLP_TN_STAG', '0')}.pt"))


if __name__ == "__main__":
    main()
