"""A/B of the bf16 weight-gradient (TN) main-loop variants (llp_set_gemm_tn_variant)
in one process, interleaved rounds, at the collab step shapes; checks first that
the variants give bit-identical weight and bias gradients.

    LLP_TN_VARIANTS=2,3 python tools/tn_variants.py [--rounds 5]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_hip as K  # noqa: E402

VARIANTS = tuple(int(v) for v in os.environ.get("LLP_TN_VARIANTS", "2,3").split(","))
NAMES = {0: "lockstep", 1: "stag", 2: "stag-late", 3: "pingpong", 4: "pingpong-split", 5: "lean-stag-late", 6: "lean-stag", 10: "stag-late-tilemajor"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    opt = ap.parse_args()
    L = K.lib()
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn(235_868, 128, device=dev, dtype=bf, generator=g)
    cases = {}
    for name, M, P, Q, gather, cnt in (("P wgrad 603032x1024x1024", 603_032, 1024, 1024, False, None),
                                       ("U wgrad 225334x1024x1024", 225_334, 1024, 1024, False, None),
                                       ("U wgrad dev-count 225334 (of 400000)", 400_000, 1024, 1024, False, 225_334),
                                       ("L0 wgrad gather 225334x1024x128", 225_334, 1024, 128, True, None),
                                       ("ragged 1000x264x200", 1000, 264, 200, False, None),
                                       ("SAGE wgrad 235868x256x512", 235_868, 256, 512, False, None)):
        dz = torch.randn(M, P, device=dev, dtype=bf, generator=g)
        rows = None
        if cnt is not None:
            rows = torch.tensor([cnt], dtype=torch.int32, device=dev)
        if gather:
            idx = torch.randint(0, 235_868, (M,), device=dev, dtype=torch.int32, generator=g)
            B = K.operand(x, idx, count=rows)
        else:
            B = K.operand(torch.relu(torch.randn(M, Q, device=dev, dtype=bf, generator=g)), count=rows)
        A = K.operand(dz, count=rows)
        gw = torch.empty(P, Q, device=dev)
        gb = torch.empty(P, device=dev)
        ws = torch.empty(K.gemm_tn_ws_bytes(1, M, P, Q) // 4 + 16, device=dev)
        fn = (lambda A=A, B=B, M=M, P=P, Q=Q, gw=gw, ws=ws, gb=gb: K.gemm_tn(A, B, M, P, Q, gw, 1, ws, colsum_a=gb))
        cases[name] = (fn, 2 * (cnt or M) * P * Q, (gw, gb))
    for name, (fn, flop, outs) in cases.items():
        res = []
        for v in VARIANTS:
            L.llp_set_gemm_tn_variant(v)
            for o in outs:
                o.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            res.append([o.clone() for o in outs])
        same = all(all(torch.equal(a, b) for a, b in zip(res[0], r)) for r in res[1:])
        print(f"{name}: variants bit-identical: {same}", flush=True)
    times = {(n, v): [] for n in cases for v in VARIANTS}
    for _ in range(opt.rounds):
        for name, (fn, flop, outs) in cases.items():
            for v in VARIANTS:
                L.llp_set_gemm_tn_variant(v)
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(opt.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[(name, v)].append(s.elapsed_time(e) / opt.iters)
    for name, (fn, flop, outs) in cases.items():
        row = []
        for v in VARIANTS:
            t = sorted(times[(name, v)])
            med = t[len(t) // 2]
            row.append(f"{NAMES[v]} {med:.3f} ms {flop / med / 1e9:.0f} TF")
        print(f"{name:38s} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
