"""A/B of the large-tile bf16 NT main-loop variants (llp_set_gemm_variant) in
one process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), on
random data at the collab step shapes.  Also checks that every variant gives
bit-identical outputs (same per-accumulator k order) and matches torch.

    python tools/gemm_variants.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_hip as K  # noqa: E402

VARIANTS = tuple(int(v) for v in os.environ.get("LLP_AB_VARIANTS", "4,6").split(","))
NAMES = {0: "pipe4", 1: "pp42", 2: "pp53", 3: "q64", 4: "q64-lean", 5: "h128", 6: "q64-stag", 7: "q64-stag-late-dma",
         8: "pp8", 9: "pp8-direct", 10: "pp8-lines", 11: "pp8-mode"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    opt = ap.parse_args()
    L = K.lib()
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    R1, R2, N0 = 747_214, 603_032, 235_868
    x = torch.randn(N0, 128, device=dev, dtype=bf, generator=g)
    xg = x[:225334].contiguous()
    idx = torch.randint(0, N0, (R1,), device=dev, dtype=torch.int32, generator=g)
    h = torch.randn(R1, 1024, device=dev, dtype=bf, generator=g)
    W = (torch.randn(1024, 1024, device=dev, generator=g) * 0.03).to(bf)
    W1 = (torch.randn(1024, 128, device=dev, generator=g) * 0.1).to(bf)
    Wt = (torch.randn(256, 512, device=dev, generator=g) * 0.05).to(bf)
    xa = torch.randn(N0, 512, device=dev, dtype=bf, generator=g)
    bias = torch.randn(1024, device=dev, generator=g)
    aux = torch.randn(R1, 1024, device=dev, dtype=bf, generator=g)
    out = torch.empty(R1, 1024, device=dev, dtype=bf)
    hr = torch.relu(h[:225334])     # activation-like operand (half zeros), as in the step
    outs = torch.empty(N0, 256, device=dev, dtype=bf)
    step_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    drop = K.Dropout(0.5, 1234, step_ctr.data_ptr(), 3)
    mask = torch.zeros(R1, 1024 // 8, dtype=torch.uint8, device=dev)
    mask_in = torch.randint(0, 256, (R1, 1024 // 8), dtype=torch.uint8, device=dev, generator=g)
    hw = torch.randn(1024, device=dev, generator=g)
    hpart = torch.zeros(K.head_parts(1024), R2, device=dev)
    # epilogue features (checked for bit-identity; not in the timing table)
    extra = {
        "L2 fwd relu + mask_out": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1, bias=bias,
                                                     act=K.ACT_RELU, aux=mask), (out, mask)),
        "L2 dgrad relu-bwd mask_in": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1,
                                                        act=K.ACT_RELU_BWD, aux=mask_in, alpha=2.0), (out,)),
        "P fwd dropout": (lambda: K.gemm_nt(K.operand(h[:R2]), K.operand(W), R2, 1024, 1024, out[:R2], 1, bias=bias,
                                            act=K.ACT_RELU, dropout=drop), (out,)),
        "P fwd head": (lambda: K.gemm_nt_head(K.operand(h[:R2]), K.operand(W), R2, 1024, 1024, out[:R2], hw, hpart,
                                              bias=bias, act=K.ACT_RELU, dropout=drop), (out, hpart)),
        "P fwd head, no C": (lambda: K.gemm_nt_head(K.operand(h[:R2]), K.operand(W), R2, 1024, 1024, None, hw, hpart,
                                                    bias=bias, act=K.ACT_RELU), (hpart,)),
        "ragged 1000x264x1024": (lambda: K.gemm_nt(K.operand(h[:1000]), K.operand(W[:264]), 1000, 264, 1024,
                                                   out[:1000, :264], 1, bias=bias, act=K.ACT_RELU), (out,)),
    }
    for name, (fn, outs_) in extra.items():
        res = []
        for v in VARIANTS:
            L.llp_set_gemm_variant(v)
            for o in outs_:
                o.zero_()
            fn()
            torch.cuda.synchronize()
            res.append([o.clone() for o in outs_])
        same = all(all(torch.equal(a, b) for a, b in zip(res[0], r)) for r in res[1:])
        print(f"{name}: variants bit-identical: {same}", flush=True)
    cases = {
        "L1 fwd gather 747214x1024x128": (lambda: K.gemm_nt(K.operand(x, idx), K.operand(W1), R1, 1024, 128, out, 1,
                                                            bias=bias, act=K.ACT_RELU), 2 * R1 * 1024 * 128, out),
        "U L0 fwd 225334x1024x128": (lambda: K.gemm_nt(K.operand(xg), K.operand(W1), 225334, 1024, 128, out[:225334],
                                                       1, bias=bias, act=K.ACT_RELU, aux=mask[:225334]),
                                     2 * 225334 * 1024 * 128, out),
        "L2 fwd 747214x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1, bias=bias,
                                                      act=K.ACT_RELU), 2 * R1 * 1024 * 1024, out),
        "L2 dgrad relu-bwd 747214x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1,
                                                                 act=K.ACT_RELU_BWD, aux=aux), 2 * R1 * 1024 * 1024,
                                               out),
        "L2 dgrad mask-bwd 747214x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R1, 1024, 1024, out, 1,
                                                                 act=K.ACT_RELU_BWD, aux=mask_in),
                                               2 * R1 * 1024 * 1024, out),
        "P fwd+head 603032x1024x1024": (lambda: K.gemm_nt_head(K.operand(h[:R2]), K.operand(W), R2, 1024, 1024,
                                                               out[:R2], hw, hpart, bias=bias, act=K.ACT_RELU),
                                        2 * R2 * 1024 * 1024, out),
        "P fwd 603032x1024x1024": (lambda: K.gemm_nt(K.operand(h[:R2]), K.operand(W), R2, 1024, 1024, out[:R2], 1,
                                                     bias=bias, act=K.ACT_RELU), 2 * R2 * 1024 * 1024, out),
        "U fwd 225334x1024x1024": (lambda: K.gemm_nt(K.operand(h[:225334]), K.operand(W), 225334, 1024, 1024,
                                                     out[:225334], 1, bias=bias, act=K.ACT_RELU),
                                   2 * 225334 * 1024 * 1024, out),
        "U fwd relu-data 225334x1024x1024": (lambda: K.gemm_nt(K.operand(hr), K.operand(W), 225334, 1024, 1024,
                                                               out[:225334], 1, bias=bias, act=K.ACT_RELU),
                                             2 * 225334 * 1024 * 1024, out),
        "SAGE L0 235868x256x256": (lambda: K.gemm_nt(K.operand(xa[:, :256]), K.operand(Wt[:, :256]), N0, 256, 256,
                                                     outs, 1, bias=bias[:256], act=K.ACT_RELU),
                                   2 * N0 * 256 * 256, outs),
        "SAGE 235868x256x512": (lambda: K.gemm_nt(K.operand(xa), K.operand(Wt), N0, 256, 512, outs, 1, bias=bias[:256],
                                                  act=K.ACT_RELU), 2 * N0 * 256 * 512, outs),
    }
    # bit-identity across variants + a torch spot check
    for name, (fn, flop, o) in cases.items():
        res = []
        for v in VARIANTS:
            L.llp_set_gemm_variant(v)
            o.zero_()
            fn()
            torch.cuda.synchronize()
            res.append(o.clone())
        same = all(torch.equal(res[0], r) for r in res[1:])
        print(f"{name}: variants bit-identical: {same}", flush=True)
    if True:   # torch check of the L2 fwd on 4096 rows
        L.llp_set_gemm_variant(VARIANTS[-1])
        cases["L2 fwd 747214x1024x1024"][0]()
        torch.cuda.synchronize()
        ref = torch.relu(h[:4096].float() @ W.float().t() + bias)
        err = (out[:4096].float() - ref).abs().max().item()
        print(f"L2 fwd vs torch fp32 (4096 rows): max abs err {err:.4f} (ref max {ref.abs().max().item():.2f})")
    times = {(n, v): [] for n in cases for v in VARIANTS}
    for r in range(opt.rounds):
        for name, (fn, flop, o) in cases.items():
            for v in VARIANTS:
                L.llp_set_gemm_variant(v)
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(opt.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[(name, v)].append(s.elapsed_time(e) / opt.iters)
    for name, (fn, flop, o) in cases.items():
        row = []
        for v in VARIANTS:
            t = sorted(times[(name, v)])
            med = t[len(t) // 2]
            row.append(f"{NAMES[v]} {med:.3f} ms {flop / med / 1e9:.0f} TF")
        print(f"{name:38s} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
