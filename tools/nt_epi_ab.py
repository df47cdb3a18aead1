"""Time the NT GEMM epilogue modes at the collab shapes under the current environment
(LLP_GEMM_LEAN_EPI, LLP_GEMM_SKEW, ...) and print per-shape medians plus a checksum of
every output (outputs of two environments must agree bit for bit).

    python tools/nt_epi_ab.py [--iters 10] [--rounds 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_hip as K  # noqa: E402


def checksum(t):
    v = t.contiguous().view(-1)
    v = v.view(torch.int16) if v.element_size() == 2 else v.view(torch.uint8)
    w = (torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521) + 1
    return int((v.to(torch.int64) * w).sum().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    opt = ap.parse_args()
    K.lib()
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    U, R2 = 225_334, 603_032
    h = torch.relu(torch.randn(R2, 1024, device=dev, dtype=bf, generator=g))
    xg = torch.randn(U, 128, device=dev, dtype=bf, generator=g)
    W = (torch.randn(1024, 1024, device=dev, generator=g) * 0.03).to(bf)
    W1 = (torch.randn(1024, 128, device=dev, generator=g) * 0.1).to(bf)
    bias = torch.randn(1024, device=dev, generator=g)
    out = torch.empty(R2, 1024, device=dev, dtype=bf)
    mask = torch.zeros(R2, 128, dtype=torch.uint8, device=dev)
    mask_in = torch.randint(0, 256, (R2, 128), dtype=torch.uint8, device=dev, generator=g)
    hw = torch.randn(1024, device=dev, generator=g)
    hpart = torch.zeros(K.head_parts(1024), R2, device=dev)
    cases = {
        "U L0 fwd relu+mask 225334x1024x128": (lambda: K.gemm_nt(K.operand(xg), K.operand(W1), U, 1024, 128, out[:U], 1,
                                                                  bias=bias, act=K.ACT_RELU, aux=mask[:U]),
                                                (out[:U], mask[:U]), 2 * U * 1024 * 128),
        "U fwd relu+mask 225334x1024x1024": (lambda: K.gemm_nt(K.operand(h[:U]), K.operand(W), U, 1024, 1024, out[:U],
                                                                1, bias=bias, act=K.ACT_RELU, aux=mask[:U]),
                                              (out[:U], mask[:U]), 2 * U * 1024 * 1024),
        "P fwd relu 603032x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R2, 1024, 1024, out, 1,
                                                          bias=bias, act=K.ACT_RELU), (out,), 2 * R2 * 1024 * 1024),
        "P fwd none 603032x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R2, 1024, 1024, out, 1,
                                                          bias=bias), (out,), 2 * R2 * 1024 * 1024),
        "P dgrad mask-bwd 603032x1024x1024": (lambda: K.gemm_nt(K.operand(h), K.operand(W), R2, 1024, 1024, out, 1,
                                                                act=K.ACT_RELU_BWD, aux=mask_in, alpha=1.0),
                                              (out,), 2 * R2 * 1024 * 1024),
        "U dgrad mask-bwd 225334x1024x1024": (lambda: K.gemm_nt(K.operand(h[:U]), K.operand(W), U, 1024, 1024, out[:U],
                                                                1, act=K.ACT_RELU_BWD, aux=mask_in[:U], alpha=2.0),
                                              (out[:U],), 2 * U * 1024 * 1024),
        "P fwd+head 603032x1024x1024": (lambda: K.gemm_nt_head(K.operand(h), K.operand(W), R2, 1024, 1024, out, hw,
                                                               hpart, bias=bias, act=K.ACT_RELU),
                                        (out, hpart), 2 * R2 * 1024 * 1024),
        "ragged relu+mask 1000x288x1024": (lambda: K.gemm_nt(K.operand(h[:1000]), K.operand(W[:288]), 1000, 288, 1024,
                                                             out[:1000, :288], 1, bias=bias, act=K.ACT_RELU,
                                                             aux=mask[:1000]), (out[:1000], mask[:1000]),
                                           2 * 1000 * 288 * 1024),
    }
    sums = {}
    for name, (fn, outs, _) in cases.items():
        for o in outs:
            o.zero_()
        fn()
        torch.cuda.synchronize()
        sums[name] = [checksum(o) for o in outs]
    times = {n: [] for n in cases}
    for _ in range(opt.rounds):
        for name, (fn, _, _) in cases.items():
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(opt.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / opt.iters)
    res = {}
    for name, (_, _, flop) in cases.items():
        t = sorted(times[name])[len(times[name]) // 2]
        res[name] = {"ms": t, "tflops": flop / t / 1e9, "sum": sums[name]}
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("LLP_")}, "res": res}))


if __name__ == "__main__":
    main()
