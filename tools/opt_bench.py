"""Optimizer-launch microbenchmark at the physics student's parameter shapes.

Times, with HIP events over many back-to-back calls on the current stream:
  * llp_grad_sumsq_t (one launch, ticket) and llp_grad_sumsq (two launches),
  * llp_adam_step_t (one launch) and llp_adam_step (Adam + transposed-shadow pass),
  * a torch device copy moving the same bytes as Adam's compulsory traffic (the HBM yardstick).
Prints one JSON line per measurement.  Shapes: the physics MLP student (8,415 -> 256 -> 256) and
its MLP predictor (256 -> 256 -> 1), weights with a bf16 shadow and a transposed bf16 shadow as
the engine keeps them (llp_engine._set_shadow).

  python tools/opt_bench.py [--reps 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "linkless-link-prediction_amd"))
import llp_hip as K  # noqa: E402

SHAPES = [((256, 8415), True), ((256,), False), ((256, 256), True), ((256,), False),
          ((256, 256), True), ((256,), False), ((1, 256), True), ((1,), False)]


def build(dev):
    keep, descs = [], []
    for shape, shadowed in SHAPES:
        p = torch.randn(*shape, device=dev)
        g = torch.randn(*shape, device=dev) * 1e-3
        m = torch.zeros_like(p)
        v = torch.zeros_like(p)
        rows, cols = (shape[0], shape[1]) if len(shape) == 2 else (1, shape[0])
        sh = st = None
        if shadowed:
            sh = torch.zeros(rows, cols, dtype=torch.bfloat16, device=dev)
            st = torch.zeros(cols, rows, dtype=torch.bfloat16, device=dev)
        keep += [p, g, m, v, sh, st]
        descs.append(K.TensorDesc(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), K.ptr(sh), K.ptr(st),
                                  p.numel(), rows, cols, 0, K.LLP_BF16 if shadowed else 0, 0, 0))
    return keep, descs


def timed(fn, reps):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    keep, descs = build(dev)
    n = len(descs)
    numel = sum(d.numel for d in descs)
    max_numel = max(d.numel for d in descs)
    shadowed = sum(d.numel for d, (_, s) in zip(descs, SHAPES) if s)
    dd = K.descs_to_device(descs, dev)
    sumsq = torch.zeros(1, device=dev)
    ws = torch.empty(K.grad_sumsq_ws_bytes(n, max_numel) // 4 + 16, device=dev)
    ticket = K.ticket_block(dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    adam_bytes = 28 * numel + 4 * shadowed          # g m v p read, m v p written, two bf16 shadows
    norm_bytes = 4 * numel
    out = []
    us = timed(lambda: K.grad_sumsq(dd, n, max_numel, 1, sumsq, ws, ticket=ticket), args.reps)
    out.append(("grad_sumsq one launch", us, norm_bytes))
    us = timed(lambda: K.grad_sumsq(dd, n, max_numel, 1, sumsq, ws), args.reps)
    out.append(("grad_sumsq two launches", us, norm_bytes))
    us = timed(lambda: K.adam_step(dd, n, max_numel, sumsq, 1e9, 1e-3, 0.9, 0.999, 1e-8, step, fused=True), args.reps)
    out.append(("adam one launch", us, adam_bytes))
    us = timed(lambda: K.adam_step(dd, n, max_numel, sumsq, 1e9, 1e-3, 0.9, 0.999, 1e-8, step), args.reps)
    out.append(("adam two launches", us, adam_bytes))
    w1 = K.descs_to_device(descs[:1], dev)    # the input weight alone: a grid with no idle tensors
    us = timed(lambda: K.adam_step(w1, 1, max_numel, sumsq, 1e9, 1e-3, 0.9, 0.999, 1e-8, step, fused=True), args.reps)
    out.append(("adam one launch, input weight alone", us, 28 * descs[0].numel + 4 * descs[0].numel))
    us = timed(lambda: K.grad_sumsq(w1, 1, max_numel, 1, sumsq, ws, ticket=ticket), args.reps)
    out.append(("grad_sumsq one launch, input weight alone", us, 4 * descs[0].numel))
    src = torch.empty(adam_bytes // 8, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    us = timed(lambda: dst.copy_(src), args.reps)
    out.append(("torch copy, Adam's bytes", us, adam_bytes))
    src2 = torch.empty(norm_bytes // 4, dtype=torch.float32, device=dev)
    us = timed(lambda: src2.sum(), args.reps)
    out.append(("torch sum, the norm's bytes", us, norm_bytes))
    us = timed(lambda: K.zero_(sumsq), args.reps)
    out.append(("empty-ish launch (llp_zero 4 B)", us, 4))
    for what, us, byts in out:
        print(json.dumps({"what": what, "us": round(us, 2), "bytes": byts, "GBps": round(byts / us / 1e3, 1),
                          "n_tensors": n, "numel": numel}), flush=True)


if __name__ == "__main__":
    main()
