"""SAGE teacher at the ogbl-collab shape (N=235,868, E=2,358,104 directed,
F=128 -> 256 -> 256 -> 256): CSR mean-aggregate bandwidth (forward and the
transposed backward) against the 8 TB/s HBM roofline, and one full teacher
train() step.  Algorithmic bytes per aggregate:
    E*F*s (neighbour rows) + 4E (col) + 4(N+1) (rowptr) + N*F*s (write)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_data  # noqa: E402
import llp_hip as K  # noqa: E402
import llp_sage  # noqa: E402
import llp_teacher  # noqa: E402
import models  # noqa: E402


def agg_only(iters, orders=("id",)):
    """Each configuration's launches in a fixed order: tools/pmc_kernels.py matches the
    csr_agg dispatches of a PMC pass to it by position.  order "locality": the graph's nodes
    renumbered by llp_sage.locality_order first, as TeacherEngine runs them."""
    dev = torch.device("cuda", 0)
    data = llp_data.synthetic_collab(seed=0, with_eval=False)
    N = data.N
    plan = []
    for order in orders:
        ei = data.edge_index
        if order == "locality":
            _, pi = llp_sage.locality_order(ei, N)
            ei = torch.from_numpy(pi[ei.numpy()])
        g = llp_sage.Graph(ei, N, dev)
        E = g.num_edges
        _agg_configs(g, N, E, iters, dev, plan, order)
    print(json.dumps({"N": N, "E": E, "plan": plan}))


def _agg_configs(g, N, E, iters, dev, plan, order):
    for dts in ("fp32", "bf16"):
        dt = torch.float32 if dts == "fp32" else torch.bfloat16
        es = 4 if dts == "fp32" else 2
        for F_ in (128, 256):
            x = torch.randn(N, F_, device=dev).to(dt)
            out = torch.empty(N, F_, device=dev, dtype=dt)
            for mode, (rp, cl, w) in (("fwd", (g.rowptr, g.col, None)), ("bwd", (g.rowptr_t, g.col_t, g.inv_deg))):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(3):
                    K.csr_aggregate(N, F_, rp, cl, x, w, 0 if mode == "fwd" else 1, out)
                s.record()
                for _ in range(iters):
                    K.csr_aggregate(N, F_, rp, cl, x, w, 0 if mode == "fwd" else 1, out)
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / iters
                nbytes = E * F_ * es + 4 * E + 4 * (N + 1) + N * F_ * es + (4 * E if mode == "bwd" else 0)
                compulsory = N * F_ * es + 4 * E + 4 * (N + 1) + N * F_ * es + (4 * N if mode == "bwd" else 0)
                plan.append({"order": order, "dtype": dts, "F": F_, "mode": mode, "launches": 3 + iters, "ms": ms,
                             "algorithmic_bytes": nbytes, "compulsory_bytes": compulsory,
                             "algorithmic_GBs": nbytes / (ms * 1e-3) / 1e9})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--agg-only", action="store_true",
                    help="every aggregate configuration (fp32 / bf16, F 128 / 256, fwd / bwd), 3 warm-up + --iters "
                         "launches each, in the printed order (rocprofv3 --pmc passes), then exit")
    ap.add_argument("--no-agg", action="store_true", help="only the teacher step (kernel traces of it)")
    ap.add_argument("--orders", default="id", help="--agg-only node orders, comma-separated: id, locality")
    ap.add_argument("--no-fused-wgrad", action="store_true",
                    help="A/B: SAGEConv's two weight gradients as two GEMMs (TeacherEngine.fused_wgrad = False)")
    opt = ap.parse_args()
    if opt.agg_only:
        return agg_only(opt.iters, tuple(opt.orders.split(",")))
    dev = torch.device("cuda", 0)
    dt = torch.float32 if opt.dtype == "fp32" else torch.bfloat16
    data = llp_data.synthetic_collab(seed=0, with_eval=False)
    N = data.N
    g = llp_sage.Graph(data.edge_index, N, dev)
    E = g.num_edges
    es = 4 if dt == torch.float32 else 2
    res = {"N": N, "E": E, "dtype": opt.dtype, "aggregate": []}
    for F_ in (() if opt.no_agg else (128, 256)):
        x = torch.randn(N, F_, device=dev).to(dt)
        out = torch.empty(N, F_, device=dev, dtype=dt)
        for mode, (rp, cl, w) in (("fwd", (g.rowptr, g.col, None)), ("bwd", (g.rowptr_t, g.col_t, g.inv_deg))):
            for _ in range(3):
                K.csr_aggregate(N, F_, rp, cl, x, w, 0 if mode == "fwd" else 1, out)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(opt.iters):
                K.csr_aggregate(N, F_, rp, cl, x, w, 0 if mode == "fwd" else 1, out)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / opt.iters
            nbytes = E * F_ * es + 4 * E + 4 * (N + 1) + N * F_ * es + (4 * E if mode == "bwd" else 0)
            gbs = nbytes / (ms * 1e-3) / 1e9
            res["aggregate"].append({"F": F_, "mode": mode, "ms": ms, "GB/s": gbs, "frac_hbm": gbs / 8000.0,
                                     "bytes": nbytes})
    # full teacher step: SAGE 128 -> 256 x3 (collab teacher: --num_layers=3), predictor 256/2 layers
    torch.manual_seed(0)
    model = models.SAGE("collab", data.F, 256, 256, 3, 0.5, llp_sage.SAGEConv).to(dev)
    pred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.5).to(dev)
    optim = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=0.005)
    eng = llp_teacher.TeacherEngine(model, pred, data.x.to(dev), data.edge_index, N, optim, dtype=opt.dtype)
    eng.fused_wgrad = not opt.no_fused_wgrad
    pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
    P = 64 * 1024
    perm = torch.randperm(pairs.shape[0], device=dev).to(torch.int32)
    nb = max(1, pairs.shape[0] // P)   # full batches of one epoch, reused past it
    for i in range(2):
        eng.step(perm[(i % nb) * P:(i % nb + 1) * P], pairs, dense_negatives=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(opt.steps):
        eng.step(perm[(i % nb) * P:(i % nb + 1) * P], pairs, dense_negatives=False)
    torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / opt.steps
    res["teacher_step_ms"] = dt_s * 1e3
    res["teacher_edges_per_s"] = P / dt_s
    print(json.dumps(res))


if __name__ == "__main__":
    main()
