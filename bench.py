#!/usr/bin/env python
"""Headline benchmark: ogbl-collab LLP relational distillation (train_minibatch,
src/main.py:52-144) at the collab script's configuration
(scripts/LLP_transductive.sh:8: --hidden_channels=1024 --num_layers=3 --hops=3
--rw_step=3 --ns_rate=3 --ps_method=nb --LLP_D=1 --LLP_R=0 --True_label=1
--margin=0.01 --lr=0.001 --dropout=0 --minibatch; link_batch_size 65,536,
node_batch_size 13,110) on synthetic collab-shape data.

One step = one link batch: device sampling, student MLP + LinkPredictor
forward/backward, frozen teacher predictor, fused LLP_D/LLP_R/BCE, clip, Adam.
Metric: positive training edges per second (the reference's
num_examples = edge.size(1), src/main.py:140), whole job.

Multi-GPU (torchrun): the global batch stays 65,536 edges / 13,110 anchors
(reference semantics) and is sharded across ranks; one RCCL all-reduce of the
gradients per step (strong scaling).

  python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "linkless-link-prediction_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "distillation edges/sec + Hits@20, ogbl-collab LLP at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def collab_args():
    return types.SimpleNamespace(hidden_channels=1024, num_layers=3, hops=3, rw_step=3, ns_rate=3, ps_method="nb",
                                 LLP_D=1.0, LLP_R=0.0, True_label=1.0, KD_RM=0.0, KD_LM=0.0, margin=0.01, lr=0.001,
                                 dropout=0.0, predictor="mlp", link_batch_size=64 * 1024, datasets="collab",
                                 transductive="transductive", minibatch=True)


def step_flops(B, C, P, F, H, L, rows_student=None):
    """Algorithmic FLOP of one distillation step; rows_student
    replaces the reference's B(C+1)+4P student rows by the rows executed (the
    engine runs the dropout-free student on unique nodes)."""
    rows_mlp = B * (C + 1) + 4 * P if rows_student is None else rows_student
    rows_pred = B * C + 2 * P
    fwd_mlp = 2 * rows_mlp * (F * H + (L - 1) * H * H)
    fwd_pred = 2 * rows_pred * ((L - 1) * H * H + H)
    fwd_t = 2 * B * C * (256 * 256 + 256)
    return 3 * (fwd_mlp + fwd_pred) - 2 * rows_mlp * F * H + fwd_t


def use_graph(flag, world):
    """--graph / --no-graph, else the default: the step replayed from a hipGraph at every
    N (at N>1 as graph segments with the RCCL all-reduces between them)."""
    return True if flag is None else bool(flag)


def cpu_baseline(data, a, t_h, init_params, B_full, P_full, sample_P=8192, steps=3):
    """The CPU oracle (torch-CPU restatement of train_minibatch) on a bounded
    sample of the same workload: one link batch of sample_P edges and the
    proportional anchor batch, same H/L/C.  Edges/s scales linearly with the
    batch, so the per-edge rate is comparable."""
    from oracle import llp_oracle as O
    B = max(1, int(B_full * sample_P / P_full))
    P = sample_P
    C = a.rw_step * a.hops * (1 + a.ns_rate)
    x = data.x
    stu = [p.clone().requires_grad_() for p in init_params[0]]
    prd = [p.clone().requires_grad_() for p in init_params[1]]
    tp = init_params[2]
    adam = O.AdamState(stu + prd, lr=a.lr)
    rowptr, colv = None, None
    import llp_engine
    rowptr, colv = llp_engine.build_sampler_csr(data.edge_index[0].numpy(), data.edge_index[1].numpy(), data.N)
    rng = np.random.default_rng(1)
    nthreads = torch.get_num_threads()
    t0 = time.perf_counter()
    for s in range(steps):
        anchors = rng.permutation(data.N)[:B]
        pos, neg = O.neighbor_samplers(rowptr, colv, anchors, data.N, a.rw_step, a.ps_method, a.ns_rate, a.hops,
                                       seed=5, stream_base=O.STREAMS_PER_STEP * s)
        samples = torch.from_numpy(np.concatenate([pos, neg], 1))
        link = rng.integers(0, data.train_pairs.shape[0], P)
        edge = data.train_pairs[link].t()
        negE = torch.from_numpy(O.randint_edges(data.N, P, seed=5, stream=O.STREAMS_PER_STEP * s + O.RANDINT_STREAM))
        r = O.distill_losses_minibatch(x, t_h, samples, edge, negE, stu[0::2], stu[1::2], prd[0::2], prd[1::2],
                                       tp[0::2], tp[1::2], a)
        new, _, _ = O.distill_step(stu, prd, adam, r["loss"])
        stu = [p.requires_grad_() for p in new[:len(stu)]]
        prd = [p.requires_grad_() for p in new[len(stu):]]
    dt = time.perf_counter() - t0
    assert C > 0
    return dict(value=P * steps / dt, unit="edges/s", cores=nthreads, kind="port",
                sample=f"{steps} oracle train_minibatch steps of {P} edges / {B} anchors at the collab shape "
                       f"(H=1024, L=3, C={C}); {dt:.1f} s on {nthreads} threads")


class Shard:
    """This rank's part of every global batch (B_full anchors, P_full edges): the whole batch
    under the engine's owner decomposition (DistillEngine.minibatch_owner: each rank picks its
    pairs itself), else its contiguous slice of both with offsets and global totals."""

    def __init__(self, eng, B_full, P_full, rank, world):
        self.B, self.P, self.rank, self.world = B_full, P_full, rank, world
        self.owner = eng.minibatch_owner
        if self.owner or world == 1:
            self.b0, self.b1, self.p0, self.p1 = 0, B_full, 0, P_full
            self.kw = {}
        else:
            self.b0, self.b1 = rank * B_full // world, (rank + 1) * B_full // world
            self.p0, self.p1 = rank * P_full // world, (rank + 1) * P_full // world
            self.kw = dict(b_offset=self.b0, p_offset=self.p0, B_total=B_full, P_total=P_full)
        self.name = "owner" if self.owner else ("whole batch" if world == 1 else "slice")

    def batch(self, node_perm, link_perm, j):
        return (node_perm[j * self.B + self.b0: j * self.B + self.b1],
                link_perm[j * self.P + self.p0: j * self.P + self.p1])

    def pairs(self, C):
        """Predictor rows of this rank per step."""
        if self.owner:
            r, w = self.rank, self.world
            return sum((r + 1) * n // w - r * n // w for n in (self.B * C, self.P, self.P))
        return (self.b1 - self.b0) * C + 2 * (self.p1 - self.p0)


def emulated_rank(eng, node_perm, link_perm, pairs, B_full, P_full, n_full, C, R, steps=20, rank=0):
    """Rank ``rank``'s part of an R-rank collab step on this GPU, replayed from a hipGraph (the
    N-rank step replays graph segments with the all-reduces between them): ms per step."""
    eng.emulate_pairs = (rank, R)
    try:
        sh = Shard(eng, B_full, P_full, rank, R)
        step = lambda j: eng.step_minibatch(*sh.batch(node_perm, link_perm, j % n_full), pairs, **sh.kw)
        for s in range(3):
            step(s)
        ga, gl = (t.clone() for t in sh.batch(node_perm, link_perm, 3 % n_full))
        g = eng.capture_minibatch(ga, gl, pairs, batches=(node_perm, sh.B, sh.b0, link_perm, sh.P, sh.p0, n_full),
                                  **sh.kw)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for s in range(steps):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t1) / steps * 1e3
        rows = eng.last_student_rows
        del g
    finally:
        eng.emulate_pairs = None
    return {"ms_per_step": ms, "ranks": R, "rank": rank, "decomposition": sh.name, "hipgraph": True,
            "student_rows": rows, "predictor_rows": sh.pairs(C)}


def dominant_only(eng, batch, pairs, kw, n):
    """One real step (buffers filled), then the dominant kernel alone n times:
    the command rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes profile."""
    import llp_hip as K
    eng.step_minibatch(*batch, pairs, **kw)
    lin = eng.stu[1]
    A = eng._bufs["H0"]
    cnt = eng._rows_dev                       # the step's launch: host bound, device unique count
    R1 = A.numel() // lin.in_f if cnt is not None else eng.last_student_rows
    out = eng._buf("H1", (R1, lin.out_f), eng.dtype)
    a_op = K.operand(A[:R1 * lin.in_f].view(R1, lin.in_f), count=cnt)
    hm = eng._bufs.get("Hm1")                 # the step's launch also writes the ReLU bit mask
    hm = hm[:R1 * (lin.out_f // 8)].view(R1, lin.out_f // 8) if hm is not None else None
    for _ in range(n):
        K.gemm_nt(a_op, K.operand(lin.Wcomp), R1, lin.out_f, lin.in_f, out, eng.dc, bias=lin.b, act=K.ACT_RELU,
                  aux=hm)
    torch.cuda.synchronize()
    print(json.dumps({"dominant_rows": R1, "H": lin.out_f, "launches": n}), flush=True)


PMC_FILES = {"bf16": os.path.join(REPO, "profiles", "r06_pmc_dominant.json"),
             "fp32": os.path.join(REPO, "profiles", "r06_fp32_pmc_dominant.json")}


def pmc_traffic(rows, H, dtype):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC passes (profiles/r06_pmc_dominant.json, r06_fp32_pmc_dominant.json;
    tools/pmc_summary.py): 2 x FETCH_SIZE (gfx950 reports half of a wide
    streaming read) + WRITE_SIZE, per dispatch.  None when the profile is
    absent or for another shape."""
    try:
        with open(PMC_FILES[dtype]) as f:
            p = json.load(f)
    except (OSError, ValueError, KeyError):
        return None
    if p.get("H") != H or p.get("dtype") != dtype or not p.get("rows"):
        return None
    # the unique-node count varies a little from step to step: scale the measured
    # launch linearly in M (the A panel and C are M x H, W is fixed) within 5 %
    if abs(rows - p["rows"]) > 0.05 * p["rows"]:
        return None
    return p.get("traffic_bytes_per_launch") * rows / p["rows"]


def evaluate(model, pred, data, dev):
    """Hits@K / AUC on the synthetic held-out split through the device eval
    path (llp_eval: test_transductive, src/train_teacher_gnn.py:76-155), fp32."""
    import llp_eval
    t0 = time.perf_counter()
    model.eval()
    pred.eval()
    h = llp_eval.embed_mlp(model, data.x.to(dev))
    score = llp_eval.EdgeScorer(pred)
    out = {}
    for split in ("valid", "test"):
        p = score(h, data.split_edge[split]["edge"].to(dev))
        n = score(h, data.split_edge[split]["edge_neg"].to(dev))
        for k, v in zip((10, 20, 50, 100), llp_eval.K.hits_at_k(p, n, (10, 20, 50, 100))):
            out.setdefault(f"Hits@{k}", {})[split] = v
    torch.cuda.synchronize()
    return {"hits@20": out["Hits@20"], "hits": out, "eval_ms": (time.perf_counter() - t0) * 1e3,
            "hits_note": "after the timed steps from random init on synthetic data (not a converged model)"}


SAGE_PMC_FILE = os.path.join(REPO, "profiles", "r05_pmc_sage_orders.json")


def practical_peak(dev, seconds=0.2, dtype="bf16"):
    """MFMA FLOP/s this device sustains on random operands (llp_mfma_probe: a bare
    v_mfma_f32_16x16x32_bf16 loop on every CU, two waves per SIMD; dtype "fp32":
    llp_mfma_probe_f32, the same loop on v_mfma_f32_16x16x4_f32), event-timed on the
    launch stream: the clock the chip holds under dense MFMA load on random data sets it
    well under the spec peak (MI355X_MICROARCH.md, DVFS give-back)."""
    import llp_hip as K
    g = torch.Generator(device="cpu").manual_seed(11)
    data = torch.randn(1 << 16, generator=g).to(torch.bfloat16 if dtype == "bf16" else torch.float32).to(dev)
    out = torch.empty(K.mfma_probe_out_floats(), dtype=torch.float32, device=dev)
    probe = K.mfma_probe if dtype == "bf16" else K.mfma_probe_f32
    iters = 20000 if dtype == "bf16" else 5000
    probe(data, iters, out)      # warm-up, and a first estimate of the rate
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fl = probe(data, iters, out)
    e1.record()
    torch.cuda.synchronize()
    rate = fl / (e0.elapsed_time(e1) * 1e-3)
    iters = max(1000, int(iters * seconds / (fl / rate)))
    e0.record()
    fl = probe(data, iters, out)
    e1.record()
    torch.cuda.synchronize()
    return fl / (e0.elapsed_time(e1) * 1e-3) / 1e12


def sage_aggregate(data, dev):
    """SAGE teacher's CSR mean aggregate (a11, src/sageconv_updated.py:65-81 / PyG SAGEConv mean)
    at the collab shape, forward, F = 128 and 256, fp32 and bf16, event-timed live, on the
    graph in TeacherEngine's node order (llp_sage.locality_order: neighbour rows mostly hit L2).
    algorithmic bytes E*F*s + 4E + 4(N+1) + N*F*s (every neighbour row from memory, SURVEY
    §8d); compulsory bytes: x, col, rowptr read once, out written once; traffic: beyond-L2
    counter bytes per launch from the committed PMC passes of the same order
    (profiles/r05_pmc_sage_orders.json: 2 x FETCH_SIZE + WRITE_SIZE, Infinity-Cache hits
    included, so an upper bound on HBM bytes).  frac = traffic / time / 8 TB/s."""
    import llp_hip as K
    import llp_sage
    _, pi = llp_sage.locality_order(data.edge_index, data.N)
    g = llp_sage.Graph(torch.from_numpy(pi[data.edge_index.numpy()]), data.N, dev)
    try:
        with open(SAGE_PMC_FILE) as f:
            pmc = {(c["dtype"], c["F"], c["mode"]): c["counter_bytes"] for c in json.load(f)["configs"]
                   if c.get("order") == "locality"}
    except (OSError, ValueError, KeyError):
        pmc = {}
    out = []
    for dts, dt, es in (("fp32", torch.float32, 4), ("bf16", torch.bfloat16, 2)):
        for F_ in (128, 256):
            x = torch.randn(data.N, F_, device=dev).to(dt)
            y = torch.empty_like(x)
            for _ in range(3):
                K.csr_aggregate(data.N, F_, g.rowptr, g.col, x, None, 0, y)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            s.record()
            for _ in range(n):
                K.csr_aggregate(data.N, F_, g.rowptr, g.col, x, None, 0, y)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / n
            algo = g.num_edges * F_ * es + 4 * g.num_edges + 4 * (data.N + 1) + data.N * F_ * es
            comp = 2 * data.N * F_ * es + 4 * g.num_edges + 4 * (data.N + 1)
            traffic = pmc.get((dts, F_, "fwd"))
            tb = (traffic if traffic else algo) / (ms * 1e-3)
            out.append({"kernel": "csr_agg_lds_kernel fwd", "order": "locality", "dtype": dts, "F": F_, "N": data.N,
                        "E": g.num_edges, "ms": ms, "achieved": tb / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "traffic_over_compulsory": traffic / comp if traffic else None,
                        "frac": tb / 1e9 / PEAK_HBM_GBS, "traffic": traffic, "algorithmic_bytes": algo,
                        # operand bytes (every neighbour row counted) per second: a gather rate,
                        # not an HBM figure -- most neighbour reads hit L2 / Infinity Cache
                        "operand_read_rate_GBs": algo / (ms * 1e-3) / 1e9, "compulsory_bytes": comp,
                        "compulsory_frac": comp / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                        "note": "achieved/frac on PMC beyond-L2 bytes (Infinity-Cache hits counted: x fits the "
                                "256 MiB cache, so most neighbour re-reads are cache hits, not HBM reads)"})
    return out


def sage_teacher_step(data, dev, dtype, steps=5):
    """One teacher train() batch (src/train_teacher_gnn.py:33-71, §8 a11-a13) at
    the collab shape: 3-layer SAGE 128 -> 256 over the full graph, predictor
    256/2, 65,536 positives + randint negatives, bf16 TeacherEngine."""
    import llp_sage
    import llp_teacher
    import models
    torch.manual_seed(0)
    # dropout 0.5: train_teacher_gnn.py's default (src/train_teacher_gnn.py:277), live in the encoder
    # and the predictor (fused Philox masks in the GEMM epilogues)
    model = models.SAGE("collab", data.F, 256, 256, 3, 0.5, llp_sage.SAGEConv).to(dev)
    pred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.5).to(dev)
    optim = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=0.005)
    eng = llp_teacher.TeacherEngine(model, pred, data.x.to(dev), data.edge_index, data.N, optim, dtype=dtype)
    pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
    P = 64 * 1024
    perm = torch.randperm(pairs.shape[0], device=dev).to(torch.int32)
    for i in range(2):
        eng.step(perm[i * P:(i + 1) * P], pairs, dense_negatives=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.step(perm[i * P:(i + 1) * P], pairs, dense_negatives=False)
    torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / steps
    return {"ms_per_step": dt_s * 1e3, "edges_per_s": P / dt_s, "dtype": dtype,
            "config": "SAGE 3x(128->256) over N=235,868 / E=2,358,104, LinkPredictor 256x2, dropout 0.5, "
                      "65,536 positives"}


def fp32_step(data, a, t_h, init, dev, steps=3):
    """The same collab step in fp32, the reference's arithmetic (fp32 GEMMs on the f32
    MFMA path, gemm.hip): a fresh engine from the same initial weights, one warm-up and
    ``steps`` timed eager steps."""
    import llp_engine
    import models
    N, F, H, L = data.N, data.F, a.hidden_channels, a.num_layers
    model = models.MLP(L, F, H, H, a.dropout).to(dev)
    pred = models.LinkPredictor("mlp", H, H, 1, L, a.dropout).to(dev)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, a.dropout).to(dev)
    for p, p0 in zip(list(model.parameters()) + list(pred.parameters()) + list(tpred.parameters()),
                     init[0] + init[1] + init[2]):
        p.data.copy_(p0)
    for p in tpred.parameters():
        p.requires_grad = False
    optim = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(dev), t_h.to(dev), data.edge_index[0].numpy(),
                                   data.edge_index[1].numpy(), N, a, optim, dtype="fp32", seed=123)
    pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
    E = data.train_pairs.shape[0]
    P = a.link_batch_size
    B = int(N / (E / P))
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    link_perm = torch.randperm(E, generator=gen, device=dev).to(torch.int32)
    node_perm = torch.randperm(N, generator=gen, device=dev).to(torch.int32)
    eng.step_minibatch(node_perm[:B], link_perm[:P], pairs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(1, steps + 1):
        eng.step_minibatch(node_perm[s * B:(s + 1) * B], link_perm[s * P:(s + 1) * P], pairs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # the dominant f32-MFMA launch (student layer 2, as in the bf16 line), event-timed on its stream
    ev = []
    for s in range(steps + 1, steps + 3):
        eng.step_minibatch(node_perm[s * B:(s + 1) * B], link_perm[s * P:(s + 1) * P], pairs, kernel_events=ev)
    torch.cuda.synchronize()
    k_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rows = eng.last_student_rows
    achieved = 2.0 * rows * H * H / (k_ms * 1e-3) / 1e12
    roof = {"bound": "mfma", "kernel": f"{getattr(eng, 'timed_kernel', '?')} student layer-2 forward "
                                       f"({rows}x{H}x{H})", "achieved": achieved, "peak": PEAK_F32_TFLOPS,
            "unit": "TFLOP/s", "frac": achieved / PEAK_F32_TFLOPS, "kernel_ms": k_ms,
            "traffic": pmc_traffic(rows, H, "fp32"),
            "algorithmic_bytes": 2.0 * rows * H * 4 + 4.0 * H * H}
    pp = practical_peak(dev, dtype="fp32")
    roof.update(practical_peak=pp, practical_frac=achieved / pp,
                practical_note="bare v_mfma_f32_16x16x4_f32 loop on random f32 operands, every CU (llp_mfma_probe_f32)")
    del eng
    torch.cuda.empty_cache()
    return {"dtype": "fp32", "ms_per_step": dt * 1e3, "edges_per_s": P / dt, "steps": steps, "roofline": roof,
            "note": "the reference's arithmetic; same configuration, eager steps"}


def physics_production_step(dtype):
    """BASELINE configs[3] at one GPU: the full-batch train() step at the
    coauthor-physics production shape (tools/physics_bench.py), plus rank 0's
    shard of the same batch at 4 ranks (no collective)."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import llp_split
    import physics_bench
    split = llp_split.production_split("coauthor-physics", os.path.join(tempfile.gettempdir(), "llp_physics"),
                                       synthetic=True)
    r1 = physics_bench.run(dtype, 10, 2, 0, split)
    r4 = physics_bench.run(dtype, 10, 2, 4, split)
    r1g = physics_bench.run(dtype, 10, 2, 0, split, graph=True)
    r4g = physics_bench.run(dtype, 10, 2, 4, split, graph=True)
    return {"config": "coauthor-physics production LLP (N_old=%d, F=%d, H=256, L=2, C=%d, 65,536 edges/step)"
                      % (r1["N_old"], r1["F"], r1["contexts_per_anchor"]),
            # the graph replay leads (it is the faster form at both widths); the eager figures follow
            "dtype": dtype, "ms_per_step": r1g["ms_per_step"], "edges_per_s": r1g["edges_per_s"],
            "rank0_ms_per_step_at_4_ranks": r4g["ms_per_step"], "hipgraph": True,
            "ms_per_step_graph": r1g["ms_per_step"], "rank0_ms_per_step_at_4_ranks_graph": r4g["ms_per_step"],
            "ms_per_step_eager": r1["ms_per_step"], "rank0_ms_per_step_at_4_ranks_eager": r4["ms_per_step"],
            "sparse_first_layer": r1["sparse_first_layer"],
            "note": "steps replayed from a hipGraph (capture_fullbatch, which fills its own input batch from the "
                    "epoch permutations: llp_batch_slices), and the same steps eagerly with no host sync (the dense "
                    "negatives' count stays on the device); two streams (samples, negatives, pairs, the frozen "
                    "teacher, the Hadamard backward's node grouping and the student's small weight gradients on a "
                    "side stream, DESIGN.md 4.7); rank 0 of 4 runs its slice of the node-sharded student, its "
                    "collectives emulated by copies"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-edges", type=int, default=8192)
    ap.add_argument("--scale", type=float, default=1.0, help="dataset scale (1.0 = ogbl-collab shape)")
    ap.add_argument("--profile-kernels", action="store_true", help="exit right after the timed region")
    ap.add_argument("--dominant-only", type=int, default=0,
                    help="run only the dominant kernel this many times (rocprofv3 --pmc passes) and exit")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=None,
                    help="replay the step from a captured hipGraph (N>1: graph segments with the RCCL "
                         "all-reduces between them; --no-graph: eager launches).  Default: on")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--no-sage", action="store_true")
    ap.add_argument("--no-physics", action="store_true")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 collab step leg")
    ap.add_argument("--no-shard8", action="store_true", help="skip the 8-rank per-rank shard leg")
    ap.add_argument("--no-practical-peak", action="store_true", help="skip the bare-MFMA probe (profiling runs)")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="single GPU: run only rank 0's shard of an R-rank job (no collective) and report "
                         "its per-step time, to see the per-rank fixed costs of strong scaling")
    ap.add_argument("--emulate-rank", type=int, default=0,
                    help="with --emulate-ranks R: which rank's shard (offsets) to run, default 0")
    opt = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # (rehearsal of N ranks on fewer GPUs: ranks share devices round-robin, LLP_BENCH_BACKEND=gloo)
    local_dev = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    backend = os.environ.get("LLP_BENCH_BACKEND", "nccl")
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    import llp_data
    import llp_engine
    import llp_hip as K
    import models

    a = collab_args()
    data = llp_data.synthetic_collab(seed=0, scale=opt.scale, with_eval=not opt.no_eval)
    N, F, H, L = data.N, data.F, a.hidden_channels, a.num_layers
    E_train = data.train_pairs.shape[0]
    P_full = a.link_batch_size
    B_full = int(N / (E_train / P_full))                    # src/main.py:335
    C = a.rw_step * a.hops * (1 + a.ns_rate)

    torch.manual_seed(1)
    model = models.MLP(L, F, H, H, a.dropout)
    pred = models.LinkPredictor("mlp", H, H, 1, L, a.dropout)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, a.dropout)
    t_h = torch.randn(N, 256) * 0.3
    init = ([p.detach().clone() for p in model.parameters()], [p.detach().clone() for p in pred.parameters()],
            [p.detach().clone() for p in tpred.parameters()])
    model, pred, tpred = model.to(dev), pred.to(dev), tpred.to(dev)
    for p in tpred.parameters():
        p.requires_grad = False
    optim = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(dev), t_h.to(dev), data.edge_index[0].numpy(),
                                   data.edge_index[1].numpy(), N, a, optim, dtype=opt.dtype, seed=123)
    pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    link_perm = torch.randperm(E_train, generator=g, device=dev).to(torch.int32)
    node_perm = torch.randperm(N, generator=g, device=dev).to(torch.int32)
    n_full = min(E_train // P_full, N // B_full)
    # this rank's part of every global batch (--emulate-ranks: one rank's part of an R-rank job on this GPU)
    shards = opt.emulate_ranks if (opt.emulate_ranks and world == 1) else world
    srank = opt.emulate_rank if (opt.emulate_ranks and world == 1) else rank
    if opt.emulate_ranks and world == 1:
        eng.emulate_pairs = (srank, shards)
    sh = Shard(eng, B_full, P_full, srank, shards)

    kern_ev = []

    def one_step(s, timed):
        eng.step_minibatch(*sh.batch(node_perm, link_perm, s % n_full), pairs,
                           kernel_events=kern_ev if timed else None, **sh.kw)

    if opt.dominant_only:
        dominant_only(eng, sh.batch(node_perm, link_perm, 0), pairs, sh.kw, opt.dominant_only)
        return
    graph_on = use_graph(opt.graph, world)
    debug = os.environ.get("LLP_BENCH_DEBUG") == "1"   # stage markers, each after a device sync

    def mark(what):
        if debug:
            torch.cuda.synchronize()
            print(f"[rank {rank}] {what}", flush=True)

    mark("engine ready")
    for s in range(opt.warmup):
        one_step(s, False)
        mark(f"warmup step {s}")
    graph = None
    if graph_on:
        # persistent input slots, filled inside the graph with batch j = step_ctr mod n_full of the epoch
        # permutations (llp_batch_slices): the timed loop is replays only
        g_anchors, g_links = (t.clone() for t in sh.batch(node_perm, link_perm, 0))
        batches = (node_perm, sh.B, sh.b0, link_perm, sh.P, sh.p0, n_full)
        try:
            graph = eng.capture_minibatch(g_anchors, g_links, pairs, batches=batches, **sh.kw)
            mark("captured")
        except RuntimeError as e:   # keep the run alive: eager launches instead (reported as hipgraph: false)
            print(f"bench.py: hipGraph capture failed ({e}); timing eager steps", file=sys.stderr, flush=True)
            graph = None
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.begin_epoch()
    t0 = time.perf_counter()
    for s in range(opt.steps):
        if graph is not None:
            graph.replay()
            mark(f"replay {s}")
        else:
            one_step(opt.warmup + s, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if opt.profile_kernels:
        if world > 1:
            dist.destroy_process_group()
        return
    if opt.emulate_ranks and world == 1:
        print(json.dumps({"emulated_ranks": shards, "rank": srank, "rank0_ms_per_step": dt / opt.steps * 1e3,
                          "decomposition": sh.name, "hipgraph": graph is not None,
                          "student_rows": eng.last_student_rows, "predictor_rows": sh.pairs(C)}), flush=True)
        return
    loss = eng.end_epoch(opt.steps * P_full)

    # dominant kernel: student layer-2 forward GEMM (rows_exec x 1024 x 1024, bf16 MFMA);
    # rows_exec = unique nodes of this rank's student rows
    rows_exec = eng.last_student_rows
    rows_all = torch.tensor([float(rows_exec)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(rows_all)
    if not kern_ev:   # graph mode: time the dominant kernel in a few eager steps after the timed region
        for s in range(3):
            one_step(opt.warmup + opt.steps + s, True)
        torch.cuda.synchronize()
    kt = [s.elapsed_time(e) for s, e in kern_ev]
    k_ms = float(np.mean(kt)) if kt else float("nan")
    k_flop = 2.0 * rows_exec * H * H
    peak = PEAK_BF16_TFLOPS if opt.dtype == "bf16" else PEAK_F32_TFLOPS
    achieved = k_flop / (k_ms * 1e-3) / 1e12
    flop_step = step_flops(B_full, C, P_full, F, H, L)
    flop_exec = step_flops(B_full, C, P_full, F, H, L, rows_student=float(rows_all.item()))

    res = None
    if rank == 0:
        value = P_full * opt.steps / dt
        res = {
            "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world, "steps": opt.steps,
            "warmup": opt.warmup, "ms_per_step": dt / opt.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": opt.dtype,
            "data": "synthetic (ogbl-collab shape: planted-partition graph, OGB-interleaved edges, random-init "
                    "weights, random teacher embeddings)",
            "config": {"workload": "ogbl-collab transductive LLP distillation (train_minibatch)", "N": N, "F": F,
                       "hidden": H, "num_layers": L, "anchors_per_step": B_full, "contexts_per_anchor": C,
                       "edges_per_step": P_full, "global_batch": P_full, "parallelism": f"dp{world}",
                       "step_tflop_reference": flop_step / 1e12, "step_tflop_executed": flop_exec / 1e12,
                       "student_rows_per_step": {"reference": B_full * (C + 1) + 4 * P_full,
                                                 "unique_nodes": int(rows_all.item())},
                       "mfma_util_step": flop_exec / (dt / opt.steps) / 1e12 / peak / world},
            "roofline": {"bound": "mfma", "kernel": f"{getattr(eng, 'timed_kernel', '?')} student layer-2 forward "
                         f"({rows_exec}x{H}x{H})", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": pmc_traffic(rows_exec, H, opt.dtype),
                         "algorithmic_bytes": 2.0 * rows_exec * H * 2 + 2.0 * H * H + rows_exec * H / 8.0,
                         "kernel_ms": k_ms},
            "loss": loss,
            "hipgraph": bool(graph is not None),
        }
        if not opt.no_practical_peak:
            pp = practical_peak(dev, dtype=opt.dtype)
            ins, fn = (("v_mfma_f32_16x16x32_bf16", "llp_mfma_probe") if opt.dtype == "bf16"
                       else ("v_mfma_f32_16x16x4_f32", "llp_mfma_probe_f32"))
            res["roofline"].update(practical_peak=pp, practical_frac=achieved / pp,
                                   practical_note=f"bare {ins} loop on random operands, every CU, timed here ({fn}): "
                                                  "the FLOP/s the chip sustains at the clock it holds under dense "
                                                  "MFMA load")
        if not opt.no_eval:
            res.update(evaluate(model, pred, data, dev))
        if world == 1 and not opt.no_shard8 and not opt.profile_kernels:
            # per-rank cost of strong scaling: rank 0's part of the same global batches at 8
            # ranks on this GPU, replayed from its hipGraph as the 8-GPU step's segments are
            # (no collective): the 8-GPU step is this + the all-reduces
            r8 = emulated_rank(eng, node_perm, link_perm, pairs, B_full, P_full, n_full, C, 8)
            res["rank0_ms_per_step_at_8_ranks"] = r8["ms_per_step"]
            res["rank0_at_8_ranks"] = r8
        if world == 1 and opt.dtype == "bf16" and not opt.no_fp32:
            res["fp32_step"] = fp32_step(data, a, t_h, init, dev)
        if not opt.no_sage:
            res["sage_aggregate"] = sage_aggregate(data, dev)
            res["sage_teacher_step"] = sage_teacher_step(data, dev, opt.dtype)
        if world == 1 and not opt.no_physics:
            res["physics_production_step"] = physics_production_step(opt.dtype)
        if world == 1 and not opt.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(data, a, t_h, init, B_full, P_full, sample_P=opt.cpu_sample_edges)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
