"""Full-batch LLP distillation (train(), src/main.py:147-236) at the
coauthor-physics production shape (BASELINE configs[3]; scripts/LLP_production.sh:5):
synthetic Coauthor-Physics graph (34,493 nodes, 8,415 binary features, 247,962
undirected edges) split by the reference's do_production_edge_split, student
MLP 8,415 -> 256 -> 256 over the old-node training graph every link batch,
LLP_D=10 LLP_R=0.01 True_label=0.1, rw_step=2 hops=2 ns_rate=4 (C=20), PyG
dense negatives.  Prints one JSON line: ms per link batch and edges/s, per
dtype; --emulate-ranks R times rank 0's shard of each batch (no collective).  The timed
steps are eager launches (--graph: replays of capture_fullbatch's hipGraph).

    python tools/physics_bench.py [--steps 10] [--dtype bf16] [--emulate-ranks 4 [--replicated]] [--graph]
"""
import argparse
import json
import os
import sys
import tempfile
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_engine  # noqa: E402
import llp_split  # noqa: E402
import models  # noqa: E402


def physics_args():
    # scripts/LLP_production.sh:5 with main.py's defaults (src/main.py:240-269)
    return types.SimpleNamespace(datasets="coauthor-physics", KD_RM=0.0, LLP_D=10.0, KD_LM=0.0, LLP_R=0.01,
                                 True_label=0.1, dropout=0.0, encoder="sage", hops=2, lr=0.0005, margin=0.2,
                                 ns_rate=4, rw_step=2, ps_method="nb", transductive="production",
                                 hidden_channels=256, num_layers=2, link_batch_size=64 * 1024, predictor="mlp")


def _hb_two_kernel(self, R, tgt, dZ, drow, h, out, grouped_in=False):
    """A/B (--hb-two-kernel): the round-3 Hadamard backward of DistillEngine._hadamard_bwd_nodes,
    the row kernel writing a [2R, H] buffer, then the per-node segment sum."""
    K = llp_engine.K
    N, H = self.N, h.shape[1]
    R2 = 2 * R
    uniq = self._buf("hb_uniq", (R2,), torch.int32)
    pos = self._buf("hb_pos", (R2,), torch.int32)
    n_u = self._buf("hb_nu", (1,), torch.int32)
    seg_ptr = self._buf("hb_segp", (R2 + 1,), torch.int32)
    seg_rows = self._buf("hb_segr", (R2,), torch.int32)
    wsd = self._buf("hb_ws", (K.dedup_ws_bytes(N, R2) // 4 + 16,), torch.float32)
    K.dedup_rows(N, R2, tgt, uniq, pos, n_u, seg_ptr, seg_rows, wsd)
    dh_rows = self._buf("hb_rows", (R2, H), h.dtype)
    K.hadamard_bwd_blocks(0, 1, R, H, dZ, h, dh_rows, drow=drow, hidx=tgt)
    out.zero_()
    K.segment_sum_rows(min(R2, N), seg_ptr, seg_rows, dh_rows, out, count=n_u, out_rows=uniq)


def run(dtype, steps, warmup, emulate, split, shard_student=True, graph=False, sparse_input=True, host_slices=False):
    dev = torch.device("cuda", 0)
    a = physics_args()
    td = split[0]                                     # training_data: old nodes, old-old edges
    N, F = td.x.size(0), td.x.size(1)
    E = td.edge_index.size(1)
    P_full = a.link_batch_size
    B_full = int(N / (E / P_full))                    # src/main.py:345-346
    torch.manual_seed(1)
    model = models.MLP(a.num_layers, F, a.hidden_channels, a.hidden_channels, a.dropout).to(dev)
    pred = models.LinkPredictor("mlp", a.hidden_channels, a.hidden_channels, 1, a.num_layers, a.dropout).to(dev)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, a.dropout).to(dev)
    for p in tpred.parameters():
        p.requires_grad = False
    t_h = torch.randn(N, 256) * 0.3
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    row, col = td.edge_index
    eng = llp_engine.DistillEngine(model, pred, tpred, td.x.to(dev), t_h.to(dev), row.numpy(), col.numpy(), N, a,
                                   opt, dtype=dtype, seed=11, shard_student=shard_student, sparse_input=sparse_input)
    if emulate and shard_student:
        eng.emulate_shard = (0, emulate)      # rank 0's slice of the node-sharded student (default)
    pairs = td.edge_index.t().to(torch.int32).to(dev).contiguous()      # pos_train_edge (src/main.py:153)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    link_perm = torch.randperm(E, generator=g, device=dev).to(torch.int32)
    node_perm = torch.randperm(N, generator=g, device=dev).to(torch.int32)
    n_full = min(E // P_full, N // B_full)
    R = emulate if emulate else 1
    b0, b1 = 0, B_full // R
    p0, p1 = 0, P_full // R

    def step(s):
        j = s % n_full
        eng.step_fullbatch(node_perm[j * B_full + b0: j * B_full + b1], link_perm[j * P_full + p0: j * P_full + p1],
                           pairs, b_offset=b0, p_offset=p0, B_total=B_full, P_total=P_full, dense_negatives=True)

    for s in range(warmup):
        step(s)
    g_a = g_l = replay = None
    if graph:   # the step replayed from a hipGraph (capture_fullbatch), inputs refilled per replay
        g_a = torch.empty(b1 - b0, dtype=torch.int32, device=dev)
        g_l = torch.empty(p1 - p0, dtype=torch.int32, device=dev)
        # the graph fills its inputs with batch j = step_ctr mod n_full (llp_batch_slices): no host copy
        # per replay (--host-slices: two device-to-device copies before each replay, the round-4 loop)
        batches = None if host_slices else (node_perm, B_full, b0, link_perm, P_full, p0, n_full)
        replay = eng.capture_fullbatch(g_a, g_l, pairs, b_offset=b0, p_offset=p0, B_total=B_full, P_total=P_full,
                                       dense_negatives=True, batches=batches)
    torch.cuda.synchronize()
    eng.begin_epoch()
    t0 = time.perf_counter()
    for s in range(steps):
        if replay is not None:
            if host_slices:
                j = (warmup + s) % n_full
                g_a.copy_(node_perm[j * B_full + b0: j * B_full + b1])
                g_l.copy_(link_perm[j * P_full + p0: j * P_full + p1])
            replay.replay()
        else:
            step(warmup + s)
    t_issue = (time.perf_counter() - t0) / steps    # host time to enqueue a step (the GPU runs behind it)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    loss = eng.end_epoch(steps * P_full)
    return {"dtype": dtype, "ms_per_step": dt * 1e3, "edges_per_s": P_full / dt if not emulate else None,
            "emulated_ranks": emulate or None, "fb_shard": eng.emulate_shard is not None, "N_old": N, "F": F, "E_train_directed": E, "anchors_per_step": B_full,
            "contexts_per_anchor": a.rw_step * a.hops * (1 + a.ns_rate), "edges_per_step": P_full,
            "steps_per_epoch": -(-E // P_full), "loss": loss, "hipgraph": replay is not None,
            "host_issue_ms_per_step": t_issue * 1e3, "sparse_first_layer": eng.xs is not None,
            "batch_inputs": None if replay is None else ("host copies" if host_slices else "in-graph slices")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="bf16,fp32")
    ap.add_argument("--emulate-ranks", type=int, default=0)
    ap.add_argument("--replicated", action="store_true", help="every rank runs the student over all nodes")
    ap.add_argument("--graph", action="store_true",
                    help="replay a hipGraph of the step (capture_fullbatch); eager measured faster, "
                         "profiles/r03_physics_devcount_graph_ab.txt")
    ap.add_argument("--dense-input", action="store_true",
                    help="A/B: the first student layer as dense GEMMs over x (not llp_spmm_rows / llp_spmm_tn)")
    ap.add_argument("--data-dir", default=os.path.join(tempfile.gettempdir(), "llp_physics"))
    ap.add_argument("--no-edge-table", action="store_true",
                    help="A/B: the dense negative sampler's membership test by binary search of the sorted keys")
    ap.add_argument("--no-overlap", action="store_true",
                    help="A/B: one stream (DistillEngine.overlap_streams = False): the dense negatives and the frozen "
                         "teacher after the student / predictor forward instead of beside them")
    ap.add_argument("--hb-two-kernel", action="store_true",
                    help="A/B: the round-3 two-kernel Hadamard backward (profiles/r03_hb_fused_fb_ab.txt)")
    ap.add_argument("--late-pairs", action="store_true",
                    help="A/B (two streams): the frozen teacher and the node grouping start after the student "
                         "forward (DistillEngine.early_pair_work = False), as with a row-sharded student")
    ap.add_argument("--main-grouping", action="store_true",
                    help="A/B (two streams): the Hadamard backward's node grouping on the main stream, before "
                         "its per-node sums (DistillEngine.side_grouping = False)")
    ap.add_argument("--main-sampler", action="store_true",
                    help="A/B (two streams): the context sampler on the main stream before the student forward "
                         "(DistillEngine.side_sampling = False)")
    ap.add_argument("--main-wgrad", action="store_true",
                    help="A/B (two streams): the student's small weight-gradient GEMMs on the main stream before "
                         "the data gradients (DistillEngine.side_wgrad = False)")
    ap.add_argument("--host-slices", action="store_true",
                    help="A/B (--graph): refill the graph's input batch by two copies before each replay instead "
                         "of the in-graph llp_batch_slices")
    opt = ap.parse_args()
    if opt.no_edge_table:
        _nsd = llp_engine.K.neg_sample_dense
        llp_engine.K.neg_sample_dense = lambda *a, edge_table=None, **kw: _nsd(*a, **kw)
    if opt.hb_two_kernel:
        llp_engine.DistillEngine._hadamard_bwd_nodes = _hb_two_kernel
    if opt.no_overlap or opt.late_pairs or opt.main_grouping or opt.main_wgrad or opt.main_sampler or opt.hb_two_kernel:
        _init = llp_engine.DistillEngine.__init__

        def _init_switches(self, *a, **kw):
            _init(self, *a, **kw)
            self.overlap_streams = not opt.no_overlap
            self.early_pair_work = not opt.late_pairs
            self.side_grouping = not (opt.main_grouping or opt.hb_two_kernel)
            self.side_wgrad = not opt.main_wgrad
            self.side_sampling = not opt.main_sampler
        llp_engine.DistillEngine.__init__ = _init_switches
    t0 = time.perf_counter()
    split = llp_split.production_split("coauthor-physics", opt.data_dir, synthetic=True)
    prep = time.perf_counter() - t0
    out = {"workload": "coauthor-physics production LLP distillation (train, full-batch student)",
           "split_s": prep, "runs": []}
    for dt in opt.dtype.split(","):
        out["runs"].append(run(dt, opt.steps, opt.warmup, opt.emulate_ranks, split, not opt.replicated,
                               opt.graph, not opt.dense_input, opt.host_slices))
        print(json.dumps(out["runs"][-1]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
