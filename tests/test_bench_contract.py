"""CPU checks of bench.py's accounting (no GPU): the step FLOP of SURVEY.md §8d,
the PMC traffic lookup of the committed profile, the hipGraph default per world
size, and the collab configuration it measures (scripts/LLP_transductive.sh:8)."""
import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_step_flops_matches_survey():
    """≈17.4 TFLOP per collab step, ≈266 MFLOP per positive edge."""
    a = bench.collab_args()
    C = a.rw_step * a.hops * (1 + a.ns_rate)
    B, P, F, H, L = 13_110, 65_536, 128, a.hidden_channels, a.num_layers
    f = bench.step_flops(B, C, P, F, H, L)
    assert C == 36
    assert 17.3e12 < f < 17.6e12
    assert 260e6 < f / P < 270e6
    # on the unique nodes (U ≈ 225k) the executed work is ≈10.6 TFLOP
    fu = bench.step_flops(B, C, P, F, H, L, rows_student=225_334)
    assert 10.5e12 < fu < 10.7e12
    # the student rows of the reference's layout: B(C+1) + 4P
    assert B * (C + 1) + 4 * P == 747_214


def test_pmc_traffic_reads_committed_profile():
    prof = bench.PMC_FILES["bf16"]
    p = json.load(open(prof))
    t = bench.pmc_traffic(p["rows"], p["H"], p["dtype"])
    assert t == pytest.approx(p["traffic_bytes_per_launch"], rel=1e-9)
    assert t / p["algorithmic_bytes"] == pytest.approx(p["traffic_over_algorithmic"], rel=1e-9)
    assert bench.pmc_traffic(p["rows"], 2 * p["H"], p["dtype"]) is None        # another shape
    assert bench.pmc_traffic(p["rows"], p["H"], "fp16") is None                 # no such profile


def test_graph_default_at_every_world_size():
    assert bench.use_graph(None, 1) is True
    assert bench.use_graph(None, 2) is True
    assert bench.use_graph(None, 8) is True
    assert bench.use_graph(True, 8) is True
    assert bench.use_graph(False, 1) is False


def test_collab_configuration():
    a = bench.collab_args()
    assert (a.hidden_channels, a.num_layers, a.hops, a.rw_step, a.ns_rate) == (1024, 3, 3, 3, 3)
    assert a.link_batch_size == 65_536 and a.dropout == 0.0 and a.minibatch
    assert a.ps_method == "nb" and a.predictor == "mlp"


def test_cpu_baseline_leg_runs_on_the_host():
    """bench.py's cpu_baseline leg (the oracle's train_minibatch on a bounded sample),
    at a reduced shape: the fields the bench line carries."""
    import torch

    import llp_data
    import models
    a = bench.collab_args()
    a.hidden_channels = 32
    data = llp_data.synthetic_collab(seed=0, scale=0.01, with_eval=False)
    torch.manual_seed(1)
    H = a.hidden_channels
    model = models.MLP(a.num_layers, data.F, H, H, 0.0)
    pred = models.LinkPredictor("mlp", H, H, 1, a.num_layers, 0.0)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0)
    init = tuple([p.detach().clone() for p in m.parameters()] for m in (model, pred, tpred))
    t_h = torch.randn(data.N, 256) * 0.3
    P_full = 1024
    B_full = int(data.N / (data.train_pairs.shape[0] / P_full))
    r = bench.cpu_baseline(data, a, t_h, init, B_full, P_full, sample_P=128, steps=1)
    assert r["kind"] == "port" and r["unit"] == "edges/s" and r["value"] > 0
    assert r["cores"] == torch.get_num_threads()
    assert "128 edges" in r["sample"]
