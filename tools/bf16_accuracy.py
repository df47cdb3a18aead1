"""bf16 against fp32 training on scaled synthetic ogbl-collab (BASELINE north_star: Hits@20
within 0.1 of the reference's; the reference trains in fp32).

The same initial weights, the same anchor / link permutations and the same device draws
(samples, negatives: integer work, identical in both dtypes) train one student in fp32 and
one in bf16 with the collab script's configuration (scripts/LLP_transductive.sh:8:
hidden 1024, 3 layers, hops 3, rw_step 3, ns_rate 3, LLP_D 1, True_label 1, lr 0.001,
dropout 0), then Hits@K on the held-out split through the device eval path in fp32
(test_transductive's collab keys, src/main.py:379-385, src/train_teacher_gnn.py:121-143).

    python tools/bf16_accuracy.py [--scale 0.1] [--link-batch 8192] [--epochs 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "linkless-link-prediction_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

KS = (10, 20, 50, 100)


def hits(model, pred, data, dev):
    import llp_eval
    import llp_hip as K
    model.eval()
    pred.eval()
    h = llp_eval.embed_mlp(model, data.x.to(dev))
    score = llp_eval.EdgeScorer(pred)
    out = {}
    for split in ("valid", "test"):
        p = score(h, data.split_edge[split]["edge"].to(dev))
        n = score(h, data.split_edge[split]["edge_neg"].to(dev))
        for k, v in zip(KS, K.hits_at_k(p, n, KS)):
            out.setdefault(f"Hits@{k}", {})[split] = v
    model.train()
    pred.train()
    return out


def train(dtype, data, epochs, link_batch, seed=0, hidden=1024, eval_every=1):
    """One run; returns the per-epoch Hits (after each eval_every-th epoch) and the loss."""
    import bench
    import llp_engine
    import models
    dev = torch.device("cuda", 0)
    a = bench.collab_args()
    a.hidden_channels = hidden
    a.link_batch_size = link_batch
    N, F, H, L = data.N, data.F, a.hidden_channels, a.num_layers
    E = data.train_pairs.shape[0]
    P = link_batch
    B = int(N / (E / P))                        # src/main.py:335
    torch.manual_seed(seed)
    model = models.MLP(L, F, H, H, a.dropout).to(dev)
    pred = models.LinkPredictor("mlp", H, H, 1, L, a.dropout).to(dev)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, a.dropout).to(dev)
    for p in tpred.parameters():
        p.requires_grad = False
    g = torch.Generator().manual_seed(seed + 1)
    t_h = torch.randn(N, 256, generator=g) * 0.3
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    eng = llp_engine.DistillEngine(model, pred, tpred, data.x.to(dev), t_h.to(dev), data.edge_index[0].numpy(),
                                   data.edge_index[1].numpy(), N, a, opt, dtype=dtype, seed=1234 + seed)
    pairs = data.train_pairs.to(torch.int32).to(dev).contiguous()
    hist = []
    t0 = time.perf_counter()
    for ep in range(epochs):
        pg = torch.Generator().manual_seed(10_000 * seed + ep)
        link_perm = torch.randperm(E, generator=pg).to(torch.int32).to(dev)
        node_perm = torch.randperm(N, generator=pg).to(torch.int32).to(dev)
        eng.begin_epoch()
        steps = min(E // P, N // B)
        for i in range(steps):
            eng.step_minibatch(node_perm[i * B:(i + 1) * B], link_perm[i * P:(i + 1) * P], pairs)
        loss = eng.end_epoch(steps * P)
        if (ep + 1) % eval_every == 0 or ep + 1 == epochs:
            hist.append({"epoch": ep + 1, "loss": loss, "hits": hits(model, pred, data, dev)})
    torch.cuda.synchronize()
    return {"dtype": dtype, "seconds": time.perf_counter() - t0, "B": B, "P": P, "history": hist}


def compare(scale=0.1, link_batch=8192, epochs=8, seed=0, hidden=1024, eval_every=1, communities=None):
    import llp_data
    data = llp_data.synthetic_collab(seed=0, scale=scale, with_eval=True, n_comm=communities)
    runs = {dt: train(dt, data, epochs, link_batch, seed=seed, hidden=hidden, eval_every=eval_every)
            for dt in ("fp32", "bf16")}
    last = {dt: runs[dt]["history"][-1]["hits"] for dt in runs}
    diff = {f"Hits@{k}": {s: last["bf16"][f"Hits@{k}"][s] - last["fp32"][f"Hits@{k}"][s] for s in ("valid", "test")}
            for k in KS}
    return {"scale": scale, "N": data.N, "test_positives": int(data.split_edge["test"]["edge"].shape[0]),
            "negatives": int(data.split_edge["test"]["edge_neg"].shape[0]), "link_batch": link_batch,
            "epochs": epochs, "runs": runs, "final": last, "bf16_minus_fp32": diff}


def _run_value(hist, k, split, rule, last):
    """One run's Hits@K (percentage points): rule "best_valid" -- the reference Logger's
    ``Highest Valid`` and ``Final Test`` (the checkpoint of the highest valid Hits@K, its valid or
    test value; src/logger.py); "last" -- the mean of the last ``last`` checkpoints."""
    if rule == "best_valid":
        i = int(np.argmax([h["hits"][k]["valid"] for h in hist]))
        return 100 * float(hist[i]["hits"][k][split])
    return 100 * float(np.mean([h["hits"][k][split] for h in hist[-last:]]))


def paired(runs, k="Hits@20", last=3, rule="best_valid"):
    """Paired bf16 - fp32 difference of Hits@K (percentage points) per seed (each run's value by
    _run_value's rule); returns per split the per-seed differences, their mean, the standard
    error of the mean, |mean| + 2 SE, and the fp32 runs' own seed-to-seed SD."""
    out = {}
    for split in ("valid", "test"):
        d, f = [], []
        for r in runs:
            v = {dt: _run_value(r["runs"][dt]["history"], k, split, rule, last) for dt in ("fp32", "bf16")}
            d.append(v["bf16"] - v["fp32"])
            f.append(v["fp32"])
        d = np.asarray(d)
        se = float(d.std(ddof=1) / np.sqrt(d.size)) if d.size > 1 else float("nan")
        out[split] = {"diff_pp": d.tolist(), "mean_pp": float(d.mean()), "se_pp": se,
                      "bound_pp": abs(float(d.mean())) + 2 * se, "fp32_mean_pp": float(np.mean(f)),
                      "fp32_seed_sd_pp": float(np.std(f, ddof=1)) if len(f) > 1 else float("nan"), "seeds": len(runs)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--link-batch", type=int, default=8192)
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--seeds", type=int, default=1)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--eval-every", type=int, default=1)
    ap.add_argument("--communities", type=int, default=None)
    ap.add_argument("--last", type=int, default=3, help="checkpoints averaged per run in the paired summary")
    opt = ap.parse_args()
    runs = []
    for s in range(opt.seeds):
        r = compare(opt.scale, opt.link_batch, opt.epochs, seed=s, hidden=opt.hidden, eval_every=opt.eval_every,
                    communities=opt.communities)
        runs.append(r)
        print(json.dumps(r), flush=True)
    summary = {rule: {k: paired(runs, k, opt.last, rule) for k in ("Hits@20", "Hits@50")}
               for rule in ("best_valid", "last")}
    print(json.dumps({"paired_bf16_minus_fp32": summary, "scale": opt.scale, "epochs": opt.epochs,
                      "eval_every": opt.eval_every, "last_checkpoints": opt.last}), flush=True)


if __name__ == "__main__":
    main()
