"""Host (CPU) cost of one engine step: a tiny batch makes GPU time negligible,
so wall time per step ~= Python + launch overhead.  Also times the same step
replayed from a captured hipGraph (DistillEngine.capture_minibatch)."""
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))

import torch  # noqa: E402

import llp_engine  # noqa: E402
import models  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, F_, H, L = 5000, 128, 256, 3
    args = types.SimpleNamespace(rw_step=3, hops=3, ns_rate=3, ps_method="nb", dropout=0.0, margin=0.01, LLP_D=1.0,
                                 LLP_R=0.0, True_label=1.0, predictor="mlp", lr=0.001)
    g = torch.Generator().manual_seed(0)
    u = torch.randint(0, N, (30000,), generator=g)
    v = torch.randint(0, N, (30000,), generator=g)
    keep = u != v
    pairs = torch.stack([u[keep], v[keep]], 1)
    ei = torch.stack([pairs, pairs.flip(1)], 1).reshape(-1, 2).t()
    model = models.MLP(L, F_, H, H, 0.0).to(dev)
    pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(dev)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(dev)
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=0.001)
    eng = llp_engine.DistillEngine(model, pred, tpred, torch.randn(N, F_, device=dev),
                                   torch.randn(N, 256, device=dev), ei[0].numpy(), ei[1].numpy(), N, args, opt,
                                   dtype="bf16", seed=1)
    anchors = torch.randperm(N)[:64].to(torch.int32).to(dev)
    links = torch.randperm(pairs.size(0))[:512].to(torch.int32).to(dev)
    pr = pairs.to(torch.int32).to(dev)
    for _ in range(5):
        eng.step_minibatch(anchors, links, pr)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        eng.step_minibatch(anchors, links, pr)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager: host {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")
    if hasattr(eng, "capture_minibatch"):
        graph = eng.capture_minibatch(anchors, links, pr)
        for _ in range(5):
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            graph.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"graph: host {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")


if __name__ == "__main__":
    main()
