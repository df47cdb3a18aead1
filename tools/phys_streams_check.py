import sys, os, tempfile, torch
sys.path[:0] = ['/root/repo', '/root/repo/linkless-link-prediction_amd', '/root/repo/tools']
import llp_split, physics_bench, models, llp_engine
DEV = "cuda"
split = llp_split.production_split("coauthor-physics", os.path.join(tempfile.gettempdir(), "llp_physics"), synthetic=True)
td, a = split[0], physics_bench.physics_args()
N, F_ = td.x.size(0), td.x.size(1)
E = td.edge_index.size(1); P = a.link_batch_size; B = int(N / (E / P)); C = 20; H, L = 256, 2
g = torch.Generator().manual_seed(7)
anchors = torch.randperm(N, generator=g)[:B]
samples = torch.cat([anchors.view(B, 1), torch.randint(0, N, (B, C), generator=g)], 1)
link = torch.randperm(E, generator=g)[:P]
neg = torch.randint(0, N, (2, P), generator=g)
t_h = torch.randn(N, 256, generator=torch.Generator().manual_seed(2))
res = {}
for name, sparse, overlap in (("sparse_2s", True, True), ("sparse_1s", True, False), ("dense_2s", False, True), ("dense_1s", False, False)):
    torch.manual_seed(1)
    model = models.MLP(L, F_, H, H, 0.0).to(DEV); pred = models.LinkPredictor("mlp", H, H, 1, L, 0.0).to(DEV)
    tpred = models.LinkPredictor("mlp", 256, 256, 1, 2, 0.0).to(DEV)
    with torch.no_grad():
        for m, gain in ((model, 6.0), (pred, 6.0), (tpred, 3.0)):
            for p in m.parameters():
                if p.dim() == 2: p.mul_(gain)
    for p in tpred.parameters(): p.requires_grad = False
    opt = torch.optim.Adam(list(model.parameters()) + list(pred.parameters()), lr=a.lr)
    row, col = td.edge_index
    eng = llp_engine.DistillEngine(model, pred, tpred, td.x.to(DEV), t_h.to(DEV), row.numpy(), col.numpy(), N, a, opt, dtype="fp32", seed=11, sparse_input=sparse)
    eng.overlap_streams = overlap
    pairs = td.edge_index.t().to(torch.int32).to(DEV).contiguous()
    eng.step_fullbatch(anchors.to(torch.int32).to(DEV), link.to(torch.int32).to(DEV), pairs, samples=samples.to(torch.int32).to(DEV), neg=neg.to(torch.int32).to(DEV))
    torch.cuda.synchronize()
    res[name] = [p.grad.detach().double().cpu().clone() for p in list(model.parameters()) + list(pred.parameters())]
    res[name + "_h"] = eng._bufs.get("H0")[: N * H].view(N, H).double().cpu().clone() if "H0" in eng._bufs else None
    print(name, "done", flush=True)
for a_, b_ in (("sparse_2s", "sparse_1s"), ("dense_2s", "dense_1s"), ("sparse_1s", "dense_1s")):
    print(a_, "vs", b_, ["%.2e" % ((x - y).abs().max().item() / max(y.abs().max().item(), 1e-30)) for x, y in zip(res[a_], res[b_])])
    if res[a_ + "_h"] is not None and res[b_ + "_h"] is not None:
        print("   H0 max abs diff", (res[a_ + "_h"] - res[b_ + "_h"]).abs().max().item())
