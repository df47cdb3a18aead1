"""Generate golden vectors by executing the REFERENCE's own code on CPU.

Run in the build container only (needs /root/reference, never on the GPU box):

    python tests/golden/gen_golden.py

What runs: the reference's own ``src/models.py`` (``MLP``, ``LinkPredictor``)
and the functions ``kl_loss``, ``neighbor_samplers``, ``train_minibatch``,
``train`` extracted (with ``ast``) from ``src/main.py``.  Their source text is
read from /root/reference at generation time and compiled here; nothing of it
is copied into the repo (the checked-in ``__pycache__`` .pyc is never loaded).

What is injected (the reference's third-party imports are not installed):
  * ``torch_geometric.nn`` names imported at models.py:3 -> inert placeholders
    (the distillation path never constructs them);
  * ``random_walk`` (torch_cluster) -> oracle.llp_oracle.random_walk on the
    reference's (row, col) with coalesced=False semantics;
  * ``negative_sampling`` (PyG) -> oracle.llp_oracle.negative_sampling_dense;
  * the string constant "cuda" (main.py:50,191) -> "cpu" (SURVEY Q7).
Every random tensor the reference draws (DataLoader permutations, randint,
walks, negatives) is recorded so a test can replay it into the HIP engine.

Output: ``tests/golden/*.npz`` (data only: inputs and expected outputs).
"""
from __future__ import annotations

import argparse
import ast
import itertools
import math
import os
import random
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import llp_oracle as O  # noqa: E402

REF = "/root/reference/src"


def _compile_file(path):
    with open(path) as f:
        return f.read()


def load_reference_models():
    """Exec src/models.py with an inert torch_geometric.nn (models.py:3)."""
    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    for n in ("GCNConv", "SAGEConv", "GATConv", "APPNP"):
        setattr(pyg_nn, n, type(n, (), {}))
    pyg.nn = pyg_nn
    saved = {k: sys.modules.get(k) for k in ("torch_geometric", "torch_geometric.nn")}
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.nn"] = pyg_nn
    try:
        mod = types.ModuleType("ref_models")
        code = compile(_compile_file(os.path.join(REF, "models.py")), os.path.join(REF, "models.py"), "exec")
        exec(code, mod.__dict__)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


class _CudaToCpu(ast.NodeTransformer):
    def visit_Constant(self, node):
        if node.value == "cuda":
            return ast.copy_location(ast.Constant("cpu"), node)
        return node


class Recorder:
    def __init__(self):
        self.log = []

    def add(self, kind, value):
        self.log.append((kind, value.detach().clone() if torch.is_tensor(value) else value))


def load_reference_main(rec: Recorder, rw_seed: int, neg_seed: int):
    """Extract kl_loss/cosine_loss/neighbor_samplers/train_minibatch/train from
    src/main.py (skipping the module-level main() call at main.py:515)."""
    src = _compile_file(os.path.join(REF, "main.py"))
    tree = ast.parse(src)
    keep = {"cosine_loss", "kl_loss", "neighbor_samplers", "train_minibatch", "train"}
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in keep]
    mod_ast = _CudaToCpu().visit(ast.Module(body=body, type_ignores=[]))
    ast.fix_missing_locations(mod_ast)

    rw_counter = itertools.count()

    def random_walk(row, col, start, walk_length, coalesced=True, p=1, q=1):
        num_nodes = int(max(int(row.max()), int(col.max()), int(start.max()))) + 1
        rowptr, colv = O.build_rowptr(row.numpy(), col.numpy(), num_nodes, coalesced=coalesced)
        out = torch.from_numpy(O.random_walk(rowptr, colv, start.numpy(), walk_length, rw_seed, next(rw_counter)))
        rec.add("random_walk", out)
        return out

    neg_rng = random.Random(neg_seed)

    def negative_sampling(edge_index, num_nodes=None, num_neg_samples=None, method="sparse"):
        assert method == "dense"
        out = O.negative_sampling_dense(edge_index, num_nodes, num_neg_samples, rng=neg_rng)
        rec.add("negative_sampling", out)
        return out

    class TorchProxy(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

    tproxy = TorchProxy("torch")

    def randint(*a, **k):
        out = torch.randint(*a, **k)
        rec.add("randint", out)
        return out

    tproxy.randint = randint

    class RecDataLoader:
        def __init__(self, *a, **k):
            self.dl = torch.utils.data.DataLoader(*a, **k)

        def __iter__(self):
            for b in self.dl:
                rec.add("perm", b)
                yield b

    class NNProxy(types.ModuleType):
        def __getattr__(self, name):
            return getattr(nn, name)

    nproxy = NNProxy("nn")

    class RecMarginRankingLoss(nn.MarginRankingLoss):
        def forward(self, a, b, y):
            out = super().forward(a, b, y)
            rec.add("llp_r", out)
            return out

    class RecBCELoss(nn.BCELoss):
        def forward(self, a, b):
            out = super().forward(a, b)
            rec.add("bce", out)
            return out

    nproxy.MarginRankingLoss = RecMarginRankingLoss
    nproxy.BCELoss = RecBCELoss

    ns = dict(torch=tproxy, nn=nproxy, F=F, np=np, itertools=itertools, DataLoader=RecDataLoader,
              random_walk=random_walk, negative_sampling=negative_sampling,
              cosine_similarity=F.cosine_similarity)
    exec(compile(mod_ast, os.path.join(REF, "main.py"), "exec"), ns)
    raw_kl = ns["kl_loss"]

    def kl_loss(s, t, T):
        out = raw_kl(s, t, T)
        rec.add("llp_d", out)
        return out

    ns["kl_loss"] = kl_loss
    return ns


class RecAdam(torch.optim.Adam):
    def __init__(self, params, rec, **kw):
        super().__init__(params, **kw)
        self.rec = rec

    def step(self, closure=None):
        grads = [p.grad.detach().clone() for g in self.param_groups for p in g["params"]]
        self.rec.add("grads", grads)
        return super().step(closure)


def synth_graph(N, n_undirected, seed, interleave=True):
    """Random simple-ish graph with a few duplicate pairs, written
    OGB-style (u,v),(v,u) interleaved (Q1) when ``interleave``."""
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, N, (n_undirected,), generator=g)
    v = torch.randint(0, N, (n_undirected,), generator=g)
    keep = u != v
    u, v = u[keep], v[keep]
    # duplicate ~5% of the pairs (multi-edges)
    nd = max(1, u.numel() // 20)
    u = torch.cat([u, u[:nd]]); v = torch.cat([v, v[:nd]])
    pairs = torch.stack([u, v], 1)                       # (E_und, 2)
    if interleave:
        ei = torch.stack([pairs, pairs.flip(1)], 1).reshape(-1, 2).t().contiguous()
    else:
        ei = torch.cat([pairs, pairs.flip(1)], 0).t().contiguous()
    return pairs, ei


def flat_log(rec: Recorder):
    return list(rec.log)


def _norm_records(out, model, x_eval, norm_type):
    """norm_type cases: parameter / buffer names of the student, its eval-mode output."""
    out["norm_type"] = np.array(norm_type)
    out["stu_param_keys"] = np.array([n for n, _ in model.named_parameters()])
    out["stu_buffer_keys"] = np.array([n for n, _ in model.named_buffers()])
    model.eval()
    with torch.no_grad():
        out["h_eval"] = model(x_eval).numpy()
    model.train()


def run_minibatch_case(name, ref_models, N, F_, H, L, E_und, lbs, args_over, seed, nepochs=1, norm_type="none"):
    rec = Recorder()
    ns = load_reference_main(rec, rw_seed=seed + 11, neg_seed=seed + 12)
    torch.manual_seed(seed)
    pairs, ei = synth_graph(N, E_und, seed)
    x = torch.randn(N, F_) * 0.5
    t_h = torch.randn(N, 256) * 0.3
    data = types.SimpleNamespace(x=x, adj_t=ei, edge_index=ei)
    split_edge = {"train": {"edge": pairs}}
    args = argparse.Namespace(
        transductive="transductive", node_batch_size=None, link_batch_size=lbs, datasets="collab",
        rw_step=3, hops=3, ns_rate=3, ps_method="nb", hidden_channels=H, num_layers=L, dropout=0.0,
        margin=0.05, LLP_D=1.0, LLP_R=1.0, True_label=0.1, KD_RM=0.0, KD_LM=0.0, predictor="mlp", lr=0.01)
    for k, v in args_over.items():
        setattr(args, k, v)
    args.node_batch_size = int(N / (pairs.size(0) / args.link_batch_size))          # main.py:335
    model = ref_models.MLP(args.num_layers, F_, H, H, args.dropout, norm_type)
    _perturb_norms(model)
    predictor = ref_models.LinkPredictor(args.predictor, H, H, 1, args.num_layers, args.dropout)
    tpred = ref_models.LinkPredictor(args.predictor, 256, 256, 1, 2, args.dropout)
    for p in tpred.parameters():
        p.requires_grad = False
    init_stu = {k: v.clone() for k, v in model.state_dict().items()}
    init_pred = {k: v.clone() for k, v in predictor.state_dict().items()}
    opt = RecAdam(list(model.parameters()) + list(predictor.parameters()), rec, lr=args.lr)
    losses = []
    for ep in range(nepochs):
        losses.append(ns["train_minibatch"](model, predictor, t_h, tpred, data, split_edge, opt, args, "cpu"))
    out = dict(N=N, F=F_, H=H, L=L, x=x.numpy(), t_h=t_h.numpy(), edge_index=ei.numpy(), train_pairs=pairs.numpy(),
               epoch_losses=np.array(losses, np.float64))
    out.update({f"args/{k}": np.array(v) for k, v in vars(args).items()})
    for k, v in init_stu.items():
        out[f"init/stu/{k}"] = v.numpy()
    for k, v in init_pred.items():
        out[f"init/pred/{k}"] = v.numpy()
    for k, v in tpred.state_dict().items():
        out[f"tpred/{k}"] = v.numpy()
    for k, v in model.state_dict().items():
        out[f"final/stu/{k}"] = v.numpy()
    for k, v in predictor.state_dict().items():
        out[f"final/pred/{k}"] = v.numpy()
    _dump_log(out, rec, kind_order="minibatch", args=args)
    if norm_type != "none":
        _norm_records(out, model, x, norm_type)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "steps:", out["nsteps"], "epoch losses:", losses)


def _dump_log(out, rec, kind_order, args):
    """Split the recorder log into per-step records."""
    log = rec.log
    step = -1
    perms = []
    cur = None
    steps = []
    for kind, v in log:
        if kind == "perm":
            perms.append(v)
            continue
        if kind in ("randint", "negative_sampling", "random_walk") and (cur is None or "grads" in cur):
            cur = {"walks": [], "randint": []}
            steps.append(cur)
        if kind == "random_walk":
            cur["walks"].append(v)
        elif kind == "randint":
            cur["randint"].append(v)
        elif kind == "negative_sampling":
            cur["neg_edge"] = v
        elif kind in ("llp_d", "llp_r", "bce"):
            cur[kind] = v
        elif kind == "grads":
            cur["grads"] = v
    out["nsteps"] = np.array(len(steps))
    out["perms_raw_count"] = np.array(len(perms))
    for i, p in enumerate(perms):
        out[f"perm/{i}"] = p.numpy()
    for s, st in enumerate(steps):
        for i, w in enumerate(st["walks"]):
            out[f"step{s}/walk{i}"] = w.numpy()
        for i, r in enumerate(st["randint"]):
            out[f"step{s}/randint{i}"] = r.numpy()
        if "neg_edge" in st:
            out[f"step{s}/neg_edge"] = st["neg_edge"].numpy()
        for k in ("llp_d", "llp_r", "bce"):
            if k in st:
                out[f"step{s}/{k}"] = st[k].numpy()
        for i, g in enumerate(st["grads"]):
            out[f"step{s}/grad{i}"] = g.numpy()


def _perturb_norms(model):
    """Non-trivial affine parameters (torch initialises them to 1 / 0) so that the norms'
    gamma and beta enter every gradient; the generator leaves torch's global RNG alone."""
    g = torch.Generator().manual_seed(77)
    with torch.no_grad():
        for m in getattr(model, "norms", []):
            m.weight.copy_(1.0 + 0.2 * torch.randn(m.weight.shape, generator=g))
            m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))


def run_fullbatch_case(name, ref_models, N, F_, E_und, lbs, args_over, seed, transductive="transductive",
                       norm_type="none"):
    rec = Recorder()
    ns = load_reference_main(rec, rw_seed=seed + 21, neg_seed=seed + 22)
    torch.manual_seed(seed)
    pairs, ei = synth_graph(N, E_und, seed, interleave=False)
    H = 256                                                 # main.py:185 needs H == t_h width
    x = (torch.rand(N, F_) < 0.1).float()
    t_h = torch.randn(N, 256) * 0.3
    args = argparse.Namespace(
        transductive=transductive, node_batch_size=None, link_batch_size=lbs, datasets="cora",
        rw_step=3, hops=2, ns_rate=1, ps_method="nb", hidden_channels=H, num_layers=2, dropout=0.0,
        margin=0.1, LLP_D=0.5, LLP_R=1.0, True_label=0.1, KD_RM=0.3, KD_LM=0.2, predictor="mlp", lr=0.01)
    for k, v in args_over.items():
        setattr(args, k, v)
    if transductive == "transductive":
        data = types.SimpleNamespace(x=x, adj_t=ei)
        split_edge = {"train": {"edge": pairs}}
        args.node_batch_size = int(N / (pairs.size(0) / args.link_batch_size))
    else:
        data = types.SimpleNamespace(x=x, edge_index=ei)
        split_edge = None
        args.node_batch_size = int(N / (ei.size(1) / args.link_batch_size))       # main.py:348
    model = ref_models.MLP(args.num_layers, F_, H, H, args.dropout, norm_type)
    _perturb_norms(model)
    predictor = ref_models.LinkPredictor(args.predictor, H, H, 1, args.num_layers, args.dropout)
    tpred = ref_models.LinkPredictor(args.predictor, 256, 256, 1, 2, args.dropout)
    for p in tpred.parameters():
        p.requires_grad = False
    init_stu = {k: v.clone() for k, v in model.state_dict().items()}
    init_pred = {k: v.clone() for k, v in predictor.state_dict().items()}
    opt = RecAdam(list(model.parameters()) + list(predictor.parameters()), rec, lr=args.lr)
    loss = ns["train"](model, predictor, t_h, tpred, data, split_edge, opt, args, "cpu")
    out = dict(N=N, F=F_, H=H, L=args.num_layers, x=x.numpy(), t_h=t_h.numpy(), edge_index=ei.numpy(),
               train_pairs=pairs.numpy(), epoch_losses=np.array([loss], np.float64))
    out.update({f"args/{k}": np.array(v) for k, v in vars(args).items()})
    for k, v in init_stu.items():
        out[f"init/stu/{k}"] = v.numpy()
    for k, v in init_pred.items():
        out[f"init/pred/{k}"] = v.numpy()
    for k, v in tpred.state_dict().items():
        out[f"tpred/{k}"] = v.numpy()
    for k, v in model.state_dict().items():
        out[f"final/stu/{k}"] = v.numpy()
    for k, v in predictor.state_dict().items():
        out[f"final/pred/{k}"] = v.numpy()
    _dump_log(out, rec, kind_order="fullbatch", args=args)
    if norm_type != "none":
        _norm_records(out, model, x, norm_type)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "steps:", out["nsteps"], "epoch loss:", loss)


def run_kl_rank_case(name, seed):
    """kl_loss (main.py:27-31) on fixed inputs, incl. T != 1."""
    rec = Recorder()
    ns = load_reference_main(rec, 0, 0)
    g = torch.Generator().manual_seed(seed)
    out = {}
    for i, (B, C, T) in enumerate([(5, 12, 1.0), (7, 36, 1.0), (3, 8, 2.0)]):
        s = torch.rand(B, C, generator=g)
        t = torch.rand(B, C, generator=g)
        out[f"case{i}/s"] = s.numpy(); out[f"case{i}/t"] = t.numpy(); out[f"case{i}/T"] = np.array(T)
        out[f"case{i}/kl"] = ns["kl_loss"](s, t, T).numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def run_model_case(name, ref_models, seed):
    """Reference MLP / LinkPredictor forward+backward on fixed inputs."""
    torch.manual_seed(seed)
    out = {}
    mlp = ref_models.MLP(3, 24, 40, 40, 0.0)
    x = torch.randn(33, 24, requires_grad=True)
    y = mlp(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    out.update({f"mlp/{k}": v.detach().numpy() for k, v in mlp.state_dict().items()})
    out.update({"mlp/x": x.detach().numpy(), "mlp/y": y.detach().numpy(), "mlp/gy": gy.numpy(),
                "mlp/gx": x.grad.numpy()})
    for k, p in mlp.named_parameters():
        out[f"mlp/grad/{k}"] = p.grad.numpy()
    for kind in ("mlp", "inner"):
        lp = ref_models.LinkPredictor(kind, 40, 40, 1, 3, 0.0)
        xi = torch.randn(29, 40, requires_grad=True)
        xj = torch.randn(29, 40, requires_grad=True)
        o = lp(xi, xj)
        go = torch.randn_like(o)
        o.backward(go)
        out.update({f"lp_{kind}/{k}": v.detach().numpy() for k, v in lp.state_dict().items()})
        out.update({f"lp_{kind}/xi": xi.detach().numpy(), f"lp_{kind}/xj": xj.detach().numpy(),
                    f"lp_{kind}/out": o.detach().numpy(), f"lp_{kind}/gout": go.numpy(),
                    f"lp_{kind}/gxi": xi.grad.numpy(), f"lp_{kind}/gxj": xj.grad.numpy()})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def run_norm_model_case(name, ref_models, seed):
    """Reference MLP with norm_type 'layer' / 'batch' (src/models.py:6-54): train-mode
    forward + backward (BatchNorm on batch statistics, running statistics updated),
    then an eval-mode forward on the running statistics."""
    torch.manual_seed(seed)
    out = {}
    for norm in ("layer", "batch"):
        mlp = ref_models.MLP(3, 24, 40, 40, 0.0, norm)
        _perturb_norms(mlp)
        x = torch.randn(67, 24, requires_grad=True)
        y = mlp(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        mlp.eval()
        with torch.no_grad():
            x2 = torch.randn(31, 24)
            y2 = mlp(x2)
        pre = f"mlp_{norm}"
        out.update({f"{pre}/{k}": v.detach().numpy() for k, v in mlp.state_dict().items()})
        out.update({f"{pre}/x": x.detach().numpy(), f"{pre}/y": y.detach().numpy(), f"{pre}/gy": gy.numpy(),
                    f"{pre}/gx": x.grad.numpy(), f"{pre}/x_eval": x2.numpy(), f"{pre}/y_eval": y2.numpy()})
        out[f"{pre}/param_keys"] = np.array([n for n, _ in mlp.named_parameters()])
        out[f"{pre}/state_keys"] = np.array(list(mlp.state_dict().keys()))
        for k, p in mlp.named_parameters():
            out[f"{pre}/grad/{k}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


# ----------------------------------------------------------------------------
# Teacher: src/train_teacher_gnn.py:21-73 (train) with the reference's own
# SAGE (src/models.py:82-119) and SAGEConv_updated (src/sageconv_updated.py).
# PyG pieces they build on are restated: SAGEConv -> oracle.sage_conv,
# MessagePassing.propagate(aggr='mean') -> oracle.sage_mean_aggregate,
# torch_geometric Linear -> nn.Linear (weights are overwritten anyway).
# ----------------------------------------------------------------------------
class _RestatedSAGEConv(nn.Module):
    def __init__(self, in_channels, out_channels, normalize=False, root_weight=True, bias=True, **kw):
        super().__init__()
        self.lin_l = nn.Linear(in_channels, out_channels, bias=bias)
        self.lin_r = nn.Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self):
        self.lin_l.reset_parameters()
        self.lin_r.reset_parameters()

    def forward(self, x, edge_index):
        return O.sage_conv(x, edge_index, self.lin_l.weight, self.lin_l.bias, self.lin_r.weight)


class _RestatedGCNConv(nn.Module):
    """PyG 2.2.0 GCNConv(cached=True) parameters: ``bias`` then ``lin.weight``."""

    def __init__(self, in_channels, out_channels, cached=False, bias=True, **kw):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(out_channels))
        self.lin = nn.Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.lin.weight)
        nn.init.zeros_(self.bias)

    def forward(self, x, edge_index):
        return O.gcn_conv(x, edge_index, self.lin.weight, self.bias)


class _MessagePassing(nn.Module):
    def __init__(self, aggr="mean", **kw):
        super().__init__()
        assert aggr == "mean"
        self.aggr = aggr

    def propagate(self, edge_index, x, size=None):
        xs = x[0]
        return O.sage_mean_aggregate(self.message(xs[edge_index[0]]), torch.arange(edge_index.size(1)),
                                     edge_index[1], xs.size(0))


def load_reference_sage():
    """Exec src/models.py and src/sageconv_updated.py over restated PyG stubs."""
    stubs = {}
    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    for n in ("GATConv", "APPNP"):
        setattr(pyg_nn, n, type(n, (), {}))
    pyg_nn.SAGEConv = _RestatedSAGEConv
    pyg_nn.GCNConv = _RestatedGCNConv
    conv = types.ModuleType("torch_geometric.nn.conv")
    conv.MessagePassing = _MessagePassing
    dense = types.ModuleType("torch_geometric.nn.dense")
    lin = types.ModuleType("torch_geometric.nn.dense.linear")
    lin.Linear = nn.Linear
    typ = types.ModuleType("torch_geometric.typing")
    typ.OptPairTensor = typ.Adj = typ.Size = object
    tsp = types.ModuleType("torch_sparse")
    tsp.SparseTensor = type("SparseTensor", (), {})
    tsp.matmul = None
    pyg.nn = pyg_nn
    for k, v in {"torch_geometric": pyg, "torch_geometric.nn": pyg_nn, "torch_geometric.nn.conv": conv,
                 "torch_geometric.nn.dense": dense, "torch_geometric.nn.dense.linear": lin,
                 "torch_geometric.typing": typ, "torch_sparse": tsp}.items():
        stubs[k] = sys.modules.get(k)
        sys.modules[k] = v
    try:
        mods = types.ModuleType("ref_models_sage")
        exec(compile(_compile_file(os.path.join(REF, "models.py")), os.path.join(REF, "models.py"), "exec"),
             mods.__dict__)
        upd = types.ModuleType("ref_sageconv_updated")
        p = os.path.join(REF, "sageconv_updated.py")
        exec(compile(_compile_file(p), p, "exec"), upd.__dict__)
    finally:
        for k, v in stubs.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mods, upd.SAGEConv_updated


def load_reference_teacher_train(rec: Recorder, neg_seed: int):
    src = _compile_file(os.path.join(REF, "train_teacher_gnn.py"))
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "train"]
    mod_ast = ast.Module(body=body, type_ignores=[])
    ast.fix_missing_locations(mod_ast)
    neg_rng = random.Random(neg_seed)

    def negative_sampling(edge_index, num_nodes=None, num_neg_samples=None, method="sparse"):
        assert method == "dense"
        out = O.negative_sampling_dense(edge_index, num_nodes, num_neg_samples, rng=neg_rng)
        rec.add("negative_sampling", out)
        return out

    class RecDataLoader:
        def __init__(self, *a, **k):
            self.dl = torch.utils.data.DataLoader(*a, **k)

        def __iter__(self):
            for b in self.dl:
                rec.add("perm", b)
                yield b

    class NNProxy(types.ModuleType):
        def __getattr__(self, name):
            return getattr(nn, name)

    nproxy = NNProxy("nn")

    class RecBCELoss(nn.BCELoss):
        def forward(self, a, b):
            out = super().forward(a, b)
            rec.add("bce", out)
            return out

    nproxy.BCELoss = RecBCELoss

    class TorchProxy(types.ModuleType):
        def __getattr__(self, name):
            return getattr(torch, name)

    tproxy = TorchProxy("torch")

    def randint(*a, **k):
        out = torch.randint(*a, **k)
        rec.add("randint", out)
        return out

    tproxy.randint = randint
    ns = dict(torch=tproxy, nn=nproxy, F=F, DataLoader=RecDataLoader, negative_sampling=negative_sampling)
    exec(compile(mod_ast, os.path.join(REF, "train_teacher_gnn.py"), "exec"), ns)
    return ns["train"]


def run_teacher_case(name, N, F_, H, L, E_und, bs, updated, transductive, seed, dataset="cora", epochs=2,
                     encoder="sage", self_loops=0, norm_type="none"):
    rec = Recorder()
    ref_mods, ref_updated = load_reference_sage()
    train = load_reference_teacher_train(rec, neg_seed=seed + 31)
    torch.manual_seed(seed)
    pairs, ei = synth_graph(N, E_und, seed, interleave=False)
    if self_loops:       # GCN's gcn_norm drops input self-loops before adding its own
        loops = torch.arange(0, N, max(1, N // self_loops))[:self_loops]
        pairs = torch.cat([pairs, torch.stack([loops, loops], 1)], 0)
        ei = torch.cat([pairs, pairs.flip(1)], 0).t().contiguous()
    x = torch.randn(N, F_) * 0.5
    if encoder == "gcn":
        model = ref_mods.GCN(F_, H, H, L, 0.0)
        for c in model.convs:     # non-zero biases so the bias path is exercised
            nn.init.uniform_(c.bias, -0.1, 0.1)
    else:
        conv_layer = ref_updated if updated else ref_mods.SAGE.__init__.__globals__["SAGEConv"]
        model = ref_mods.SAGE(dataset, F_, H, H, L, 0.0, conv_layer, norm_type)
        _perturb_norms(model)
    predictor = ref_mods.LinkPredictor("mlp", H, H, 1, 2, 0.0)
    init_enc = {k: v.clone() for k, v in model.state_dict().items()}
    init_pred = {k: v.clone() for k, v in predictor.state_dict().items()}
    opt = RecAdam(list(model.parameters()) + list(predictor.parameters()), rec, lr=0.005)
    if transductive == "transductive":
        # non-collab: adj_t = split_edge['train']['edge'].t() (one direction, src/train_teacher_gnn.py:317-318)
        data = types.SimpleNamespace(x=x, adj_t=pairs.t().contiguous())
        split_edge = {"train": {"edge": pairs}}
    else:
        data = types.SimpleNamespace(x=x, edge_index=ei)
        split_edge = None
    losses = [train(model, predictor, data, split_edge, opt, bs, encoder, dataset, transductive)
              for _ in range(epochs)]
    mp_edges = data.adj_t if transductive == "transductive" else ei
    out = dict(N=N, F=F_, H=H, L=L, x=x.numpy(), edge_index=mp_edges.numpy(), train_pairs=pairs.numpy(),
               epoch_losses=np.array(losses, np.float64), updated=np.array(int(updated)), batch_size=np.array(bs),
               transductive=np.array(transductive), dataset=np.array(dataset), encoder=np.array(encoder))
    for k, v in init_enc.items():
        out[f"init/enc/{k}"] = v.numpy()
    for k, v in init_pred.items():
        out[f"init/pred/{k}"] = v.numpy()
    for k, v in model.state_dict().items():
        out[f"final/enc/{k}"] = v.numpy()
    for k, v in predictor.state_dict().items():
        out[f"final/pred/{k}"] = v.numpy()
    out["enc_keys"] = np.array(list(init_enc.keys()))
    out["enc_param_keys"] = np.array([n for n, _ in model.named_parameters()])
    out["norm_type"] = np.array(norm_type)
    out["pred_keys"] = np.array(list(init_pred.keys()))
    _dump_log(out, rec, kind_order="teacher", args=None)
    # eval-mode embedding after training (src/train_teacher_gnn.py:87): the saved teacher features
    model.eval()
    with torch.no_grad():
        out["h_eval"] = model(x, mp_edges).numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "steps:", out["nsteps"], "epoch losses:", losses)


class _PygData:
    """torch_geometric.data.Data stand-in for the production-split stubs."""

    def __init__(self, x=None, edge_index=None, **kw):
        self.x, self.edge_index = x, edge_index
        self.__dict__.update(kw)

    @property
    def num_nodes(self):
        return self.x.size(0)

    def clone(self):
        return _PygData(**{k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.__dict__.items()})


def _pyg_sample(population, k):
    if population <= k:
        return torch.arange(population)
    return torch.tensor(random.sample(range(population), k))


def _pyg_negative_sampling(edge_index, num_nodes=None, num_neg_samples=None, method="sparse",
                           force_undirected=False):
    """PyG 2.2.0 torch_geometric.utils.negative_sampling, sparse method."""
    assert method == "sparse"
    n = num_nodes
    row, col = edge_index
    if force_undirected:
        m = row < col
        r, c = row[m], col[m]
        idx = r * n + c - torch.arange(1, n).cumsum(0)[r]
        population = n * (n + 1) // 2 - n
    else:
        m = row != col
        r, c = row[m], col[m].clone()
        c[r < c] -= 1
        idx = r * (n - 1) + c
        population = n * n - n
    if idx.numel() >= population:
        return edge_index.new_empty((2, 0))
    if num_neg_samples is None:
        num_neg_samples = edge_index.size(1)
    if force_undirected:
        num_neg_samples = num_neg_samples // 2
    sample_size = int(1.1 * num_neg_samples / (1.0 - idx.numel() / population))
    neg = None
    for _ in range(3):
        rnd = _pyg_sample(population, sample_size)
        bad = np.isin(rnd, idx)
        if neg is not None:
            bad |= np.isin(rnd, neg)
        rnd = rnd[~torch.from_numpy(bad).to(torch.bool)]
        neg = rnd if neg is None else torch.cat([neg, rnd])
        if neg.numel() >= num_neg_samples:
            neg = neg[:num_neg_samples]
            break
    if force_undirected:
        off = torch.arange(1, n).cumsum(0)
        end = torch.arange(n, n * n, n).sub_(off)
        r = torch.bucketize(neg, end, right=True)
        c = off[r].add_(neg) % n
        return torch.stack([torch.cat([r, c]), torch.cat([c, r])], 0)
    r = torch.div(neg, n - 1, rounding_mode="floor")
    c = neg % (n - 1)
    c[r <= c] += 1
    return torch.stack([r, c], 0)


class _PygRandomNodeSplit:
    def __init__(self, split="train_rest", num_splits=1, num_train_per_class=20, num_val=500, num_test=1000,
                 key="y"):
        assert split == "train_rest" and num_splits == 1
        self.num_val, self.num_test = num_val, num_test

    def __call__(self, data):
        out = data.clone()
        n = out.num_nodes
        masks = [torch.zeros(n, dtype=torch.bool) for _ in range(3)]
        nv = round(n * self.num_val) if isinstance(self.num_val, float) else self.num_val
        nt = round(n * self.num_test) if isinstance(self.num_test, float) else self.num_test
        perm = torch.randperm(n)
        masks[1][perm[:nv]] = True
        masks[2][perm[nv:nv + nt]] = True
        masks[0][perm[nv + nt:]] = True
        out.train_mask, out.val_mask, out.test_mask = masks
        return out


class _PygRandomLinkSplit:
    def __init__(self, num_val=0.1, num_test=0.2, is_undirected=False, key="edge_label", split_labels=False,
                 add_negative_train_samples=True, neg_sampling_ratio=1.0, disjoint_train_ratio=0.0):
        assert is_undirected and not split_labels and add_negative_train_samples and disjoint_train_ratio == 0
        self.num_val, self.num_test, self.ratio = num_val, num_test, neg_sampling_ratio

    def __call__(self, data):
        ei = data.edge_index
        perm = (ei[0] <= ei[1]).nonzero(as_tuple=False).view(-1)
        perm = perm[torch.randperm(perm.size(0), device=perm.device)]
        nv = int(self.num_val * perm.numel())
        nt = int(self.num_test * perm.numel())
        ntr = perm.numel() - nv - nt
        tr, va, te, trva = perm[:ntr], perm[ntr:ntr + nv], perm[ntr + nv:], perm[:ntr + nv]
        n_tr, n_va, n_te = int(ntr * self.ratio), int(nv * self.ratio), int(nt * self.ratio)
        neg = _pyg_negative_sampling(ei, data.num_nodes, num_neg_samples=n_tr + n_va + n_te, method="sparse")
        assert neg.size(1) == n_tr + n_va + n_te

        def make(mp, lab_idx, negs):
            e = ei[:, mp]
            out = _PygData(data.x, torch.cat([e, e.flip([0])], dim=-1))
            out.edge_label = torch.cat([torch.ones(lab_idx.numel()), torch.zeros(negs.size(1))], dim=0)
            out.edge_label_index = torch.cat([ei[:, lab_idx], negs], dim=-1)
            return out
        return (make(tr, tr, neg[:, n_va + n_te:]), make(tr, va, neg[:, :n_va]),
                make(trva, te, neg[:, n_va:n_va + n_te]))


def _pyg_subgraph(subset, edge_index, relabel_nodes=False):
    assert subset.dtype == torch.bool and relabel_nodes
    node_idx = torch.zeros(subset.numel(), dtype=torch.long)
    node_idx[subset] = torch.arange(int(subset.sum()))
    keep = subset[edge_index[0]] & subset[edge_index[1]]
    return node_idx[edge_index[:, keep]], None


def load_reference_production_split():
    """Exec src/generate_production_split.py over the PyG stubs above."""
    pyg = types.ModuleType("torch_geometric")
    pd = types.ModuleType("torch_geometric.data")
    pd.Data, pd.Dataset = _PygData, list
    pt = types.ModuleType("torch_geometric.transforms")
    pt.RandomLinkSplit, pt.RandomNodeSplit = _PygRandomLinkSplit, _PygRandomNodeSplit
    pu = types.ModuleType("torch_geometric.utils")
    pu.negative_sampling, pu.subgraph = _pyg_negative_sampling, _pyg_subgraph
    pu.add_self_loops = pu.train_test_split_edges = pu.to_networkx = None
    ogb = types.ModuleType("ogb")
    ogl = types.ModuleType("ogb.linkproppred")
    ogl.PygLinkPropPredDataset = None
    stubs = {"torch_geometric": pyg, "torch_geometric.data": pd, "torch_geometric.transforms": pt,
             "torch_geometric.utils": pu, "ogb": ogb, "ogb.linkproppred": ogl}
    saved = {k: sys.modules.get(k) for k in stubs}
    sys.modules.update(stubs)
    try:
        mod = types.ModuleType("ref_generate_production_split")
        p = os.path.join(REF, "generate_production_split.py")
        exec(compile(_compile_file(p), p, "exec"), mod.__dict__)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def run_production_split_case(name, N, F_, E_und, ratios, seed):
    """src/generate_production_split.py:32-95 on a coalesced synthetic graph."""
    import contextlib
    import io
    mod = load_reference_production_split()
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, N, (E_und,), generator=g)
    v = torch.randint(0, N, (E_und,), generator=g)
    keep = u != v
    und = torch.stack([u[keep], v[keep]])
    key = torch.unique(torch.cat([und, und.flip([0])], -1)[0] * N + torch.cat([und, und.flip([0])], -1)[1])
    ei = torch.stack([key // N, key % N])
    x = torch.randn(N, F_, generator=g)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        tr, va, inf, _, bundle, neg = mod.do_production_edge_split([_PygData(x, ei)], name, *ratios)
    out = dict(N=np.int64(N), x=x.numpy(), edge_index=ei.numpy(), ratios=np.array(ratios, np.float64),
               train_x=tr.x.numpy(), train_edge_index=tr.edge_index.numpy(),
               train_edge_label=tr.edge_label.numpy(), train_edge_label_index=tr.edge_label_index.numpy(),
               val_edge_index=va.edge_index.numpy(), val_edge_label=va.edge_label.numpy(),
               val_edge_label_index=va.edge_label_index.numpy(), inference_edge_index=inf.edge_index.numpy(),
               old_old=bundle[0].numpy(), old_new=bundle[1].numpy(), new_new=bundle[2].numpy(),
               test=bundle[3].numpy(), negative_samples=neg.numpy(),
               stdout=np.frombuffer(buf.getvalue().encode(), np.uint8))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)



def _pyg_coalesce_und(ei, n):
    e = torch.cat([ei, ei.flip([0])], 1)
    key = torch.unique(e[0] * n + e[1])
    return torch.stack([key // n, key % n])


def _pyg_train_test_split_edges(data, val_ratio=0.05, test_ratio=0.1):
    """PyG 2.2.0 torch_geometric.utils.train_test_split_edges (no edge_attr)."""
    n = data.num_nodes
    row, col = data.edge_index
    data.edge_index = None
    m = row < col
    row, col = row[m], col[m]
    n_v = int(math.floor(val_ratio * row.size(0)))
    n_t = int(math.floor(test_ratio * row.size(0)))
    perm = torch.randperm(row.size(0))
    row, col = row[perm], col[perm]
    data.val_pos_edge_index = torch.stack([row[:n_v], col[:n_v]], dim=0)
    data.test_pos_edge_index = torch.stack([row[n_v:n_v + n_t], col[n_v:n_v + n_t]], dim=0)
    data.train_pos_edge_index = _pyg_coalesce_und(torch.stack([row[n_v + n_t:], col[n_v + n_t:]], dim=0), n)
    neg_adj_mask = torch.ones(n, n, dtype=torch.uint8).triu(diagonal=1).to(torch.bool)
    neg_adj_mask[row, col] = 0
    neg_row, neg_col = neg_adj_mask.nonzero(as_tuple=False).t()
    perm = torch.randperm(neg_row.size(0))[:n_v + n_t]
    neg_row, neg_col = neg_row[perm], neg_col[perm]
    data.val_neg_edge_index = torch.stack([neg_row[:n_v], neg_col[:n_v]], dim=0)
    data.test_neg_edge_index = torch.stack([neg_row[n_v:n_v + n_t], neg_col[n_v:n_v + n_t]], dim=0)
    return data


def _pyg_add_self_loops(edge_index, edge_attr=None, num_nodes=None):
    n = num_nodes if num_nodes is not None else int(edge_index.max()) + 1
    loops = torch.arange(n).unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index, loops], dim=1), None


def load_reference_utils():
    """Exec src/utils.py (get_dataset / do_edge_split) over restated PyG stubs."""
    pyg = types.ModuleType("torch_geometric")
    pyg.datasets = types.ModuleType("torch_geometric.datasets")
    pd = types.ModuleType("torch_geometric.data")
    pd.Data, pd.Dataset = _PygData, list
    pu = types.ModuleType("torch_geometric.utils")
    pu.negative_sampling, pu.add_self_loops = _pyg_negative_sampling, _pyg_add_self_loops
    pu.train_test_split_edges = _pyg_train_test_split_edges
    pt = types.ModuleType("torch_geometric.transforms")
    for n in ("NormalizeFeatures", "Compose", "BaseTransform", "ToDevice", "RandomLinkSplit"):
        setattr(pt, n, None)
    stubs = {"torch_geometric": pyg, "torch_geometric.datasets": pyg.datasets, "torch_geometric.data": pd,
             "torch_geometric.utils": pu, "torch_geometric.transforms": pt}
    saved = {k: sys.modules.get(k) for k in stubs}
    sys.modules.update(stubs)
    try:
        mod = types.ModuleType("ref_utils")
        p = os.path.join(REF, "utils.py")
        exec(compile(_compile_file(p), p, "exec"), mod.__dict__)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def run_edge_split_case(name, N, E_und, seed, fast_split=False):
    """src/utils.py:62-105 (the SEAL split the reference caches as ../data/<ds>.pkl)."""
    mod = load_reference_utils()
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, N, (E_und,), generator=g)
    v = torch.randint(0, N, (E_und,), generator=g)
    keep = u != v
    ei = _pyg_coalesce_und(torch.stack([u[keep], v[keep]]), N)
    x = torch.randn(N, 4, generator=g)
    se = mod.do_edge_split([_PygData(x, ei)], fast_split=fast_split)
    out = dict(N=np.int64(N), x=x.numpy(), edge_index=ei.numpy(), fast_split=np.array(int(fast_split)))
    for s in ("train", "valid", "test"):
        for k in ("edge", "edge_neg"):
            out[f"{s}/{k}"] = se[s][k].numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def run_logger_case(name):
    """src/logger.py printed output for fixed result tables (the CLI's outputs
    must stay byte-identical)."""
    import contextlib
    import io
    import json
    mod = types.ModuleType("ref_logger")
    p = os.path.join(REF, "logger.py")
    exec(compile(_compile_file(p), p, "exec"), mod.__dict__)
    cases = []
    for cls, width in (("Logger", 2), ("ProductionLogger", 5)):
        table = [[[float(v) for v in torch.rand(width, generator=torch.Generator().manual_seed(run * 10 + ep))]
                  for ep in range(4)] for run in range(3)]
        L = getattr(mod, cls)(3)
        for run, rows in enumerate(table):
            for r in rows:
                L.add_result(run, tuple(r))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            L.print_statistics(1)
            L.print_statistics()
        cases.append({"cls": cls, "table": table, "stdout": buf.getvalue()})
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(cases, f, indent=1)


def main_norm(ref_models):
    """norm_type 'layer' / 'batch' (src/models.py:14,27-37,84-101): the student in the
    minibatch and full-batch steps, the SAGE teacher, and the modules alone."""
    run_norm_model_case("models_norm_fwd_bwd", ref_models, 3)
    run_minibatch_case("minibatch_layernorm_small", ref_models, N=257, F_=16, H=32, L=3, E_und=300, lbs=128,
                       args_over={}, seed=23, nepochs=1, norm_type="layer")
    run_minibatch_case("minibatch_batchnorm_small", ref_models, N=211, F_=16, H=32, L=3, E_und=260, lbs=96,
                       args_over={}, seed=24, nepochs=1, norm_type="batch")
    run_fullbatch_case("fullbatch_batchnorm_small", ref_models, N=120, F_=40, E_und=260, lbs=96, args_over={},
                       seed=25, norm_type="batch")
    run_fullbatch_case("fullbatch_layernorm_small", ref_models, N=90, F_=30, E_und=180, lbs=1024,
                       args_over=dict(KD_RM=0.0, KD_LM=0.0, LLP_D=1.0, LLP_R=0.5, hops=1, ns_rate=4),
                       seed=26, transductive="production", norm_type="layer")
    run_teacher_case("teacher_sage_batchnorm_small", N=130, F_=16, H=32, L=3, E_und=500, bs=200, updated=False,
                     transductive="transductive", seed=27, norm_type="batch")
    run_teacher_case("teacher_updated_layernorm_small", N=100, F_=48, H=64, L=3, E_und=350, bs=256,
                     updated=True, transductive="production", seed=29, norm_type="layer")


def main():
    ref_models = load_reference_models()
    if os.environ.get("GOLDEN_ONLY") == "norm":
        return main_norm(ref_models)
    run_edge_split_case("edge_split_small", N=200, E_und=700, seed=14)
    run_edge_split_case("edge_split_fast_small", N=150, E_und=500, seed=15, fast_split=True)
    if os.environ.get("GOLDEN_ONLY") == "edge_split":
        return
    run_production_split_case("production_split_cora_small", N=300, F_=8, E_und=900, ratios=(0.3, 0.3, 0.3, 0.1),
                              seed=12)
    run_production_split_case("production_split_small", N=500, F_=4, E_und=2500, ratios=(0.1, 0.1, 0.1, 0.1),
                              seed=13)
    if os.environ.get("GOLDEN_ONLY") == "production_split":
        return
    # GCN teacher (src/models.py:56-80): directed transductive graph (one-direction
    # adj_t, self-loops in the input) and a symmetric production graph, 3 layers
    run_teacher_case("teacher_gcn_small", N=110, F_=24, H=64, L=2, E_und=400, bs=160, updated=False,
                     transductive="transductive", seed=21, encoder="gcn", self_loops=6)
    run_teacher_case("teacher_gcn3_production_small", N=120, F_=40, H=32, L=3, E_und=380, bs=256,
                     updated=False, transductive="production", seed=22, encoder="gcn")
    if os.environ.get("GOLDEN_ONLY") == "gcn":
        return
    run_logger_case("logger_output")
    run_teacher_case("teacher_sage_small", N=110, F_=24, H=64, L=2, E_und=400, bs=160, updated=False,
                     transductive="transductive", seed=7)
    run_teacher_case("teacher_sage3_collab_small", N=130, F_=16, H=32, L=3, E_und=500, bs=200, updated=False,
                     transductive="transductive", seed=9, dataset="collab")
    run_teacher_case("teacher_updated_production_small", N=100, F_=48, H=64, L=2, E_und=350, bs=256,
                     updated=True, transductive="production", seed=8)
    run_kl_rank_case("kl_loss", 1)
    run_model_case("models_fwd_bwd", ref_models, 2)
    # collab-style minibatch path (main.py:52-144), C = 3*3*(1+3) = 36 like the
    # collab script, 3 link batches per epoch incl. a partial one, 2 epochs.
    run_minibatch_case("minibatch_collab_small", ref_models, N=257, F_=16, H=32, L=3, E_und=300, lbs=128,
                       args_over={}, seed=3, nepochs=2)
    # ps_method='rw', ns_rate=1, hops=2, rw_step=2 (C = 8), LLP_R only weight
    run_minibatch_case("minibatch_rw_small", ref_models, N=97, F_=8, H=24, L=2, E_und=150, lbs=64,
                       args_over=dict(ps_method="rw", rw_step=2, hops=2, ns_rate=1, LLP_D=0.0, LLP_R=2.0,
                                      True_label=1.0, margin=0.1), seed=4)
    # full-batch path (main.py:147-236) with dense negative sampling + KD terms
    run_fullbatch_case("fullbatch_cora_small", ref_models, N=120, F_=40, E_und=260, lbs=96, args_over={},
                       seed=5)
    run_fullbatch_case("fullbatch_production_small", ref_models, N=90, F_=30, E_und=180, lbs=1024,
                       args_over=dict(KD_RM=0.0, KD_LM=0.0, LLP_D=1.0, LLP_R=0.5, hops=1, ns_rate=4),
                       seed=6, transductive="production")
    main_norm(ref_models)


if __name__ == "__main__":
    main()
