"""Drop-in replacements for the reference's training and evaluation functions,
same names, arguments and return values:

  train_minibatch(model, predictor, t_h, teacher_predictor, data, split_edge, optimizer, args, device)
                                                              src/main.py:52-144
  train(model, predictor, t_h, teacher_predictor, data, split_edge, optimizer, args, device)
                                                              src/main.py:147-236
  train_teacher(model, predictor, data, split_edge, optimizer, batch_size, encoder_name, dataset, transductive)
                                                              src/train_teacher_gnn.py:21-73 (``train`` there)
  test_transductive(model, predictor, data, split_edge, evaluator, batch_size, encoder_name, dataset, args)
                                                              src/train_teacher_gnn.py:76-155
  test_production(model, predictor, val_data, inference_data, test_edge_bundle, negative_samples,
                  evaluator, batch_size, encoder_name, dataset)
                                                              src/train_teacher_gnn.py:157-268

Each epoch runs on a cached engine (llp_engine.DistillEngine /
llp_teacher.TeacherEngine) bound to the given modules and optimizer: the
modules' parameters stay the masters (state_dict / torch.save unchanged), the
optimizer's Adam state is the engine's.  ``args.dtype`` ('fp32' default, as
the reference; 'bf16' for the MFMA fast path) is an additive option.

Shuffling: the reference's DataLoader(shuffle=True) permutations come from
torch's global generator; here one seed is drawn from that generator per
epoch and the permutations are generated on the device, so runs are
reproducible under seed_everything but not bit-identical to the reference's
streams (RNG streams are not portable anyway).

Multi-GPU: when torch.distributed is initialised, every rank draws the same
permutations.  The minibatch step gives each rank the whole batch and the
engine assigns every predictor pair to one rank (the owner decomposition,
DistillEngine.minibatch_owner; with dropout or BatchNorm each rank takes its
contiguous slice of the anchor / link batch instead); the full-batch step
slices.  Gradients are all-reduced inside the engine (strong scaling).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import llp_eval
import llp_hip as K
from llp_engine import DistillEngine

_ENGINES = {}


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def _epoch_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _device_perm(n, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randperm(n, generator=g, device=device).to(torch.int32)


def _as_pairs(t, device):
    return t.to(device).to(torch.int32).contiguous()


def _distill_engine(model, predictor, t_h, teacher_predictor, data, optimizer, args, device, row, col):
    key = ("distill", id(model), id(predictor), id(optimizer), id(data))
    eng = _ENGINES.get(key)
    if eng is None:
        for k in [k for k in _ENGINES if k[0] == "distill" and k[1:3] == key[1:3]]:
            del _ENGINES[k]          # a new run (fresh optimizer) replaces the old engine
        dev = torch.device(device) if not isinstance(device, torch.device) else device
        if dev.type != "cuda":
            dev = torch.device("cuda", torch.cuda.current_device())
        eng = DistillEngine(model, predictor, teacher_predictor, data.x, t_h, row.cpu().numpy(), col.cpu().numpy(),
                            data.x.size(0), args, optimizer, dtype=getattr(args, "dtype", "fp32"),
                            seed=_epoch_seed(), device=dev)
        _ENGINES[key] = eng
    return eng


def _slices(total, world, rank):
    return rank * total // world, (rank + 1) * total // world


def train_minibatch(model, predictor, t_h, teacher_predictor, data, split_edge, optimizer, args, device):
    """src/main.py:52-144 on the device: returns the epoch's mean loss."""
    if args.transductive == "transductive":
        pos_train_edge = split_edge["train"]["edge"]
        row, col = data.adj_t
    else:
        pos_train_edge = data.edge_index.t()
        row, col = data.edge_index
    model.train()
    predictor.train()
    eng = _distill_engine(model, predictor, t_h, teacher_predictor, data, optimizer, args, device, row, col)
    world, rank = _world()
    dev = eng.dev
    pairs = _as_pairs(pos_train_edge, dev)
    E = pairs.shape[0]
    N = data.x.size(0)
    seed = _epoch_seed()
    link_perm = _device_perm(E, seed, dev)
    node_perm = _device_perm(N, seed ^ 0x5A5A5A5A, dev)
    lbs, nbs = int(args.link_batch_size), int(args.node_batch_size)
    dense = args.datasets != "collab"                                   # src/main.py:80-84
    eng.begin_epoch()
    total = 0
    for i, s in enumerate(range(0, E, lbs)):
        P_tot = min(lbs, E - s)
        n0 = i * nbs
        if n0 >= N:
            raise StopIteration("node loader exhausted (the reference's next(node_loader) raises here)")
        B_tot = min(nbs, N - n0)
        if eng.minibatch_owner:   # every rank takes the whole batch and evaluates the pairs it owns
            eng.step_minibatch(node_perm[n0:n0 + B_tot], link_perm[s:s + P_tot], pairs, dense_negatives=dense)
        else:
            b0, b1 = _slices(B_tot, world, rank)
            p0, p1 = _slices(P_tot, world, rank)
            eng.step_minibatch(node_perm[n0 + b0:n0 + b1], link_perm[s + p0:s + p1], pairs, b_offset=b0,
                               p_offset=p0, B_total=B_tot, P_total=P_tot, dense_negatives=dense)
        total += P_tot
    return eng.end_epoch(total)


def train(model, predictor, t_h, teacher_predictor, data, split_edge, optimizer, args, device):
    """src/main.py:147-236 (student MLP over all nodes each link batch)."""
    if args.transductive == "transductive":
        pos_train_edge = split_edge["train"]["edge"]
        row, col = data.adj_t
    else:
        pos_train_edge = data.edge_index.t()
        row, col = data.edge_index
    model.train()
    predictor.train()
    eng = _distill_engine(model, predictor, t_h, teacher_predictor, data, optimizer, args, device, row, col)
    world, rank = _world()
    dev = eng.dev
    pairs = _as_pairs(pos_train_edge, dev)
    E = pairs.shape[0]
    N = data.x.size(0)
    seed = _epoch_seed()
    link_perm = _device_perm(E, seed, dev)
    node_perm = _device_perm(N, seed ^ 0x5A5A5A5A, dev)
    lbs, nbs = int(args.link_batch_size), int(args.node_batch_size)
    dense = args.datasets != "collab"                                   # src/main.py:205-209
    eng.begin_epoch()
    total = 0
    for i, s in enumerate(range(0, E, lbs)):
        P_tot = min(lbs, E - s)
        n0 = i * nbs
        if n0 >= N:
            raise StopIteration("node loader exhausted (the reference's next(node_loader) raises here)")
        B_tot = min(nbs, N - n0)
        b0, b1 = _slices(B_tot, world, rank)
        p0, p1 = _slices(P_tot, world, rank)
        eng.step_fullbatch(node_perm[n0 + b0:n0 + b1], link_perm[s + p0:s + p1], pairs, b_offset=b0, p_offset=p0,
                           B_total=B_tot, P_total=P_tot, dense_negatives=dense)
        total += P_tot
    return eng.end_epoch(total)


def _teacher_engine(model, predictor, data, optimizer, edge_index, dtype):
    import llp_teacher
    key = ("teacher", id(model), id(predictor), id(optimizer), id(data))
    eng = _ENGINES.get(key)
    if eng is None:
        for k in [k for k in _ENGINES if k[0] == "teacher" and k[1:3] == key[1:3]]:
            del _ENGINES[k]
        eng = llp_teacher.TeacherEngine(model, predictor, data.x, edge_index, data.x.size(0), optimizer, dtype=dtype,
                                        seed=_epoch_seed())
        _ENGINES[key] = eng
    return eng


def train_teacher(model, predictor, data, split_edge, optimizer, batch_size, encoder_name, dataset, transductive,
                  dtype="fp32"):
    """src/train_teacher_gnn.py:21-73 for encoder_name 'sage' / 'gcn'
    (TeacherEngine) and 'mlp' (the full-batch DistillEngine with every
    distillation weight zero)."""
    if transductive == "transductive":
        mp_edges = data.adj_t
        pos_train_edge = split_edge["train"]["edge"]
    else:
        mp_edges = data.edge_index
        pos_train_edge = data.edge_index.t()
    if encoder_name == "mlp":
        return _train_teacher_mlp(model, predictor, data, pos_train_edge, mp_edges, optimizer, batch_size, dataset,
                                  dtype)
    if encoder_name not in ("sage", "gcn"):
        raise ValueError(f"unknown encoder {encoder_name!r}")
    model.train()
    predictor.train()
    eng = _teacher_engine(model, predictor, data, optimizer, mp_edges, dtype)
    dev = eng.dev
    pairs = _as_pairs(pos_train_edge, dev)
    E = pairs.shape[0]
    perm = _device_perm(E, _epoch_seed(), dev)
    eng.begin_epoch()
    for s in range(0, E, batch_size):
        eng.step(perm[s:s + batch_size], pairs, dense_negatives=(dataset != "collab"))
    return eng.end_epoch(E)


def _train_teacher_mlp(model, predictor, data, pos_train_edge, mp_edges, optimizer, batch_size, dataset, dtype):
    """The supervised MLP baseline of src/train_teacher_gnn.py:36-37: BCE on
    (pos, neg) with h = model(x) over all nodes — the full-batch distillation
    step with every distillation weight zero."""
    import types
    import models
    key = ("mlp-teacher", id(model), id(predictor), id(optimizer), id(data))
    eng = _ENGINES.get(key)
    if eng is None:
        for k in [k for k in _ENGINES if k[0] == "mlp-teacher" and k[1:3] == key[1:3]]:
            del _ENGINES[k]
        a = types.SimpleNamespace(rw_step=1, hops=1, ns_rate=0, ps_method="nb", dropout=float(model.dropout.p),
                                  margin=0.0, LLP_D=0.0, LLP_R=0.0, True_label=1.0, KD_RM=0.0, KD_LM=0.0,
                                  predictor=predictor.predictor)
        dummy = models.LinkPredictor("mlp", 16, 16, 1, 2, 0.0)
        N = data.x.size(0)
        eng = DistillEngine(model, predictor, dummy, data.x, torch.zeros(N, 16), mp_edges[0].cpu().numpy(),
                            mp_edges[1].cpu().numpy(), N, a, optimizer, dtype=dtype, seed=_epoch_seed(),
                            device=torch.device("cuda", torch.cuda.current_device()))
        _ENGINES[key] = eng
    model.train()
    predictor.train()
    dev = eng.dev
    pairs = _as_pairs(pos_train_edge, dev)
    E = pairs.shape[0]
    perm = _device_perm(E, _epoch_seed(), dev)
    none = torch.zeros(0, dtype=torch.int32, device=dev)
    eng.begin_epoch()
    for s in range(0, E, batch_size):
        eng.step_fullbatch(none, perm[s:s + batch_size], pairs, dense_negatives=(dataset != "collab"))
    return eng.end_epoch(E)


def _embed(model, data, x, adj, encoder_name):
    if encoder_name == "mlp":
        return llp_eval.embed_mlp(model, x)
    for k, eng in _ENGINES.items():
        if k[0] == "teacher" and k[1] == id(model) and k[4] == id(data):
            return eng.embed()       # the engine's resident graph is this data's graph
    with torch.no_grad():   # module path (autograd ops, eval mode)
        return model(x, adj)


@torch.no_grad()
def test_transductive(model, predictor, data, split_edge, evaluator, batch_size, encoder_name, dataset, args=None):
    """src/train_teacher_gnn.py:76-155 -> (results, h); ``evaluator`` is not
    needed (the ogb hits@K formula runs on the device)."""
    model.eval()
    predictor.eval()
    x = data.x if data.x.is_cuda else data.x.to("cuda")
    h = _embed(model, data, x, getattr(data, "adj_t", None), encoder_name)
    return llp_eval.test_transductive(h, predictor, split_edge, dataset)


@torch.no_grad()
def test_production(model, predictor, val_data, inference_data, test_edge_bundle, negative_samples, evaluator,
                    batch_size, encoder_name, dataset):
    """src/train_teacher_gnn.py:157-268 -> (results, h of val_data)."""
    model.eval()
    predictor.eval()
    hv = _embed(model, val_data, val_data.x.to("cuda"), val_data.edge_index.to("cuda"), encoder_name)
    hi = _embed(model, inference_data, inference_data.x.to("cuda"), inference_data.edge_index.to("cuda"),
                encoder_name)
    ve = val_data.edge_label_index.t()
    lab = val_data.edge_label.bool()
    return llp_eval.test_production(hv, hi, predictor, ve[lab], ve[~lab], test_edge_bundle, negative_samples)


__all__ = ["train_minibatch", "train", "train_teacher", "test_transductive", "test_production", "K"]
