"""Load the golden fixtures written by tests/golden/gen_golden.py into replayable
per-step records (inputs injected into the engine / oracle, expected outputs)."""
from __future__ import annotations

import os
import types

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def _args(z):
    a = types.SimpleNamespace()
    for k in z.files:
        if k.startswith("args/"):
            v = z[k]
            v = v.item() if v.ndim == 0 else v
            if isinstance(v, np.str_):
                v = str(v)
            setattr(a, k[5:], v)
    return a


def _params(z, prefix, names):
    return [torch.from_numpy(z[f"{prefix}/{n}"].copy()) for n in names]


def stu_names(L):
    return [f"layers.{i}.{w}" for i in range(L) for w in ("weight", "bias")]


def pred_names(L):
    return [f"lins.{i}.{w}" for i in range(L) for w in ("weight", "bias")]


def _keys(z, name):
    return [str(k) for k in z[name]] if name in z.files else []


def load_case(name):
    z = load(name)
    a = _args(z)
    L = int(z["L"])
    Lp = L  # LinkPredictor(..., args.num_layers, ...) (main.py:353-354)
    # norm_type cases name the student's parameters (Linear layers, then the norms' gamma / beta, as
    # model.parameters()) and its buffers (BatchNorm running statistics)
    snames = _keys(z, "stu_param_keys") or stu_names(L)
    bnames = _keys(z, "stu_buffer_keys")
    case = types.SimpleNamespace(
        name=name, args=a, N=int(z["N"]), F=int(z["F"]), H=int(z["H"]), L=L,
        x=torch.from_numpy(z["x"].copy()), t_h=torch.from_numpy(z["t_h"].copy()),
        edge_index=torch.from_numpy(z["edge_index"].copy()),
        train_pairs=torch.from_numpy(z["train_pairs"].copy()),
        epoch_losses=z["epoch_losses"],
        stu0=_params(z, "init/stu", snames), pred0=_params(z, "init/pred", pred_names(Lp)),
        tpred=_params(z, "tpred", pred_names(2)),
        stu_final=_params(z, "final/stu", snames), pred_final=_params(z, "final/pred", pred_names(Lp)),
        norm_type=str(z["norm_type"]) if "norm_type" in z.files else "none",
        stu_buffer_names=bnames, stu_buf0=_params(z, "init/stu", bnames),
        stu_buf_final=_params(z, "final/stu", bnames),
        h_eval=torch.from_numpy(z["h_eval"].copy()) if "h_eval" in z.files else None,
        steps=[])
    nsteps = int(z["nsteps"])
    minibatch = name.startswith("minibatch")
    full = not minibatch
    if a.transductive == "transductive":
        pos_train_edge = case.train_pairs
    else:
        pos_train_edge = case.edge_index.t()
    case.pos_train_edge = pos_train_edge
    for s in range(nsteps):
        st = types.SimpleNamespace()
        st.link_perm = torch.from_numpy(z[f"perm/{2 * s}"].copy())
        st.node_perm = torch.from_numpy(z[f"perm/{2 * s + 1}"].copy())
        st.edge = pos_train_edge[st.link_perm].t()
        walks = []
        w = 0
        while f"step{s}/walk{w}" in z.files:
            walks.append(torch.from_numpy(z[f"step{s}/walk{w}"].copy()))
            w += 1
        ri = []
        r = 0
        while f"step{s}/randint{r}" in z.files:
            ri.append(torch.from_numpy(z[f"step{s}/randint{r}"].copy()))
            r += 1
        if minibatch:
            st.neg_edge = ri[0]                       # main.py:84
            neg_batch = ri[1] if len(ri) > 1 else None
        else:
            st.neg_edge = torch.from_numpy(z[f"step{s}/neg_edge"].copy())   # main.py:206
            neg_batch = ri[0] if ri else None
        if walks:
            pos = walks[0]
            for wk in walks[1:]:
                pos = torch.cat([pos, wk[:, 1:]], 1)   # main.py:45
            st.samples = torch.cat([pos, neg_batch], 1)  # main.py:94,183
        else:
            st.samples = None
        for k in ("llp_d", "llp_r", "bce"):
            key = f"step{s}/{k}"
            setattr(st, k, float(z[key]) if key in z.files else None)
        ng = len(case.stu0) + len(case.pred0)
        st.grads = [torch.from_numpy(z[f"step{s}/grad{i}"].copy()) for i in range(ng)]
        case.steps.append(st)
    case.full = full
    return case


def load_teacher_case(name):
    """Fixtures of the reference teacher's train() (src/train_teacher_gnn.py:21-73)."""
    z = load(name)
    enc_keys = _keys(z, "enc_param_keys") or [str(k) for k in z["enc_keys"]]   # the encoder's parameters
    buf_keys = [k for k in _keys(z, "enc_keys") if k not in enc_keys]           # its buffers (BatchNorm)
    pred_keys = [str(k) for k in z["pred_keys"]]
    c = types.SimpleNamespace(
        name=name, N=int(z["N"]), F=int(z["F"]), H=int(z["H"]), L=int(z["L"]), updated=bool(int(z["updated"])),
        batch_size=int(z["batch_size"]), transductive=str(z["transductive"]), dataset=str(z["dataset"]),
        x=torch.from_numpy(z["x"].copy()), edge_index=torch.from_numpy(z["edge_index"].copy()),
        train_pairs=torch.from_numpy(z["train_pairs"].copy()), epoch_losses=z["epoch_losses"],
        enc0=_params(z, "init/enc", enc_keys), pred0=_params(z, "init/pred", pred_keys),
        enc_final=_params(z, "final/enc", enc_keys), pred_final=_params(z, "final/pred", pred_keys),
        h_eval=torch.from_numpy(z["h_eval"].copy()), steps=[],
        encoder=str(z["encoder"]) if "encoder" in z.files else "sage",
        norm_type=str(z["norm_type"]) if "norm_type" in z.files else "none",
        enc_buffer_names=buf_keys, enc_buf0=_params(z, "init/enc", buf_keys),
        enc_buf_final=_params(z, "final/enc", buf_keys))
    c.pos_train_edge = c.train_pairs if c.transductive == "transductive" else c.edge_index.t()
    ng = len(c.enc0) + len(c.pred0)
    for s in range(int(z["nsteps"])):
        st = types.SimpleNamespace()
        st.link_perm = torch.from_numpy(z[f"perm/{s}"].copy())
        st.edge = c.pos_train_edge[st.link_perm].t()
        if f"step{s}/neg_edge" in z.files:
            st.neg_edge = torch.from_numpy(z[f"step{s}/neg_edge"].copy())
        else:
            st.neg_edge = torch.from_numpy(z[f"step{s}/randint0"].copy())
        st.bce = float(z[f"step{s}/bce"])
        st.grads = [torch.from_numpy(z[f"step{s}/grad{i}"].copy()) for i in range(ng)]
        c.steps.append(st)
    return c


TEACHER_CASES = ["teacher_sage_small", "teacher_sage3_collab_small", "teacher_updated_production_small",
                 "teacher_gcn_small", "teacher_gcn3_production_small", "teacher_sage_batchnorm_small",
                 "teacher_updated_layernorm_small"]
MINIBATCH_CASES = ["minibatch_collab_small", "minibatch_rw_small", "minibatch_layernorm_small",
                   "minibatch_batchnorm_small"]
FULLBATCH_CASES = ["fullbatch_cora_small", "fullbatch_production_small", "fullbatch_batchnorm_small",
                   "fullbatch_layernorm_small"]


def free_params(case, per_layer=2):
    """Indices (in model.parameters() order) of the Linear / lin_l biases that feed a
    BatchNorm (norm_type 'batch'): their gradient is 0 in exact arithmetic, so the
    recorded one is rounding noise and Adam moves them by up to +-lr per step either way."""
    if getattr(case, "norm_type", "none") != "batch":
        return set()
    return {per_layer * l + 1 for l in range(case.L - 1)}


def set_state(model, params, buffers):
    """Copy parameters (model.parameters() order) and buffers (model.buffers() order) in."""
    with torch.no_grad():
        for p, v in zip(model.parameters(), params):
            p.copy_(v)
        for b, v in zip(model.buffers(), buffers):
            b.copy_(v)
