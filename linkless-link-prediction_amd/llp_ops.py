"""Module-level HIP ops (autograd-aware) behind the reference's nn.Module API.

Each op is a torch.autograd.Function whose forward/backward launch
libllp_hip kernels (llp_hip.py); nothing here computes on the CPU.  These serve
the reference's module surface — ``MLP``, ``LinkPredictor``, ``SAGE``
(src/models.py) — for evaluation (src/train_teacher_gnn.py:76-268) and for the
teacher's autograd training step (src/train_teacher_gnn.py:21-73).  The
distillation hot path itself runs in llp_engine.DistillEngine, which fuses
these pieces without autograd.
"""
from __future__ import annotations

import torch

import llp_hip as K

_seed_ctr = None


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("LLP ops run only on the MI355X HIP device (got a CPU tensor; no CPU fallback)")


def _dropout_state(device):
    """Per-process dropout stream counter on the device (graph-safe)."""
    global _seed_ctr
    if _seed_ctr is None or _seed_ctr.device != device:
        _seed_ctr = torch.zeros(1, dtype=torch.int64, device=device)
    return _seed_ctr


def _dropout_seed():
    return int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF


def _row2d(x):
    return x.reshape(-1, x.shape[-1]).contiguous()


class _LinearAct(torch.autograd.Function):
    """y = dropout(act(x W^T + b)) with x optionally x_i * x_j (Hadamard operand)."""

    @staticmethod
    def forward(ctx, x, x2, W, b, relu, p, training):
        M, Kd = x.shape
        N = W.shape[0]
        dt = x.dtype
        y = torch.empty(M, N, dtype=dt, device=x.device)
        drop = None
        if training and p > 0:
            ctr = _dropout_state(x.device)
            drop = K.Dropout(float(p), _dropout_seed(), ctr.data_ptr(), 3)
        Wc = W if W.dtype == dt else W.to(dt)
        A = K.operand(x, None, x2, None) if x2 is not None else K.operand(x)
        K.gemm_nt(A, K.operand(Wc.contiguous()), M, N, Kd, y, K.dtype_code(dt), bias=b.float().contiguous()
                  if b is not None else None, act=K.ACT_RELU if relu else K.ACT_NONE, dropout=drop)
        if drop is not None:
            K.increment(_dropout_state(x.device))
        ctx.save_for_backward(x, x2, W, y)
        ctx.relu = relu
        ctx.alpha = 1.0 / (1.0 - p) if (training and p > 0) else 1.0
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, x2, W, y = ctx.saved_tensors
        gy = gy.contiguous()
        M, N = gy.shape
        Kd = W.shape[1]
        dt = x.dtype
        dc = K.dtype_code(dt)
        if ctx.relu or ctx.alpha != 1.0:
            gz = torch.empty_like(gy)
            K.relu_bwd(gy, y if ctx.relu else None, ctx.alpha, gz)
        else:
            gz = gy
        gx = gx2 = gW = gb = None
        Wt = K.transpose(W.to(dt).contiguous())
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gA = torch.empty(M, Kd, dtype=dt, device=gy.device)
            K.gemm_nt(K.operand(gz), K.operand(Wt), M, Kd, N, gA, dc)
            if x2 is None:
                gx = gA
            else:
                gx = K.mul(gA, x2) if ctx.needs_input_grad[0] else None
                gx2 = K.mul(gA, x) if ctx.needs_input_grad[1] else None
        if ctx.needs_input_grad[2]:
            gW = torch.empty(N, Kd, dtype=torch.float32, device=gy.device)
            ws = torch.empty(K.gemm_tn_ws_bytes(dc, M, N, Kd) // 4 + 16, dtype=torch.float32, device=gy.device)
            A_in = K.operand(x, None, x2, None) if x2 is not None else K.operand(x)
            K.gemm_tn(K.operand(gz), A_in, M, N, Kd, gW, dc, ws)
            gW = gW.to(W.dtype)
        if ctx.has_b and ctx.needs_input_grad[3]:
            gb = torch.empty(N, dtype=torch.float32, device=gy.device)
            ws = torch.empty(K.colsum_ws_bytes(M, N) // 4 + 16, dtype=torch.float32, device=gy.device)
            K.colsum(gz, M, N, gb, ws)
        return gx, gx2, gW, gb, None, None, None


def linear(x, weight, bias=None, relu=False, dropout=0.0, training=False, x2=None):
    """nn.Linear (+ReLU, +dropout) on the HIP GEMM; ``x2`` makes the input x*x2."""
    _require_cuda(x, weight)
    shp = x.shape
    x2d = _row2d(x)
    x22d = _row2d(x2) if x2 is not None else None
    if x22d is not None and x22d.dtype != x2d.dtype:
        x22d = x22d.to(x2d.dtype)
    y = _LinearAct.apply(x2d, x22d, weight, bias, relu, float(dropout), bool(training))
    return y.reshape(*shp[:-1], weight.shape[0])


class _ReluDropout(torch.autograd.Function):
    """F.dropout(F.relu(x)) between SAGE layers (src/models.py:117-118)."""

    @staticmethod
    def forward(ctx, x, p, training):
        y = torch.empty_like(x)
        drop = None
        if training and p > 0:
            ctr = _dropout_state(x.device)
            drop = K.Dropout(float(p), _dropout_seed(), ctr.data_ptr(), 4)
        K.act_2d(x, y, act=K.ACT_RELU, dropout=drop)
        if drop is not None:
            K.increment(_dropout_state(x.device))
        ctx.save_for_backward(y)
        ctx.alpha = 1.0 / (1.0 - p) if (training and p > 0) else 1.0
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gx = torch.empty_like(y)
        K.relu_bwd_2d(gy.contiguous(), y, ctx.alpha, gx)
        return gx, None, None


def relu_dropout(x, p=0.0, training=False):
    _require_cuda(x)
    x2d = _row2d(x)
    return _ReluDropout.apply(x2d, float(p), bool(training)).reshape(x.shape)


class _NormAct(torch.autograd.Function):
    """dropout(relu(norm(y))) with norm an nn.LayerNorm / nn.BatchNorm1d module
    (norm_type 'layer' / 'batch', src/models.py:50-53, :114-118).  BatchNorm in train
    mode normalises by the batch statistics and updates the module's running
    statistics in place (torch's BatchNorm1d.train()); in eval mode it uses them."""

    @staticmethod
    def forward(ctx, y, gamma, beta, mod, p, training):
        M, H = y.shape
        batch = isinstance(mod, torch.nn.BatchNorm1d)
        kind = K.NORM_BATCH if batch else K.NORM_LAYER
        bn_train = batch and (training or not mod.track_running_stats)
        stats = torch.empty(2, H if batch else M, dtype=torch.float32, device=y.device)
        ws = torch.empty(K.norm_ws_bytes(M, H), dtype=torch.uint8, device=y.device)
        sums = None
        if bn_train:
            if mod.momentum is None and mod.track_running_stats:
                raise NotImplementedError("BatchNorm1d(momentum=None) (cumulative average)")
            sums = torch.empty(2, H, dtype=torch.float64, device=y.device)
            K.norm_colsums(y, sums, ws)
        drop = None
        if training and p > 0:
            drop = K.Dropout(float(p), _dropout_seed(), _dropout_state(y.device).data_ptr(), 5)
        out = torch.empty_like(y)
        upd = batch and training and mod.track_running_stats
        K.norm_fwd(kind, y, out, stats, None if gamma is None else gamma.detach(),
                   None if beta is None else beta.detach(), float(mod.eps), bn_train or not batch, sums, float(M),
                   float(getattr(mod, "momentum", 0.0) or 0.0), mod.running_mean if upd or (batch and not bn_train) else None,
                   mod.running_var if upd or (batch and not bn_train) else None,
                   mod.num_batches_tracked if upd else None, relu=True, dropout=drop)
        if drop is not None:
            K.increment(_dropout_state(y.device))
        ctx.save_for_backward(y, out, stats, gamma)
        ctx.kind, ctx.batch, ctx.bn_train = kind, batch, bn_train
        ctx.alpha = 1.0 / (1.0 - p) if (training and p > 0) else 1.0
        ctx.has = (gamma is not None, beta is not None)
        return out

    @staticmethod
    def backward(ctx, gout):
        y, out, stats, gamma = ctx.saved_tensors
        if ctx.batch and not ctx.bn_train:
            raise NotImplementedError("backward through BatchNorm1d in eval mode")
        M, H = y.shape
        gout = gout.contiguous()
        ws = torch.empty(K.norm_ws_bytes(M, H), dtype=torch.uint8, device=y.device)
        sums = torch.empty(2, H, dtype=torch.float64, device=y.device)
        dgamma = torch.empty(H, dtype=torch.float32, device=y.device) if ctx.has[0] else None
        dbeta = torch.empty(H, dtype=torch.float32, device=y.device) if ctx.has[1] else None
        K.norm_bwd_sums(ctx.kind, gout, out, ctx.alpha, y, stats, sums, ws, dgamma=dgamma, dbeta=dbeta)
        gy = torch.empty_like(y)
        K.norm_bwd(ctx.kind, gout, out, ctx.alpha, y, stats, gy, None if gamma is None else gamma.detach(), sums,
                   float(M))
        return gy, dgamma, dbeta, None, None, None


def norm_act(y, mod, p=0.0, training=False):
    """dropout(relu(mod(y))) for mod an nn.LayerNorm(H) / nn.BatchNorm1d(H)."""
    _require_cuda(y)
    y2d = _row2d(y)
    if isinstance(mod, torch.nn.LayerNorm) and tuple(mod.normalized_shape) != (y2d.shape[1],):
        raise NotImplementedError(f"LayerNorm over {tuple(mod.normalized_shape)}")
    if not isinstance(mod, (torch.nn.LayerNorm, torch.nn.BatchNorm1d)):
        raise NotImplementedError(type(mod).__name__)
    w = getattr(mod, "weight", None)
    b = getattr(mod, "bias", None)
    return _NormAct.apply(y2d, w, b, mod, float(p), bool(training)).reshape(y.shape)


class _Head(torch.autograd.Function):
    """sigmoid(z w + b) (w = None: sigmoid(sum(z * z2))) — LinkPredictor's tail."""

    @staticmethod
    def forward(ctx, z, z2, w, b):
        R, H = z.shape
        prob = torch.empty(R, dtype=torch.float32, device=z.device)
        K.head_fwd(z, R, H, w.float().reshape(-1).contiguous() if w is not None else None,
                   b.float().contiguous() if b is not None else None, prob=prob, Z2=z2)
        ctx.save_for_backward(z, z2, w, prob)
        return prob

    @staticmethod
    def backward(ctx, gprob):
        z, z2, w, prob = ctx.saved_tensors
        R, H = z.shape
        dlogit = torch.empty(R, dtype=torch.float32, device=z.device)
        K.sigmoid_bwd(gprob.float().contiguous(), prob, dlogit)
        gz = gz2 = gw = gb = None
        if w is not None:
            gz = torch.empty_like(z)
            gwf = torch.empty(H, dtype=torch.float32, device=z.device)
            gbf = torch.empty(1, dtype=torch.float32, device=z.device)
            ws = torch.empty(K.head_bwd_ws_bytes(R, H) // 4 + 16, dtype=torch.float32, device=z.device)
            K.head_bwd(dlogit, z, R, H, w.float().reshape(-1).contiguous(), False, gz, gwf, gbf, ws)
            gw = gwf.reshape(w.shape).to(w.dtype)
            gb = gbf.to(w.dtype) if ctx.needs_input_grad[3] else None
        else:
            gz = K.row_scale(z2, dlogit)
            gz2 = K.row_scale(z, dlogit)
        return gz, gz2, gw, gb


def head(z, weight=None, bias=None, z2=None):
    _require_cuda(z)
    shp = z.shape
    z2d = _row2d(z)
    z22d = _row2d(z2) if z2 is not None else None
    p = _Head.apply(z2d, z22d, weight, bias)
    return p.reshape(*shp[:-1], 1) if weight is not None else p.reshape(*shp[:-1])


class _MeanAgg(torch.autograd.Function):
    """PyG mean aggregation over a CSR by destination (llp_csr_aggregate)."""

    @staticmethod
    def forward(ctx, x, graph):
        out = torch.empty(graph.num_dst, x.shape[1], dtype=x.dtype, device=x.device)
        K.csr_aggregate(graph.num_dst, x.shape[1], graph.rowptr, graph.col, x.contiguous(), None, 0, out)
        ctx.graph = graph
        ctx.n_src = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, gout):
        g = ctx.graph
        gx = torch.empty(ctx.n_src, gout.shape[1], dtype=gout.dtype, device=gout.device)
        K.csr_aggregate(ctx.n_src, gout.shape[1], g.rowptr_t, g.col_t, gout.contiguous(), g.inv_deg, 1, gx)
        return gx, None


def mean_aggregate(x, graph):
    _require_cuda(x)
    return _MeanAgg.apply(x, graph)


class _GCNAgg(torch.autograd.Function):
    """GCN propagation D^-1/2 A D^-1/2 y (+ bias) over the self-loop CSR (llp_gcn_aggregate)."""

    @staticmethod
    def forward(ctx, y, bias, graph):
        out = torch.empty(graph.num_dst, y.shape[1], dtype=y.dtype, device=y.device)
        K.gcn_aggregate(graph.num_dst, y.shape[1], graph.rowptr, graph.col, y.contiguous(), graph.dinv, out,
                        bias=None if bias is None else bias.detach().float().contiguous())
        ctx.graph = graph
        ctx.n_src = y.shape[0]
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        g = ctx.graph
        gout = gout.contiguous()
        gy = torch.empty(ctx.n_src, gout.shape[1], dtype=gout.dtype, device=gout.device)
        K.gcn_aggregate(ctx.n_src, gout.shape[1], g.rowptr_t, g.col_t, gout, g.dinv, gy)
        gb = None
        if ctx.has_bias and ctx.needs_input_grad[1]:
            gb = torch.empty(gout.shape[1], dtype=torch.float32, device=gout.device)
            ws = torch.empty(K.colsum_ws_bytes(gout.shape[0], gout.shape[1]), dtype=torch.uint8, device=gout.device)
            K.colsum(gout, gout.shape[0], gout.shape[1], gb, ws)
        return gy, gb, None


def gcn_aggregate(y, graph, bias=None):
    _require_cuda(y)
    return _GCNAgg.apply(y, bias, graph)
