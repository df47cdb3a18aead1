"""MI355X LLP distillation engine: one relational-distillation step (sampling,
student MLP + LinkPredictor forward/backward, frozen teacher predictor, fused
LLP_D / LLP_R / BCE loss, clip_grad_norm_ per group, Adam) as a fixed sequence
of hand-written gfx950 kernels on preallocated HBM buffers.

Reference: ``train_minibatch`` (src/main.py:52-144) and ``train``
(src/main.py:147-236).  The nn.Modules stay the source of truth for the
weights (their ``.data``/``.grad``/optimizer state are the engine's buffers),
so ``state_dict()`` / ``torch.save`` interoperate with the reference's files.

Layout in HBM (minibatch path, one step, rows of h follow src/main.py:95):
    target  int32[R1]        node id per student row: samples.flat | src(2P) | dst(2P)
    H_l     dtype[R1, H]     student activations, R1 = B*(C+1) + 4P
    Z_l     dtype[R2, H]     predictor activations, R2 = B*C + 2P
    logit   f32[R2]          predictor logits: B*C context pairs | 2P label pairs
    T1      dtype[B*C, 256]  teacher predictor hidden layer
Weights: f32 masters (the modules' parameters) + a compute-dtype copy and a
transposed copy, refreshed by the Adam kernel.
"""
from __future__ import annotations

import contextlib
import functools
import math
import os

import numpy as np
import torch
import torch.distributed as dist

import llp_hip as K

# Philox streams per step (csrc/llp_common.h LLP_STREAMS_PER_STEP): a draw of step s at
# offset o uses stream STREAMS_PER_STEP * s + o.  Offsets under self.seed: the context
# sampler's walks 0 .. rw_step-1 and its negatives rw_step; randint negatives S-1; PyG-dense
# negatives S-2 under their own key; dropout 1 + layer under per-module keys.
STREAMS_PER_STEP = 64
RANDINT_STREAM = STREAMS_PER_STEP - 1
DENSE_NEG_STREAM = STREAMS_PER_STEP - 2
MAX_RW_STEP = STREAMS_PER_STEP - 3          # walks + negatives below DENSE_NEG_STREAM
# dropout Philox keys (EngineBase._dropout): one per module, one stream per layer and step
DROP_ENCODER, DROP_PREDICTOR, DROP_TEACHER_PRED = 0, 1, 2
# x at most this dense runs the full-batch student's first layer sparse (llp_spmm_rows): a
# gathered 512-B weight row per nonzero against a dense 256-wide MFMA pass over every column
SPARSE_X_MAX_DENSITY = 0.05
_MAX_DROPOUT_LAYERS = STREAMS_PER_STEP - 1

_DT = {"bf16": torch.bfloat16, "fp32": torch.float32, torch.bfloat16: torch.bfloat16, torch.float32: torch.float32}


def build_sampler_csr(row: np.ndarray, col: np.ndarray, num_nodes: int, sorted_: bool = False):
    """CSR for the context sampler with torch_cluster random_walk semantics
    (coalesced=False, src/main.py:37-45): rowptr = prefix sum of row degrees,
    col kept in the given (possibly unsorted) order.  ``sorted_``
    (--rw_sorted) sorts by (row, col) instead."""
    row = np.asarray(row, np.int64)
    col = np.asarray(col, np.int64)
    if sorted_:
        perm = np.argsort(row * num_nodes + col, kind="stable")
        col = col[perm]
    deg = np.bincount(row, minlength=num_nodes)
    rowptr = np.zeros(num_nodes + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    assert rowptr[-1] < 2 ** 31
    return rowptr.astype(np.int32), col.astype(np.int32)


class _Linear:
    """Device view of one nn.Linear: f32 master W/b (the module's params), their
    grads (views into the flat grad buffer), compute copies."""

    def __init__(self, lin: torch.nn.Linear, dtype, need_t: bool, need_c: bool):
        self.W = lin.weight.data
        self.b = lin.bias.data
        self.out_f, self.in_f = self.W.shape
        self.k_in = self.in_f      # GEMM inner dimension (the first student layer may run on zero-padded K)
        self.Wc = None
        self.Wt = None
        if need_c and dtype != torch.float32:
            self.Wc = torch.empty_like(self.W, dtype=dtype)
        if need_t:
            self.Wt = torch.empty(self.in_f, self.out_f, dtype=dtype, device=self.W.device)
        self.lin = lin

    @property
    def Wcomp(self):
        return self.Wc if self.Wc is not None else self.W


class _Norm:
    """Device view of one norm module after a hidden layer (``norm_type`` 'layer' /
    'batch', src/models.py:27-37,90-101): nn.LayerNorm(H) or nn.BatchNorm1d(H) with
    the reference's defaults (affine; BatchNorm with running statistics, momentum
    0.1).  gamma / beta are the module's parameters (their .grad views into the flat
    gradient); BatchNorm's running_mean / running_var / num_batches_tracked buffers
    are updated in place by the forward kernel, as torch's train() forward does."""

    def __init__(self, m: torch.nn.Module, width: int):
        if isinstance(m, torch.nn.LayerNorm):
            self.kind = K.NORM_LAYER
            if tuple(m.normalized_shape) != (width,):
                raise NotImplementedError(f"LayerNorm over {tuple(m.normalized_shape)} (the layer is {width} wide)")
        elif isinstance(m, torch.nn.BatchNorm1d):
            self.kind = K.NORM_BATCH
            if m.num_features != width:
                raise NotImplementedError(f"BatchNorm1d({m.num_features}) after a {width}-wide layer")
            if not m.track_running_stats or m.momentum is None:
                raise NotImplementedError("BatchNorm1d with running statistics and a fixed momentum (torch defaults)")
        else:
            raise NotImplementedError(f"norm module {type(m).__name__} (norm_type 'layer' or 'batch')")
        self.m = m
        self.eps = float(m.eps)
        self.momentum = float(getattr(m, "momentum", 0.0) or 0.0)
        self.params = [p for p in (m.weight, m.bias) if p is not None]

    @property
    def batch(self):
        return self.kind == K.NORM_BATCH

    def gamma(self):
        return None if self.m.weight is None else self.m.weight.data

    def beta(self):
        return None if self.m.bias is None else self.m.bias.data


def _norms_of(model, n_hidden, width):
    """The model's norm modules (one per hidden layer) as _Norm, or [] for norm_type 'none'."""
    mods = list(getattr(model, "norms", []))
    if not mods:
        return []
    if len(mods) != n_hidden:
        raise NotImplementedError(f"{len(mods)} norm modules for {n_hidden} hidden layers")
    return [_Norm(m, width) for m in mods]


def _acc_dtype(t):
    """f32, or the tensor's own dtype when that is wider (gloo has no bf16 sums)."""
    return t.dtype if t.dtype in (torch.float32, torch.float64) else torch.float32


def _resets_on_error(step):
    """Engine step decorator: a step that raises resets the persistent device state
    (EngineBase.reset_device_state) before the exception propagates."""
    @functools.wraps(step)
    def run(self, *args, **kw):
        return self._guarded(lambda: step(self, *args, **kw))
    return run


class _SegmentedGraph:
    """A multi-rank step as hipGraph segments with the collectives between them.

    Capture cuts the graph at every collective (``cut``); ``replay`` launches the
    segments on the current stream and runs each collective eagerly in between,
    so RCCL (or gloo) orders itself against the segments by the stream, exactly
    as in an eager step.  All segments share one memory pool."""

    def __init__(self, dev, mode="thread_local"):
        self.items = []
        self.stream = torch.cuda.Stream(device=dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.mode = mode
        self.g = None
        self._ctx = None

    def begin(self):
        self._ctx = torch.cuda.stream(self.stream)
        self._ctx.__enter__()
        self._open()

    def _open(self):
        self.g = torch.cuda.CUDAGraph()
        # thread_local: the process group's own threads may query events meanwhile
        self.g.capture_begin(pool=self.pool, capture_error_mode=self.mode)

    def _close(self):
        self.g.capture_end()
        self.items.append(self.g)
        self.g = None

    def cut(self, fn):
        self._close()
        self.items.append(fn)
        self._open()

    def end(self):
        try:
            if self.g is not None:
                self._close()
        finally:
            self._ctx.__exit__(None, None, None)

    def replay(self):
        for it in self.items:
            if isinstance(it, torch.cuda.CUDAGraph):
                it.replay()
            else:
                it()


class EngineBase:
    """Device state shared by the distillation and teacher engines: the flat
    f32 gradient buffer the parameters' ``.grad`` view, Adam state in the
    torch optimizer, the device descriptor table of the fused clip+Adam
    kernel (with each weight's compute-dtype / transposed shadows), the
    LinkPredictor's forward/backward, scratch buffers and the loss counters."""

    def _init_device(self, x_device, device, dtype, seed, group, name):
        self.dev = torch.device(device) if device is not None else x_device
        if self.dev.type != "cuda":
            raise RuntimeError(f"{name} runs only on a HIP device (no CPU fallback)")
        K.lib()
        self.dtype = _DT[dtype]
        self.dc = K.dtype_code(self.dtype)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.group = group
        self.world = dist.get_world_size(group) if (group is not None or (dist.is_available() and dist.is_initialized())) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=self.dev)   # RNG stream counter
        self.terms = torch.zeros(8, dtype=torch.float32, device=self.dev)
        # last-arriver ticket blocks of the one-launch loss and gradient norm (llp_llp_loss_heads,
        # llp_grad_sumsq_t): zero, and left zero by every call
        self.loss_ticket = K.ticket_block(self.dev)
        self.sumsq_ticket = K.ticket_block(self.dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self._bufs = {}
        self._shadows = {}
        self._act_mask = {}     # id(activation buffer) -> its ReLU bit mask (or None)
        self._seg = None        # _SegmentedGraph while a multi-rank step is being captured
        self._seg_debug = False  # extra segment cuts that sync and name the stage (capture_minibatch)
        self.emulate_shard = None   # (rank, world): time one rank's full-batch student slice (_fb_shard)
        # full-batch step: the dense negatives beside the student forward and the frozen teacher beside the
        # predictor forward, on a second stream (step_fullbatch); False: one stream
        self.overlap_streams = True
        # with overlap_streams (A/B switches, tools/physics_bench.py): the teacher and the node grouping
        # start right after the pairs when no row-sharded student needs a collective first; the node
        # grouping of the Hadamard backward runs on the side stream
        self.early_pair_work = True
        self.side_grouping = True
        self.side_sampling = True   # the context sampler on the side stream, before the negatives
        self.side_wgrad = True   # the full-batch student's small weight-gradient GEMMs beside the data gradients
        self._side = None
        self._side_open = False   # work forked onto the side stream since its last join
        self._cut_gen = 0         # segment cuts so far (events from an earlier segment are not waited on)
        self.emulate_pairs = None   # (rank, world): time one rank's owner-decomposed minibatch step

    def _init_params(self, all_params, groups, optimizer):
        """``groups[i]``: clip group of all_params[i] (clip_grad_norm_ per module, Q9)."""
        self.all_params = list(all_params)
        self.param_groups_of = list(groups)
        self.n_groups = max(self.param_groups_of) + 1
        total = sum(p.numel() for p in self.all_params)
        self.flat_grad = torch.zeros(total, dtype=torch.float32, device=self.dev)
        off = 0
        for p in self.all_params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        # group 0 (student / encoder) first, then the predictor: the predictor's
        # gradients are the tail of flat_grad, final once its backward is done
        assert self.param_groups_of == sorted(self.param_groups_of)
        self._tail_off = sum(p.numel() for p, gr in zip(self.all_params, self.param_groups_of) if gr == 0)
        self._works = []        # async all-reduce handles of this step's gradient buckets
        self._issued = []       # their [lo, hi) ranges in flat_grad
        self.optimizer = optimizer
        self._init_optimizer_state()

    def _set_shadow(self, p, shadow=None, shadow_t=None, ld=0, ld_t=0):
        """Register the compute-dtype copy (row stride ld) and/or transposed copy
        (row stride ld_t) the Adam kernel refreshes for parameter p."""
        self._shadows[id(p)] = (shadow, shadow_t, int(ld), int(ld_t))

    def _setup_predictor(self, predictor, kind):
        if kind not in ("mlp", "inner"):
            raise ValueError(kind)
        self.predictor_kind = kind
        prd = list(predictor.lins)
        if kind == "mlp":
            self.prd = [_Linear(l, self.dtype, need_t=True, need_c=True) for l in prd[:-1]]
            self.head = prd[-1]
        else:
            self.prd, self.head = [], None
        for l in self.prd:
            self._set_shadow(l.lin.weight, l.Wc, l.Wt)
        return [p for l in prd for p in (l.weight, l.bias)]

    # ------------------------------------------------------------------ setup
    def _init_optimizer_state(self):
        opt = self.optimizer
        if not isinstance(opt, torch.optim.Adam):
            raise NotImplementedError("the LLP engine implements torch.optim.Adam (src/main.py:400-402)")
        g = opt.param_groups
        if len(g) != 1 or g[0]["weight_decay"] != 0 or g[0]["amsgrad"] or g[0].get("maximize", False):
            raise NotImplementedError("Adam with one param group, no weight decay / amsgrad / maximize")
        ids = {id(p) for p in g[0]["params"]}
        if ids != {id(p) for p in self.all_params}:
            raise ValueError("optimizer must hold exactly model.parameters() + predictor.parameters()")
        step0 = 0
        for p in self.all_params:
            st = opt.state[p]
            if "exp_avg" not in st:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            step0 = int(float(st["step"]))
        self.adam_step = torch.full((1,), step0, dtype=torch.int64, device=self.dev)

    def _build_descs(self):
        opt = self.optimizer
        descs, shapes = [], []
        for p, grp in zip(self.all_params, self.param_groups_of):
            st = opt.state[p]
            shadow, shadow_t, ld, ld_t = self._shadows.get(id(p), (None, None, 0, 0))
            rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
            descs.append(K.TensorDesc(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                      st["exp_avg_sq"].data_ptr(), K.ptr(shadow), K.ptr(shadow_t), p.numel(), rows,
                                      cols, grp, self.dc, ld, ld_t))
            # the compact grids' item counts from the very tuples the descriptor holds
            shapes.append((p.numel(), rows, cols, shadow_t is not None))
        self.n_desc = len(descs)
        self.max_numel = max(p.numel() for p in self.all_params)
        # compact grids of the one-launch gradient norm and Adam (llp_grad_sumsq_w / llp_adam_step_w)
        self.n_work_sumsq, self.n_work_adam = K.work_items(shapes)
        self.descs_dev = K.descs_to_device(descs, self.dev)
        self.sumsq = torch.zeros(self.n_groups, dtype=torch.float32, device=self.dev)
        self.ws_sumsq = torch.empty(K.grad_sumsq_ws_bytes(self.n_desc, self.max_numel) // 4 + 1, dtype=torch.float32,
                                    device=self.dev)
        K.refresh_shadows(self.descs_dev, self.n_desc, self.max_numel)

    def refresh_weights(self):
        """Call after loading weights into the modules (reset_parameters, load_state_dict)."""
        K.refresh_shadows(self.descs_dev, self.n_desc, self.max_numel)

    def _buf(self, name, shape, dtype):
        numel = int(np.prod(shape))
        b = self._bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype:
            b = torch.empty(max(numel, 1), dtype=dtype, device=self.dev)
            self._bufs[name] = b
        return b[:numel].view(*shape)

    def _mask(self, name, rows, cols, k_fwd, k_bwd):
        """ReLU bit mask [rows, cols/8] (bf16 engine): the forward GEMM (inner
        dimension k_fwd) writes it, the ReLU-backward GEMM (inner dimension k_bwd)
        reads it instead of the bf16 activations.  Both must run on the 256-tile
        path (K % 64, N % 32), else None (the bf16 activations serve as before)."""
        if self.dtype != torch.bfloat16 or cols % 32 != 0 or k_fwd % 64 != 0 or k_bwd % 64 != 0:
            return None
        return self._buf(name, (rows, cols // 8), torch.uint8)

    def _ws(self, name, nbytes):
        return self._buf(name, (nbytes // 4 + 16,), torch.float32)

    def _dedup_ws(self, name, num_nodes, R):
        """The llp_dedup_rows2 workspace of one call site (its state persists between steps)."""
        d = self.__dict__.setdefault("_dedup_wss", {})
        w = d.get(name)
        if w is None or not w.fits(num_nodes, R):
            w = d[name] = K.DedupWorkspace(num_nodes, R, self.dev)
        return w

    def _splitk_plan(self, M, N, Kd):
        """Split count of the bf16 split-K GEMM for this shape (1: the plain GEMM), cached."""
        if self.dtype != torch.bfloat16:
            return 1
        cache = self.__dict__.setdefault("_splitk", {})
        key = (int(M), int(N), int(Kd))
        if key not in cache:
            cache[key] = int(K.gemm_nt_splitk_plan(*key))
        return cache[key]

    def _dropout(self, p, module, layer):
        """Dropout draws of ``layer`` of ``module`` (DROP_ENCODER: the student MLP / the
        teacher's GNN, DROP_PREDICTOR: the trained LinkPredictor, DROP_TEACHER_PRED: the
        frozen teacher predictor).  Each module has its own Philox key and each layer its
        own stream STREAMS_PER_STEP * step_ctr + 1 + layer, so no two (module, layer) pairs and no two
        steps share draws; the other seeds' streams (sampler, negatives) never meet them."""
        if p <= 0.0:
            return None
        if not 0 <= layer < _MAX_DROPOUT_LAYERS:
            raise ValueError(f"dropout on layer {layer}: at most {_MAX_DROPOUT_LAYERS} dropout layers per module "
                             f"(one Philox stream each per step)")
        key = (self.seed ^ 0xD0D0 ^ (int(module) << 40)) & 0xFFFFFFFFFFFFFFFF
        return K.Dropout(float(p), key, self.step_ctr.data_ptr(), 1 + layer)

    def _fusable(self, K_in, N_out, p_drop=0.0):
        """The last predictor layer's GEMM can carry the Linear(H,1) head: bf16 (any dropout), or
        fp32 without dropout on the persistent f32 kernel's shapes (N % 256 == 0)."""
        if self.dtype == torch.bfloat16:
            return K_in % 64 == 0 and N_out % 8 == 0
        return K_in % 64 == 0 and N_out % 256 == 0 and float(p_drop) == 0.0

    # ------------------------------------------------------------------ negatives
    def _neg_setup(self):
        """Keys of the negative-sampling graph ``edge_index = stack([col, row])``
        (src/main.py:156, src/train_teacher_gnn.py:28) in PyG's dense encoding
        (host, once per engine); ``self._neg_rc`` = (row, col) numpy arrays."""
        if getattr(self, "_neg_keys", None) is None:
            r, c = self._neg_rc
            src, dst = np.asarray(c, np.int64), np.asarray(r, np.int64)   # edge_index = [col, row]
            m = src != dst
            src, dst = src[m], dst[m]
            key = src * (self.N - 1) + dst - (src < dst)
            self._neg_n_idx = int(key.size)                              # duplicates counted, as PyG does
            self._neg_keys = torch.from_numpy(np.unique(key)).to(self.dev)
            self._neg_table = K.edge_table_build(self._neg_keys)          # membership set for the sampler
        return self._neg_keys

    def neg_sample_size(self, num_neg):
        """int(1.1 * num_neg / prob), prob = 1 - |idx| / (N(N-1)) (PyG 2.2.0)."""
        self._neg_setup()
        population = self.N * (self.N - 1)
        if self._neg_n_idx >= population:
            return 0
        prob = 1.0 - self._neg_n_idx / population
        return int(1.1 * num_neg / prob)

    def _negatives(self, P, P_total, p_offset, neg, dense, device_count=False):
        """This rank's negative edges: injected, PyG-dense (non-collab) or
        randint (collab) — src/main.py:205-209, src/train_teacher_gnn.py:49-54.
        Returns (int32[2, n] view, n, n_total, count): count is None, or with
        ``device_count`` and PyG-dense sampling the whole batch's int32 device count,
        in which case the view holds this rank's P negative SLOTS (columns
        [p_offset, p_offset + P) of the whole batch's list; slots past the count are
        inert in llp_fullbatch_pairs / llp_llp_loss), n = P and n_total = None: no
        host read."""
        N = self.N
        if neg is not None:
            n_neg = int(neg.shape[1])
            if self.world > 1:
                # the true total over the ranks' shards (BCE normaliser, BatchNorm row count),
                # not a proportional estimate; injected negatives are host-known (no capture)
                t = torch.tensor([n_neg], dtype=torch.int64, device=self.device)
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                n_neg_total = int(t.item())
            else:   # one rank, or an emulated shard (timing): proportional to the link slice
                n_neg_total = n_neg if P_total == P else int(round(n_neg * P_total / max(P, 1)))
            negb = self._buf("neg", (2, max(n_neg, 1)), torch.int32)
            negb[:, :n_neg].copy_(neg.to(torch.int32))
            return negb[:, :n_neg], n_neg, n_neg_total, None
        if dense:
            # every rank draws the same global list and keeps its column slice
            keys = self._neg_setup()
            ss = self.neg_sample_size(P_total)
            population = N * (N - 1)
            M = population if population <= ss else 3 * ss
            negg = self._buf("neg_all", (2, max(P_total, 1)), torch.int32)
            cnt = self._buf("neg_count", (1,), torch.int32)
            if population < (1 << 40):   # two launches, the sampler's state persisting between steps
                d = self.__dict__.setdefault("_neg_wss", {})
                if d.get("neg") is None or d["neg"].key != M:
                    d["neg"] = K.StatefulWorkspace(K.neg_sample2_ws_bytes(M), M, self.dev,
                                                   state_bytes=K.neg_sample2_state_bytes(M))
                K.neg_sample_dense2(N, keys, P_total, ss, self.seed ^ 0x5EED, self.step_ctr, DENSE_NEG_STREAM, negg,
                                    cnt, d["neg"], edge_table=self._neg_table)
            else:
                ws = self._buf("ws_neg", (K.neg_sample_ws_bytes(M) // 4 + 16,), torch.float32)
                K.neg_sample_dense(N, keys, P_total, ss, self.seed ^ 0x5EED, self.step_ctr, DENSE_NEG_STREAM, negg,
                                   cnt, ws, edge_table=self._neg_table)
            if device_count:
                return negg[:, p_offset:p_offset + P], P, None, cnt
            n_neg_total = int(cnt.item())
            lo = min(p_offset, n_neg_total)         # this shard's columns (all of them unsharded)
            hi = min(p_offset + P, n_neg_total)
            return negg[:, lo:hi], hi - lo, n_neg_total, None
        negb = self._buf("neg", (2, max(P, 1)), torch.int32)
        K.randint_pairs(N, P, self.seed, self.step_ctr, RANDINT_STREAM, negb, n_total=P_total, offset=p_offset)
        return negb, P, P_total, None

    def _predictor_forward(self, h, ia, ib, R2, logit, p_drop, defer_head=False):
        """LinkPredictor(h[ia], h[ib]) logits (src/models.py:139-150).  Returns
        (A0, zacts): the first layer's input operand and hidden activations.  With
        ``defer_head`` and the head fused into the last GEMM, the logits are left as head
        partials in ``self._s_head`` (K.head_in) for the loss launch to finish and write;
        otherwise ``self._s_head`` is None and ``logit`` is written here."""
        H = h.shape[1]
        dt, dc = self.dtype, self.dc
        zacts = []
        self._s_head = None
        if self.predictor_kind != "mlp":
            K.head_fwd(h, R2, H, None, None, logit=logit, Z2=h, iz=ia, iz2=ib)
            return None, zacts
        zin_ok = (H * h.element_size()) % 16 == 0
        if zin_ok:
            # materialise x_i * x_j once: layer-1 forward and its weight-gradient then
            # stream a plain operand with global_load_lds
            zin = self._buf("Zin", (R2, H), dt)
            K.hadamard_rows(h, ia, h, ib, zin)
            A0 = K.operand(zin)
        else:
            A0 = K.operand(h, ia, h, ib)
        A = A0
        fused = False
        for l, lin in enumerate(self.prd):
            out = self._buf(f"Z{l}", (R2, lin.out_f), dt)
            last = l == len(self.prd) - 1
            if last and self._fusable(lin.in_f, lin.out_f, p_drop) and (A0 is not A or zin_ok):
                # last hidden layer + Linear(H,1) head in one GEMM (partials per 256 columns)
                parts = K.head_parts(lin.out_f)
                hpart = self._buf("hpart", (parts, R2), torch.float32)
                if dt == torch.float32:   # the persistent f32 kernel's head epilogue (no dropout)
                    K.gemm_nt_head_f32(A, K.operand(lin.Wcomp), R2, lin.out_f, lin.in_f, out,
                                       self.head.weight.data.view(-1), hpart, bias=lin.b)
                else:
                    K.gemm_nt_head(A, K.operand(lin.Wcomp), R2, lin.out_f, lin.in_f, out,
                                   self.head.weight.data.view(-1), hpart, bias=lin.b, act=K.ACT_RELU,
                                   dropout=self._dropout(p_drop, DROP_PREDICTOR, l))
                if defer_head:
                    self._s_head = K.head_in(hpart, parts, R2, self.head.bias.data)
                else:
                    K.head_finish(parts, R2, hpart, self.head.bias.data, logit=logit)
                fused = True
            else:
                zm = self._mask(f"Zm{l}", R2, lin.out_f, lin.in_f, self.prd[l + 1].out_f) if not last else None
                K.gemm_nt(A, K.operand(lin.Wcomp), R2, lin.out_f, lin.in_f, out, dc, bias=lin.b, act=K.ACT_RELU,
                          aux=zm, dropout=self._dropout(p_drop, DROP_PREDICTOR, l))
                self._act_mask[id(out)] = zm
            zacts.append(out)
            A = K.operand(out)
        if not fused:
            K.head_fwd(zacts[-1], R2, zacts[-1].shape[1], self.head.weight.data.view(-1), self.head.bias.data,
                       logit=logit)
        return A0, zacts

    def _predictor_backward(self, dlogit, R2, A0, zacts, p_drop):
        """Backward of _predictor_forward from d(loss)/d(logit): the head (dZ of the last
        hidden layer, the head's weight / bias gradients), then per layer the weight-gradient
        (TN) and data-gradient (NT, ReLU-mask epilogue) GEMMs.  The predictor's gradients are
        final after its first layer's weight gradient: their all-reduce starts there.
        (A second HIP stream for the weight gradients measured slower)"""
        dt, dc = self.dtype, self.dc
        if self.predictor_kind != "mlp":
            self._allreduce_tail_begin()
            return None
        alpha = 1.0 / (1.0 - p_drop) if p_drop > 0 else 1.0
        Zl = zacts[-1]
        Hh = Zl.shape[1]
        g = self._buf("gP0", (R2, Hh), dt)
        ws = self._ws("ws_col", K.head_bwd_ws_bytes(R2, max(Hh, 1)))
        K.head_bwd(dlogit, Zl, R2, Hh, self.head.weight.data.view(-1), True, g, self.head.weight.grad.view(-1),
                   self.head.bias.grad, ws, alpha=alpha)
        self._dbg_cut("head backward")
        names = ["gP0", "gP1"]
        k = 0
        for l in range(len(self.prd) - 1, -1, -1):
            lin = self.prd[l]
            gcur = self._buf(names[k % 2], (R2, lin.out_f), dt)
            A_in = K.operand(zacts[l - 1]) if l > 0 else A0
            wsb = K.gemm_tn_ws_bytes(dc, R2, lin.out_f, lin.in_f)
            K.gemm_tn(K.operand(gcur), A_in, R2, lin.out_f, lin.in_f, lin.lin.weight.grad, dc, self._ws("ws_tn", wsb),
                      colsum_a=lin.lin.bias.grad)
            self._dbg_cut(f"predictor weight gradient {l}")
            if l == 0:
                self._allreduce_tail_begin()      # every predictor gradient is final here
            k += 1
            gnext = self._buf(names[k % 2], (R2, lin.in_f), dt)
            if l > 0:
                K.gemm_nt(K.operand(gcur), K.operand(lin.Wt), R2, lin.in_f, lin.out_f, gnext, dc,
                          act=K.ACT_RELU_BWD, aux=self._relu_aux(zacts[l - 1]), alpha=alpha)
            else:
                K.gemm_nt(K.operand(gcur), K.operand(lin.Wt), R2, lin.in_f, lin.out_f, gnext, dc)
        return gnext   # d(loss)/d(h[ia] * h[ib]), the input gradient of the first predictor layer

    def _hadamard_bwd_nodes(self, R, tgt, dZ, drow, h, out, grouped_in=False):
        """d(loss)/dh of the predictor input h[ia] * h[ib] into ``out`` [N, H] (compute dtype, or f32),
        deterministically: the 2R endpoint rows tgt = [ia | ib] are grouped by node
        (llp_dedup_rows2), and one pass per node (llp_hadamard_bwd_segments in the label-row
        layout, B = C = 0) forms each of its rows' gradient dZ[r] * h[partner] as the row
        kernel would store it and sums them in row order (f32) into its row of ``out``
        (drow: the 'inner' predictor's scalar); other rows are 0.  Bit-identical to
        llp_hadamard_bwd_blocks + llp_segment_sum_rows without their [2R, H] row buffer.
        grouped_in: the grouping (``_hadamard_group_nodes`` on the same R, tgt, out) already ran,
        e.g. on the side stream beside the predictor (it needs only the pairs)."""
        N, H = self.N, h.shape[1]
        if not self._grouped_ok(H):
            # rows wider than the grouping kernels take: f32 scatter-add (atomics, so not
            # bit-reproducible), then into ``out`` (possibly a strided slot, another dtype)
            d32 = self._buf("hb_d32", (N, H), torch.float32)
            d32.zero_()
            K.hadamard_bwd_scatter(R, H, dZ, tgt[:R], tgt[R:], h, d32, drow=drow)
            out.copy_(d32)
            return
        if not grouped_in:
            self._hadamard_group_nodes(R, tgt, out)
        R2 = 2 * R
        K.hadamard_bwd_segments(min(R2, N), 0, 0, R, H, self._buf("hb_segp", (R2 + 1,), torch.int32),
                                self._buf("hb_segr", (R2,), torch.int32), tgt, dZ, h, out, None, drow=drow,
                                count=self._buf("hb_nu", (1,), torch.int32),
                                out_rows=self._buf("hb_uniq", (R2,), torch.int32))

    def _hadamard_group_nodes(self, R, tgt, out):
        """The grouping half of ``_hadamard_bwd_nodes``: the 2R endpoint rows tgt = [ia | ib] by
        node (llp_dedup_rows2: unique nodes, segments of rows in row order) and the rows of
        ``out`` that no pair touches zeroed.  Reads only tgt; writes only its own buffers and
        those rows of ``out``."""
        N = self.N
        R2 = 2 * R
        uniq = self._buf("hb_uniq", (R2,), torch.int32)
        pos = self._buf("hb_pos", (R2,), torch.int32)
        n_u = self._buf("hb_nu", (1,), torch.int32)
        seg_ptr = self._buf("hb_segp", (R2 + 1,), torch.int32)
        seg_rows = self._buf("hb_segr", (R2,), torch.int32)
        # the rows of nodes no pair touches are zeroed by the compaction's pass over the nodes
        # (no fill of the whole [N, H] before the per-node sums overwrite nearly all of it)
        rb = out.element_size()
        zfill = (out.dim() == 2 and out.stride(1) == 1 and (out.stride(0) * rb) % 16 == 0
                 and (out.shape[1] * rb) % 16 == 0 and out.data_ptr() % 16 == 0)
        K.dedup_rows2(N, R2, tgt, uniq, pos, n_u, seg_ptr, seg_rows, self._dedup_ws("hb", N, R2),
                      zero_rows=out if zfill else None)
        if not zfill:
            out.zero_()

    def _grouped_ok(self, H):
        """The node-grouped Hadamard-backward kernels (llp_hadamard_bwd_segments,
        llp_segment_sum_rows, llp_hadamard_bwd_blocks with an index) take rows of up to
        256 16-B chunks: H <= 2048 in bf16, <= 1024 in fp32 (the collab sweep's 2048 in
        fp32 takes the row-wise / scatter paths)."""
        return H * (2 if self.dtype == torch.bfloat16 else 4) <= 256 * 16

    def _relu_aux(self, act):
        """What the ReLU-backward GEMM reads for activation ``act``: its bit mask when
        the forward wrote one, else the activations themselves."""
        m = self._act_mask.get(id(act))
        return m if m is not None else act

    def _norm_forward(self, nm, tag, y, out, p_drop, module, layer, rows=None, count=0.0, sync=False, training=True):
        """out = dropout(relu(norm(y))) (src/models.py:49-53 / :114-118).  BatchNorm in
        training: column sums over this call's rows, SUM-all-reduced across ranks when
        ``sync`` (each rank holds a different share of the batch), then normalised by the
        ``count`` rows of the whole batch.  The per-layer statistics stay in buffer
        nstat_<tag> for the backward."""
        M, H = y.shape
        stats = self._buf(f"nstat_{tag}", (2, H if nm.batch else M), torch.float32)
        sums = None
        if nm.batch and training:
            sums = self._buf(f"nsum_{tag}", (2, H), torch.float64)
            K.norm_colsums(y, sums, self._ws("ws_norm", K.norm_ws_bytes(M, H)))
            if sync and self.world > 1:
                self._collective(lambda: dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group))
        m = nm.m
        K.norm_fwd(nm.kind, y, out, stats, nm.gamma(), nm.beta(), nm.eps, training, sums, count, nm.momentum,
                   getattr(m, "running_mean", None), getattr(m, "running_var", None),
                   getattr(m, "num_batches_tracked", None), relu=True,
                   dropout=self._dropout(p_drop, module, layer) if training else None, rows=rows)

    def _norm_backward(self, nm, tag, gout, out, alpha, y, gy, rows=None, count=0.0, sync=False):
        """gy = d(loss)/dy of _norm_forward from gout = d(loss)/dout; gamma / beta gradients
        (this rank's rows) into the module's .grad.  BatchNorm's sum(g), sum(g*xhat) are
        SUM-all-reduced across ranks when ``sync`` before they enter gy."""
        M, H = y.shape
        stats = self._buf(f"nstat_{tag}", (2, H if nm.batch else M), torch.float32)
        sums = self._buf(f"nsumb_{tag}", (2, H), torch.float64)
        m = nm.m
        K.norm_bwd_sums(nm.kind, gout, out, alpha, y, stats, sums, self._ws("ws_norm", K.norm_ws_bytes(M, H)),
                        dgamma=None if m.weight is None else m.weight.grad,
                        dbeta=None if m.bias is None else m.bias.grad, rows=rows)
        if nm.batch and sync and self.world > 1:
            self._collective(lambda: dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group))
        K.norm_bwd(nm.kind, gout, out, alpha, y, stats, gy, nm.gamma(), sums, count, rows=rows)

    def _allreduce_tail_begin(self):
        """Start the SUM all-reduce of the predictor's gradients on RCCL's stream
        (async; it waits for the kernels already queued) so it overlaps the
        Hadamard / student (encoder) backward."""
        self._allreduce_bucket(self._tail_off, self.flat_grad.numel())

    def _allreduce_bucket(self, lo, hi):
        """Start the async SUM all-reduce of flat_grad[lo:hi] once those gradients
        are final (stream order); the rest of flat_grad goes in _finish_allreduce."""
        if self.world > 1 and hi > lo and all(hi <= a or lo >= b for a, b in self._issued):
            self._issued.append((lo, hi))
            self._collective(lambda: self._works.append(
                dist.all_reduce(self.flat_grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)))

    def _grad_slice(self, *params):
        """[lo, hi) of the given parameters' gradients in flat_grad (contiguous)."""
        base = self.flat_grad.data_ptr()
        offs = [((p.grad.data_ptr() - base) // 4, (p.grad.data_ptr() - base) // 4 + p.numel()) for p in params]
        lo, hi = min(o[0] for o in offs), max(o[1] for o in offs)
        assert hi - lo == sum(p.numel() for p in params)
        return lo, hi

    def _finish_allreduce(self, rest):
        """All-reduce the ranges not yet issued (``rest``), then make the stream
        wait for every bucket (stream-ordered: no host block on RCCL)."""
        for lo, hi in rest:
            dist.all_reduce(self.flat_grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
        for w in self._works:
            w.wait()
        self._works = []

    def _collective(self, fn):
        """Run the collective ``fn`` now or, while a multi-rank step is being
        captured (``_seg``), close the current graph segment and replay ``fn``
        eagerly between the segments (RCCL is never inside a hipGraph)."""
        if self._seg is None:
            fn()
        else:
            # a segment cannot end with side-stream work unjoined: join it here (the segments
            # then run it before the collective; the later joins and event waits see it done)
            if self._side_open:
                self._join(self._side)
            self._seg.cut(fn)
            self._cut_gen += 1

    def _dbg_cut(self, what):
        """capture_minibatch(debug_cuts=True): one more segment cut here, whose eager step
        syncs the device and names the stage (locates a faulting segment)."""
        if self._seg is not None and self._seg_debug:
            rank = self.rank

            def fn():
                torch.cuda.synchronize()
                print(f"[rank {rank}] segment ok: {what}", flush=True)
            if self._side_open:
                self._join(self._side)
            self._seg.cut(fn)
            self._cut_gen += 1

    def _allreduce_and_update(self):
        if self.world > 1:
            rest, pos = [], 0
            for lo, hi in sorted(self._issued):
                if lo > pos:
                    rest.append((pos, lo))
                pos = max(pos, hi)
            if pos < self.flat_grad.numel():
                rest.append((pos, self.flat_grad.numel()))
            self._issued = []
            self._collective(lambda: self._finish_allreduce(rest))
        g = self.optimizer.param_groups[0]
        K.grad_sumsq(self.descs_dev, self.n_desc, self.max_numel, self.n_groups, self.sumsq, self.ws_sumsq,
                     ticket=self.sumsq_ticket, n_work=self.n_work_sumsq)
        b1, b2 = g["betas"]
        # the one-launch Adam reads the step counter; the step-end launch advances it
        K.adam_step(self.descs_dev, self.n_desc, self.max_numel, self.sumsq, 1.0, float(g["lr"]), float(b1),
                    float(b2), float(g["eps"]), self.adam_step, fused=True, n_work=self.n_work_adam)

    def _cu_count(self):
        if getattr(self, "_cus", None) is None:
            self._cus = torch.cuda.get_device_properties(self.dev).multi_processor_count
        return self._cus

    def _fork(self, side):
        """The side stream continues from here (stream order of the current stream)."""
        side.wait_stream(torch.cuda.current_stream(self.dev))
        self._side_open = True

    def _join(self, side):
        """The current stream waits for everything forked onto the side stream."""
        if self._side_open:
            torch.cuda.current_stream(self.dev).wait_stream(side)
            self._side_open = False

    def _side_event(self, side):
        """An event at the side stream's current point, waited on by ``_wait_side``."""
        ev = torch.cuda.Event()
        ev.record(side)
        return ev, self._cut_gen

    def _wait_side(self, evg):
        """The current stream waits for the side stream's work up to the event.  Not needed
        (and, in a segmented capture, not legal) once the side stream was joined at a
        collective's segment cut since the event was recorded."""
        ev, gen = evg
        if self._side_open and gen == self._cut_gen:
            torch.cuda.current_stream(self.dev).wait_event(ev)

    def _side_stream(self):
        """The engine's second HIP stream (created once): forks / joins with the current stream
        by events, so a hipGraph capture records the two branches."""
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        return self._side

    # ------------------------------------------------------------------ device state
    def _stateful_workspaces(self):
        """Every workspace whose state persists between calls (dedup, dense negatives)."""
        out = list(self.__dict__.get("_dedup_wss", {}).values())
        out += [w for w in self.__dict__.get("_neg_wss", {}).values() if w is not None]
        return out

    def _device_error_flag(self):
        """0.0 / 1.0 (float64 device scalar): whether a single-pass scan of this engine (the dedup
        compaction, the dense negatives' compaction) timed out in its look-back since the last
        reset.  No host read."""
        words = [w.error_word() for w in self._stateful_workspaces()]
        words = [w for w in words if w is not None]
        if not words:
            return torch.zeros((), dtype=torch.float64, device=self.dev)
        return (torch.stack(words) != 0).any().to(torch.float64)

    def check_device_errors(self, flag=None):
        """Raise if a single-pass scan timed out since the last check: that call's outputs were
        invalid (in bounds, csrc/llp_common.h).  ``flag``: the error flag already reduced over
        the ranks (end_epoch), so that every rank raises and resets together; else this rank's.
        Parameters updated during the failed steps are NOT rolled back."""
        bad = float((self._device_error_flag() if flag is None else flag).item()) != 0.0
        if bad:
            self.reset_device_state()
            raise RuntimeError("a device look-back scan timed out (dedup / dense-negative compaction) on this or "
                               "another rank; the affected steps are invalid and the parameters they updated are "
                               "not rolled back. The engine's persistent device state was reset.")

    def reset_device_state(self):
        """Return every piece of persistent device state to zero: the last-arriver ticket
        blocks of the one-launch loss and gradient norm, and the dedup / dense-negative
        workspaces' state (counts, look-back flags, control and error words).  For use after
        a step raised or a launch aborted part-way, which can leave a ticket or a count
        non-zero; zero is the state every call starts from, so captured graphs stay valid."""
        self.loss_ticket.zero_()
        self.sumsq_ticket.zero_()
        for w in self._stateful_workspaces():
            w.reset()

    def _guarded(self, step):
        """Run one step; if it raises (outside a capture), reset the persistent device state."""
        try:
            return step()
        except Exception:
            # (not KeyboardInterrupt / SystemExit: a synchronize behind a hung kernel or a stalled
            # collective would block Ctrl-C; the next step then starts from whatever state is left,
            # and reset_device_state() is the caller's to run)
            if not torch.cuda.is_current_stream_capturing():
                try:
                    torch.cuda.synchronize(self.dev)
                    self.reset_device_state()
                except Exception:
                    pass
            raise

    # ------------------------------------------------------------------ epoch bookkeeping
    def begin_epoch(self):
        self.loss_sum.zero_()

    def end_epoch(self, total_examples):
        """Returns total_loss / total_examples (src/main.py:141-144); one host sync.  Raises
        if a device scan failed during the epoch (check_device_errors)."""
        # the loss sum and the device-error flag in one buffer: with several ranks one all-reduce
        # carries both, so a scan failure on any rank makes every rank raise (and reset) together
        # instead of leaving the others to hang in the next epoch's collectives
        tot = torch.stack([self.loss_sum.view(()), self._device_error_flag()])
        if self.world > 1:
            dist.all_reduce(tot, group=self.group)
        self.check_device_errors(flag=tot[1])
        steps = int(self.adam_step.item())
        for p in self.all_params:
            self.optimizer.state[p]["step"] = torch.tensor(float(steps))
        return float(tot[0].item()) / max(total_examples, 1)


class DistillEngine(EngineBase):
    """Holds every device buffer of the distillation step.

    Parameters mirror ``train_minibatch``'s arguments (src/main.py:52): the
    student ``model`` (MLP), ``predictor`` (LinkPredictor), the frozen
    ``teacher_predictor`` and teacher embeddings ``t_h``; ``x`` the node
    features; ``row``/``col`` the sampler graph (data.adj_t, src/main.py:56);
    ``optimizer`` a torch.optim.Adam over model+predictor parameters whose
    hyper-parameters and state this engine uses.
    """

    def __init__(self, model, predictor, teacher_predictor, x, t_h, row, col, num_nodes, args, optimizer,
                 dtype="bf16", seed=0, rw_sorted=False, group=None, device=None, dedup=True, shard_student=True,
                 owner_pairs=True, owner_locality=True, sparse_input=True):
        self._init_device(x.device, device, dtype, seed, group, "DistillEngine")
        # run the dropout-free student on unique nodes (step_minibatch); the unique
        # count stays on the device, so this path is hipGraph-capturable too
        self.dedup = bool(dedup)
        # multi-rank full-batch step: each rank runs the student on its slice of the nodes
        # (_fb_shard); rank 0 of 4 on coauthor-physics 0.94 -> 0.81 ms (first
        # table: tools/physics_bench.py --emulate-ranks 4 with and without --replicated)
        self.shard_student = bool(shard_student)
        # multi-rank minibatch step: the owner decomposition (minibatch_owner), node
        # ownership by a locality order of the graph (_owner_table) or by id ranges
        self.owner_pairs = bool(owner_pairs)
        self.owner_locality = bool(owner_locality)
        self._rows_dev = None      # int32 device count of the unique-node student (last step), or None
        self._rows_host = 0
        self.args = args
        self.N = int(num_nodes)
        # Philox streams per step under self.seed: the context sampler's walks 0..rw_step-1 and its
        # negatives rw_step (STREAMS_PER_STEP * step_ctr + offset)
        if not 1 <= int(args.rw_step) <= MAX_RW_STEP:
            raise ValueError(f"rw_step={args.rw_step}: the context sampler has {MAX_RW_STEP + 1} Philox streams per "
                             f"step (1 <= rw_step <= {MAX_RW_STEP})")

        # ---------------- parameters
        self.model, self.predictor, self.tpred = model, predictor, teacher_predictor
        stu = list(model.layers)
        # bag-of-words inputs (coauthor-physics: 8,415 binary keywords, ~0.5 % nonzero): the full-batch
        # student's first layer gathers rows of its transposed bf16 weight by x's nonzeros
        # (llp_spmm_rows / llp_spmm_tn, csrc/spmm.hip) instead of dense MFMA tiles over zeros
        H0 = stu[0].out_features
        self.sparse_x = (bool(sparse_input) and self.dtype in (torch.bfloat16, torch.float32) and x.dim() == 2
                         and x.shape[1] >= 256
                         and H0 % 8 == 0 and H0 <= 1024
                         and float(torch.count_nonzero(x)) <= SPARSE_X_MAX_DENSITY * x.numel())
        self.stu = [_Linear(l, self.dtype, need_t=(i > 0 or self.sparse_x), need_c=True) for i, l in enumerate(stu)]
        # bf16: the input width is zero-padded to a multiple of 64 (x and the first layer's compute
        # copy) so that the first layer runs on the 256-tile MFMA kernels (cora 1,433 -> 1,472,
        # coauthor-physics 8,415 -> 8,448, ...); padded columns are 0 in both, the products exact
        F_in = self.stu[0].in_f
        self.F_pad = -(-F_in // 64) * 64 if (self.dtype == torch.bfloat16 and F_in % 64) else F_in
        if self.F_pad != F_in:
            l0 = self.stu[0]
            l0.Wc = torch.zeros(l0.out_f, self.F_pad, dtype=self.dtype, device=l0.W.device)
            l0.k_in = self.F_pad
        for l in self.stu:
            self._set_shadow(l.lin.weight, l.Wc, l.Wt, l.k_in if l.Wc is not None else 0)
        # norm_type 'layer' / 'batch' (src/models.py:27-37): a norm after every hidden layer, its
        # parameters after the Linear ones, as in model.parameters()
        self.stu_norms = _norms_of(model, len(stu) - 1, self.stu[0].out_f if len(stu) > 1 else 0)
        stu_params = [p for l in stu for p in (l.weight, l.bias)] + [p for n in self.stu_norms for p in n.params]
        prd_params = self._setup_predictor(predictor, args.predictor)
        self._init_params(stu_params + prd_params, [0] * len(stu_params) + [1] * len(prd_params), optimizer)

        # teacher predictor (frozen; dropout stays live as in the reference, Q3)
        tl = list(teacher_predictor.lins)
        self.t_kind = teacher_predictor.predictor
        self.t_hidden = []
        for l in tl[:-1]:
            W = l.weight.data.to(self.dev)
            self.t_hidden.append((W.to(self.dtype).contiguous(), l.bias.data.to(self.dev).float().contiguous()))
        self.t_head = (tl[-1].weight.data.to(self.dev).float().reshape(-1).contiguous(),
                       tl[-1].bias.data.to(self.dev).float().contiguous())
        self.t_dropout = float(getattr(teacher_predictor, "dropout", 0.0)) if teacher_predictor.training else 0.0

        # ---------------- data
        if self.F_pad != F_in:
            self.x = torch.zeros(self.N, self.F_pad, dtype=self.dtype, device=self.dev)
            self.x[:, :F_in].copy_(x.to(self.dev))
        else:
            self.x = x.to(self.dev).to(self.dtype).contiguous()
        self.xs = K.SparseRows(x.to(self.dev), round_bf16=self.dtype == torch.bfloat16) if self.sparse_x else None
        self.t_h = t_h.to(self.dev).to(self.dtype).contiguous()
        self._neg_rc = (np.asarray(row), np.asarray(col))
        self._neg_keys = None
        rowptr, colv = build_sampler_csr(np.asarray(row), np.asarray(col), self.N, rw_sorted)
        self.rowptr = torch.from_numpy(rowptr).to(self.dev)
        self.col = torch.from_numpy(colv).to(self.dev)

        self._build_descs()

    # ------------------------------------------------------------------ helpers
    @property
    def last_student_rows(self):
        """Student rows of the last minibatch step: the unique-node count (a
        device read, so it synchronises) or the row-wise R1."""
        if self._rows_dev is not None:
            return int(self._rows_dev.item())
        return self._rows_host

    def last_logits(self):
        """The last single-rank step's predictor outputs, as the reference names them
        (src/main.py:105-106,126 / 186-187,213): ``s_r`` [B, C] student context-pair probabilities,
        ``t_r`` [B, C] the frozen teacher's, ``out`` [n_lab] label-pair probabilities, plus the
        student's pre-sigmoid logits ``s_logit`` / ``out_logit`` (f32 device views of the step's
        buffers, valid until the next step).  The loss launch finishes every logit from the head
        partials and writes it back, so these are exactly what the loss terms were computed on."""
        lay = getattr(self, "_logit_layout", None)
        if lay is None:
            raise RuntimeError("last_logits: no single-rank step has run (the owner decomposition keeps each "
                               "rank's pairs in its own order)")
        B, C, n_lab = lay
        logit = self._bufs["logit"][:B * C + n_lab]
        s_logit, out_logit = logit[:B * C].view(B, C), logit[B * C:]
        t_r = self._bufs["t_r"][:B * C].view(B, C) if B * C else self._bufs["logit"][:0].view(0, C)
        return dict(s_r=torch.sigmoid(s_logit), t_r=t_r, out=torch.sigmoid(out_logit), s_logit=s_logit,
                    out_logit=out_logit)

    def _rows_index(self, B, C, P2):
        """Predictor-row -> h-row index for the minibatch layout (static per shape)."""
        key = ("rows", B, C, P2)
        if key not in self._bufs:
            C1 = C + 1
            b = torch.arange(B, device=self.dev, dtype=torch.int64).repeat_interleave(C)
            c = torch.arange(C, device=self.dev, dtype=torch.int64).repeat(B)
            ia_ctx = b * C1
            ib_ctx = b * C1 + 1 + c
            lab = torch.arange(P2, device=self.dev, dtype=torch.int64)
            ia_lab = B * C1 + lab
            ib_lab = B * C1 + P2 + lab
            iab = torch.stack([torch.cat([ia_ctx, ia_lab]), torch.cat([ib_ctx, ib_lab])]).to(torch.int32).contiguous()
            self._bufs[key] = (iab[0], iab[1], iab)
        return self._bufs[key][:2]

    def _rows_index_flat(self, B, C, P2):
        """_rows_index's two arrays as one contiguous [2 * R2] index (one gather launch)."""
        self._rows_index(B, C, P2)
        return self._bufs[("rows", B, C, P2)][2].view(-1)

    # ------------------------------------------------------------------ the step
    @property
    def minibatch_owner(self):
        """Whether step_minibatch runs the owner decomposition: several ranks
        (or ``emulate_pairs``), ``owner_pairs`` on, and the unique-node student (no dropout,
        no BatchNorm, rows the grouping kernels take).  Callers then pass the WHOLE batch on
        every rank; otherwise each rank passes its slice with offsets."""
        if not self.owner_pairs or (self.world <= 1 and self.emulate_pairs is None):
            return False
        return self._dedup_ok()

    def _dedup_ok(self):
        """The unique-node student applies: without dropout the student is row-wise, so
        duplicate rows of x[this_target] give identical activations (BatchNorm's statistics
        run over every row, duplicates included, so it keeps the row-wise student)."""
        return (self.dedup and float(self.args.dropout) == 0.0 and self._grouped_ok(self.stu[-1].out_f)
                and not self._batch_norm)

    def _owner_rank(self):
        if self.world > 1:
            return self.rank, self.world
        return self.emulate_pairs

    @_resets_on_error
    def step_minibatch(self, anchors, link_ids, pairs, b_offset=0, p_offset=0, B_total=None, P_total=None,
                       samples=None, neg=None, kernel_events=None, dense_negatives=False):
        """One link batch of train_minibatch (src/main.py:73-143).

        anchors  int32[B]   this rank's slice of node_perm (src/main.py:76)
        link_ids int32[P]   this rank's slice of link_perm (src/main.py:73,78)
        pairs    int32[E,2] pos_train_edge (src/main.py:55)
        samples / neg: optional injected samples int32[B, 1+C] / negatives int32[2, n]
        (parity tests); otherwise drawn on the device: randint (collab,
        src/main.py:83-84) or, with dense_negatives, PyG dense sampling
        (non-collab, src/main.py:80-82; one host read of its count).
        With ``minibatch_owner`` (several ranks) anchors / link_ids / samples / neg are the
        WHOLE batch on every rank (no offsets): every rank draws the same samples, and
        llp_pair_owner_assign gives each predictor pair to one rank.
        Returns nothing; the loss terms stay on the device (self.terms).
        """
        self._act_mask.clear()
        a = self.args
        B = int(anchors.numel())
        P = int(link_ids.numel())
        owner = self.minibatch_owner
        if owner and (b_offset or p_offset or B_total not in (None, B) or P_total not in (None, P)):
            raise ValueError("step_minibatch: the owner decomposition takes the whole batch on every rank "
                             "(no offsets / totals); see DistillEngine.minibatch_owner")
        B_total = B if B_total is None else int(B_total)
        P_total = P if P_total is None else int(P_total)
        rw_step, hops, ns_rate = int(a.rw_step), int(a.hops), int(a.ns_rate)
        C = rw_step * hops * (1 + ns_rate)
        C1 = C + 1
        H = self.stu[-1].out_f
        dt, dc = self.dtype, self.dc

        # ---- a1-a3: negatives and samples (src/main.py:80-84,93); ``target`` = this_target
        # (src/main.py:95): samples.flat | src | dst
        samp = self._buf("samples", (B, C1), torch.int32)
        t_ia = t_ib = None
        if not owner:
            t_ia = self._buf("t_ia", (B * C,), torch.int32)
            t_ib = self._buf("t_ib", (B * C,), torch.int32)
        if samples is None and neg is None and not dense_negatives:
            # collab path: walks, context negatives, randint label negatives, the student's
            # target rows and the teacher's pair index in one launch (llp_minibatch_sample)
            negb, n_neg, n_neg_total = self._buf("neg", (2, max(P, 1)), torch.int32), P, P_total
            target = self._buf("target", (B * C1 + 4 * P,), torch.int32)
            K.minibatch_sample(self.rowptr, self.col, self.N, anchors, B, a.ps_method, rw_step, hops, ns_rate,
                               self.seed, self.step_ctr, 0, pairs, link_ids, P, P_total, p_offset, RANDINT_STREAM,
                               samp, negb, target, t_ia, t_ib, b_offset=b_offset)
            self._dbg_cut("sample")
        else:
            negb, n_neg, n_neg_total, _ = self._negatives(P, P_total, p_offset, neg, dense_negatives)
            if samples is not None:
                samp.copy_(samples.to(torch.int32))
            else:
                K.context_sampler(self.rowptr, self.col, self.N, anchors, B, a.ps_method, rw_step, hops, ns_rate,
                                  self.seed, self.step_ctr, 0, samp, b_offset=b_offset)
            target = self._buf("target", (B * C1 + 2 * (P + n_neg),), torch.int32)
            K.build_targets(B, C1, samp, pairs, link_ids, None, 0, P, negb, target, n_neg=n_neg)
            if not owner:
                K.pair_index_from_samples(B, C, samp, t_ia, t_ib)
        n_lab = P + n_neg                      # train_edges columns (src/main.py:86)
        p_drop = float(a.dropout)

        if owner:
            # ---- the owner decomposition: this rank's context pairs (by the context node's owner)
            # and label pairs (by the source's owner); the student rows are their ends [ia | ib]
            rank, world = self._owner_rank()
            own = self._owner_assign(B, C, C1, P, n_neg, target, rank, world)
            R2, n_ctx, n_pos = own["R2"], own["ctx"], own["pos"]
            n_lab_loc = R2 - n_ctx
            target = own["rows"]
            R1 = 2 * R2
        else:
            R1 = B * C1 + 2 * n_lab
            R2 = B * C + n_lab
            n_ctx, n_pos, n_lab_loc = B * C, P, n_lab
            ia, ib = self._rows_index(B, C, n_lab)

        # ---- unique-node compaction: run the student on the U distinct nodes of the rows
        # and sum each node's row gradients (_dedup_ok)
        dedup = self._dedup_ok()
        n_u = None
        if dedup:
            fresh = "uniq" not in self._bufs or self._bufs["uniq"].numel() < R1
            uniq = self._buf("uniq", (R1,), torch.int32)
            if fresh:   # slots past the live count are read (never used) by the q64 GEMM prologue: keep them ids
                uniq.zero_()
            pos = self._buf("pos", (R1,), torch.int32)
            n_u = self._buf("n_unique", (1,), torch.int32)
            seg_ptr = self._buf("seg_ptr", (R1 + 1,), torch.int32)
            seg_rows = self._buf("seg_rows", (R1,), torch.int32)
            K.dedup_rows2(self.N, R1, target, uniq, pos, n_u, seg_ptr, seg_rows, self._dedup_ws("mb", self.N, R1))
            self._dbg_cut("sample + dedup")
            if owner:   # the rows ARE the pairs' ends: row k and row R2 + k
                ia_h, ib_h = pos[:R2], pos[R2:R1]
            else:
                iab_h = self._buf("iab_u", (2, R2), torch.int32)   # both pair sides in one gather
                K.gather_i32(self._rows_index_flat(B, C, n_lab), pos, iab_h.view(-1))
                ia_h, ib_h = iab_h[0], iab_h[1]
            # No host read of U: the student kernels are launched for the bound
            # min(R1, N) and run on the *n_unique live rows (llp_operand.rows_dev),
            # so the step stays asynchronous and hipGraph-capturable.
            rows_s, gather_s = min(R1, self.N), uniq
        else:
            rows_s, gather_s, ia_h, ib_h = R1, target, ia, ib
        self._rows_dev = n_u
        self._rows_host = rows_s

        t_r = self._buf("t_r", (max(n_ctx, 1),), torch.float32)[:n_ctx]
        if owner:
            # ---- a6 first (src/main.py:104,106): the frozen teacher's probabilities depend only on
            # the sampled pairs, so their grid slice is reduce-scattered under the student forward
            # (beside the unique-node compaction on the side stream it measured 1 % slower, §4.5)
            self._teacher_forward(n_ctx, target[:n_ctx], target[R2:R2 + n_ctx], t_r)
            t_slice = self._owner_grid_scatter("t", B, C, world, rank, own, None, t_r, n_ctx)

        # ---- a4: student MLP over the gathered rows (src/main.py:95-96)
        R1_total = B_total * C1 + 2 * (P_total + n_neg_total)    # this_target rows of the whole batch
        acts, x_rows = self._student_forward(rows_s, gather_s, n_u, p_drop, R1_total, kernel_events)
        h = acts[-1]

        # ---- a5: predictor on context pairs + label pairs (src/main.py:103-105,126)
        logit = self._buf("logit", (R2,), torch.float32)
        self._dbg_cut("student forward")
        # (one rank: the heads' finish is left to the loss launch; the owner decomposition
        # all-reduces the logits first)
        A0, zacts = self._predictor_forward(h, ia_h, ib_h, R2, logit, p_drop, defer_head=not owner)
        self._dbg_cut("predictor forward")

        # ---- a6: frozen teacher predictor on the same context pairs (src/main.py:104,106)
        if not owner:
            self._teacher_forward(B * C, t_ia, t_ib, t_r, defer_head=True)

        # ---- a7-a9: fused LLP_D + LLP_R + BCE and d(loss)/d(logit) (src/main.py:107-130)
        if not (a.LLP_D or a.LLP_R):
            raise UnboundLocalError("train_minibatch: loss is only defined when LLP_D or LLP_R is set "
                                    "(src/main.py:129-130)")
        dlogit = self._buf("dlogit", (R2,), torch.float32)
        ws = self._ws("ws_loss", K.llp_loss_ws_bytes(B, n_lab_loc))
        if owner:
            # every anchor's KL / rank needs all C of its logits.  The [B, C] grid of context logits
            # (this rank's pairs scattered in, zeros elsewhere) is reduce-scattered by anchor slices
            # of Bc = ceil(B / W) anchors, each rank evaluates the KL / rank loss of ITS slice (and
            # the BCE of its label pairs), and the slices' d(logit) are all-gathered back, from
            # which each rank takes its own pairs' entries.  The teacher's grid went the same way
            # before the student forward (t_slice above).  Per step: 2 x 1.9 MB reduce-scatter and
            # 1.9 MB all-gather at the collab shape, against one 3.8 MB all-reduce and the loss of
            # all B anchors on every rank in round 4
            lo = own["ctx_lo"]
            Bc = -(-B // world)
            B_loc = max(0, min(Bc, B - rank * Bc))
            s_slice = self._owner_grid_scatter("s", B, C, world, rank, own, logit, None, n_ctx)
            dslice = self._buf("owner_dslice", (Bc * C,), torch.float32)
            K.llp_loss(B_loc, C, s_slice, t_slice, n_lab_loc, n_pos, logit[n_ctx:], B, P + n_neg, float(a.margin),
                       1.0, float(a.True_label), float(a.LLP_D), float(a.LLP_R), dslice, dlogit[n_ctx:], self.terms,
                       ws, ticket=self.loss_ticket)
            dfull = self._buf("owner_dfull", (world * Bc * C,), torch.float32)
            self._collective(lambda: self._all_gather_rows(dfull, dslice, world, rank))
            K.gather_i32(own["sel"][lo:lo + n_ctx], dfull.view(torch.int32), dlogit[:n_ctx].view(torch.int32))
        else:
            K.llp_loss(B, C, logit, t_r, n_lab, P, logit[B * C:], B_total, P_total + n_neg_total, float(a.margin),
                       1.0, float(a.True_label), float(a.LLP_D), float(a.LLP_R), dlogit, dlogit[B * C:], self.terms,
                       ws, s_head=self._s_head, t_head=self._t_head, ticket=self.loss_ticket)

        self._logit_layout = None if owner else (B, C, n_lab)

        # ---- a10: backward
        self._dbg_cut("teacher + loss")
        dZ0 = self._predictor_backward(dlogit, R2, A0, zacts, p_drop)
        mlp = self.predictor_kind == "mlp"
        if dedup:
            # Hadamard backward reduced straight onto the unique nodes (no [R1, H] row gradients);
            # the owner layout is label rows only (B = C = 0: rows k and R2 + k are pair k's ends)
            dh = self._buf("gS0", (rows_s, H), dt)
            Bl, Cl = (0, 0) if owner else (B, C)
            arow = None if owner else self._buf("anchor_rows", (max(B, 1), H), dt)
            K.hadamard_bwd_segments(rows_s, Bl, Cl, R2 if owner else n_lab, H, seg_ptr, seg_rows, pos,
                                    dZ0 if mlp else None, h, dh, arow, drow=None if mlp else dlogit, count=n_u)
        else:
            dh = self._buf("gS0", (R1, H), dt)
            K.hadamard_bwd_blocks(B, C, n_lab, H, dZ0 if mlp else None, h, dh, drow=None if mlp else dlogit)
        self._student_backward(dh, rows_s, gather_s, acts, p_drop, count=n_u, x_rows=x_rows, norm_count=R1_total,
                               norm_sync=True)
        self._allreduce_and_update()
        K.step_end(self.terms[:1], float(P_total), self.loss_sum, self.step_ctr, adam_step=self.adam_step)

    def _owner_assign(self, B, C, C1, P, n_neg, target, rank, world):
        """This rank's pairs under the owner decomposition (llp_pair_owner_assign): categories
        context pairs (b, c) keyed by the context node, positive and negative label pairs
        keyed by their source; ``target`` is the whole batch's this_target (samples.flat |
        src | dst).  Returns the rank's [ia | ib] rows, its counts, sel / gpos."""
        n_lab = P + n_neg
        BC1 = B * C1
        ns = (B * C, P, n_neg)
        caps = [(rank + 1) * n // world - rank * n // world for n in ns]
        R2 = sum(caps)
        cats = [K.owner_cat(B * C, target, target, (C, C1, 0, 0), (C, C1, 1, 1), key_b=True),
                K.owner_cat(P, target[BC1:], target[BC1 + n_lab:]),
                K.owner_cat(n_neg, target[BC1 + P:], target[BC1 + n_lab + P:])]
        n_all = sum(ns)
        sel = self._buf("owner_sel", (max(n_all, 1),), torch.int32)
        gpos = self._buf("owner_gpos", (max(n_all, 1),), torch.int32)
        rows = self._buf("owner_rows", (max(2 * R2, 1),), torch.int32)[:2 * R2]
        ws = self._buf("owner_ws", (K.pair_owner_ws_bytes(ns, world) // 4 + 16,), torch.int32)
        K.pair_owner_assign(cats, self.N, world, rank, sel, ws, gpos=gpos, target=rows, R2=R2,
                            owner_tab=self._owner_table(world))
        return {"R2": R2, "ctx": caps[0], "pos": caps[1], "neg": caps[2], "rows": rows, "sel": sel,
                "gpos": gpos, "ctx_lo": rank * ns[0] // world}

    def _owner_grid_scatter(self, which, B, C, world, rank, own, s_loc, t_loc, n_ctx):
        """This rank's context-pair values (student logits ``s_loc`` or teacher probabilities
        ``t_loc``) scattered into the [world * Bc, C] grid of the whole batch (zeros elsewhere;
        Bc = ceil(B / world), the padded tail stays zero), then reduce-scattered: returns this
        rank's [Bc * C] slice (anchors [rank * Bc, ...)), the SUM over ranks, which is exact as
        each entry has one owner.  The teacher's ("t") is issued asynchronously on RCCL's stream
        and waited for by the student's ("s"), so it runs under the student forward."""
        Bc = -(-B // world)
        key = ("owner_grid", which, world * Bc * C)
        if key not in self._bufs:       # zero once: the scatter writes [0, B*C) every step
            self._bufs[key] = torch.zeros(world * Bc * C, dtype=torch.float32, device=self.dev)
        full = self._bufs[key]
        lo = own["ctx_lo"]
        K.pair_owner_scatter(B * C, own["gpos"], lo, lo + n_ctx, s_loc, t_loc, full if s_loc is not None else None,
                             full if t_loc is not None else None)
        part = self._buf(f"owner_{which}slice", (Bc * C,), torch.float32)

        def rs():
            if which == "t" and self.world > 1 and dist.get_backend(self.group) == "nccl":
                self._owner_work = dist.reduce_scatter_tensor(part, full, op=dist.ReduceOp.SUM, group=self.group,
                                                              async_op=True)
                return
            self._reduce_scatter_rows(part, full, world, rank)
            if which == "s" and getattr(self, "_owner_work", None) is not None:
                self._owner_work.wait()          # the teacher's slice (stream-ordered, no host block)
                self._owner_work = None
        self._collective(rs)
        return part

    def _owner_table(self, world):
        """Node -> owner rank for the owner decomposition (``owner_locality``): contiguous ranges
        of a locality order of the sampler graph (llp_sage.locality_order, label propagation),
        so a positive label pair's two ends and a walk's contexts mostly have one owner and a
        rank's pairs reach fewer foreign nodes; None: contiguous ranges of node ids.  Host
        work once per engine (the same on every rank: deterministic)."""
        if not self.owner_locality:
            return None
        key = ("owner_tab", int(world))
        if key not in self._bufs:
            if getattr(self, "_locality_pi", None) is None:
                import llp_sage
                r, c = self._neg_rc
                self._locality_pi = llp_sage.locality_order(np.stack([np.asarray(r), np.asarray(c)]), self.N)[1]
            tab = (self._locality_pi * int(world)) // self.N
            self._bufs[key] = torch.from_numpy(tab.astype(np.int32)).to(self.dev)
        return self._bufs[key]

    def _student_forward(self, rows_s, gather_s, n_u, p_drop, R1_total, kernel_events=None):
        """Student MLP over x[gather_s] (src/models.py:45-54), rows_s rows (n_u: device row
        count of the unique-node student).  x[gather_s] is gathered once into a plain
        buffer that the first layer's forward and weight-gradient GEMMs read (plain operands
        take the LDS-DMA kernels, in fp32 too: §4.8).  Returns (activations per layer, the
        gathered x rows)."""
        dt, dc = self.dtype, self.dc
        acts = []
        x_rows = self._buf("Xg", (rows_s, self.x.shape[1]), dt)
        K.gather_rows(self.x, gather_s, x_rows, count=n_u)
        A = K.operand(x_rows, count=n_u)
        for l, lin in enumerate(self.stu):
            last = l == len(self.stu) - 1
            out = self._buf(f"H{l}", (rows_s, lin.out_f), dt)
            timed = kernel_events is not None and l == 1
            if timed:   # the dominant MFMA kernel, timed on the launch stream (bench.py roofline)
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            if not last and self.stu_norms:
                # Linear, then norm + ReLU + dropout (src/models.py:48-53)
                y = self._buf(f"Y{l}", (rows_s, lin.out_f), dt)
                K.gemm_nt(A, K.operand(lin.Wcomp), rows_s, lin.out_f, lin.k_in, y, dc, bias=lin.b)
                self._norm_forward(self.stu_norms[l], f"s{l}", y, out, p_drop, DROP_ENCODER, l, rows=n_u,
                                   count=R1_total, sync=True)
                self._act_mask[id(out)] = None
            else:
                hm = None if last else self._mask(f"Hm{l}", rows_s, lin.out_f, lin.k_in, self.stu[l + 1].out_f)
                self._act_mask[id(out)] = hm
                K.gemm_nt(A, K.operand(lin.Wcomp), rows_s, lin.out_f, lin.k_in, out, dc, bias=lin.b,
                          act=K.ACT_NONE if last else K.ACT_RELU, aux=hm,
                          dropout=None if last else self._dropout(p_drop, DROP_ENCODER, l))
            if timed:
                ev[1].record()
                kernel_events.append(ev)
                self.timed_kernel = K.last_gemm_kernel()
            acts.append(out)
            A = K.operand(out, count=n_u)
        return acts, x_rows

    @property
    def _batch_norm(self):
        return any(n.batch for n in self.stu_norms)

    # ------------------------------------------------------------------ full-batch step
    @_resets_on_error
    def step_fullbatch(self, anchors, link_ids, pairs, b_offset=0, p_offset=0, B_total=None, P_total=None,
                       samples=None, neg=None, dense_negatives=True):
        """One link batch of ``train`` (src/main.py:167-235): the student MLP runs
        over all N nodes (src/main.py:173), the predictor over h[samples] context
        pairs and h[train_edges] label pairs, plus KD_RM / KD_LM.

        anchors  int32[B]  this rank's slice of node_perm (src/main.py:169)
        link_ids int32[P]  this rank's slice of link_perm
        pairs    int32[E,2] pos_train_edge (data.edge_index.t() for production, src/main.py:153)
        dense_negatives: PyG dense negative sampling (non-collab, src/main.py:205-207)
            else torch.randint pairs (collab, src/main.py:208-209).
        neg      optional injected negatives int32[2, n_neg] (parity tests).
        Returns the number of negatives: a host int for injected / randint ones (and
        with KD_LM, whose kernel reads the dense count on the host), else the whole
        batch's PyG-dense count as an int32 device tensor: that path has no host
        sync, and capture_fullbatch records it as a hipGraph."""
        self._act_mask.clear()
        a = self.args
        B = int(anchors.numel())
        P = int(link_ids.numel())
        B_total = B if B_total is None else int(B_total)
        P_total = P if P_total is None else int(P_total)
        use_llp = bool(a.LLP_D or a.LLP_R)
        rw_step, hops, ns_rate = int(a.rw_step), int(a.hops), int(a.ns_rate)
        C = rw_step * hops * (1 + ns_rate)
        C1 = C + 1
        Bc = B if use_llp else 0
        N = self.N
        H = self.stu[-1].out_f
        dt, dc = self.dtype, self.dc
        p_drop = float(a.dropout)

        # ---- samples (src/main.py:180-183)
        def sample():
            if not use_llp:
                return None
            samp = self._buf("samples", (B, C1), torch.int32)
            if samples is not None:
                samp.copy_(samples.to(torch.int32))
            else:
                K.context_sampler(self.rowptr, self.col, N, anchors, B, a.ps_method, rw_step, hops, ns_rate,
                                  self.seed, self.step_ctr, 0, samp, b_offset=b_offset)
            return samp
        # ---- negatives (src/main.py:205-209) and the pair index.  PyG-dense ones keep their count on
        # the device (label slots past it inert, no host read, so the step is graph-capturable) unless
        # KD_LM, whose kernel takes the host count, needs it.  Without a host read they run on a side
        # stream beside the student forward (overlap_streams): both are small launches on this path
        # (the physics student at rank 0 of 4: 31-tile GEMMs), so the GPU has room for both
        w_rm, w_lm = float(a.KD_RM), float(a.KD_LM)
        BC = Bc * C
        side = self._side_stream() if (self.overlap_streams and dense_negatives and neg is None and w_lm == 0.0) \
            else None
        side_samp = side is not None and self.side_sampling
        samp = None if side_samp else sample()      # (with the side stream: sampled there, first)

        def negatives_and_pairs():
            negb, n_neg, n_neg_total, cnt = self._negatives(P, P_total, p_offset, neg, dense_negatives,
                                                            device_count=w_lm == 0.0)
            R2 = BC + P + n_neg
            ia_ib = self._buf("fb_iab", (max(2 * R2, 1),), torch.int32)[:2 * R2]   # [ia | ib]: endpoint rows
            K.fullbatch_pairs(Bc, C1, samp, pairs, link_ids, P, negb if n_neg > 0 else None, n_neg, ia_ib[:R2],
                              ia_ib[R2:], neg_count=cnt, neg_offset=p_offset)
            return n_neg, n_neg_total, cnt, R2, ia_ib

        # d(loss)/dh: without KD_RM, the pair rows' Hadamard gradients are grouped by node and
        # summed in row order (deterministic, straight into the compute-dtype buffer); with KD_RM
        # (which adds at the anchors) they accumulate by f32 scatter-add, then convert
        grouped = w_rm == 0.0 and self._grouped_ok(H)
        shard = self._fb_shard(p_drop, grouped)
        r0, n_rows, n_loc, s_world, s_rank = (0, N, N, 1, 0) if shard is None else shard
        R_t_of = (lambda R2: R2 if w_lm != 0.0 else BC)
        t_r = None
        ev_t = None

        def pair_work(R2, ia_ib, dh_out):
            """a6 (the frozen teacher on the context pairs, src/main.py:187) and the node grouping of
            the Hadamard backward: both need only the pairs.  On the side stream the loss waits for
            the teacher (event ev_t) and the backward for the grouping (the stream's end)."""
            nonlocal t_r, ev_t
            R_t = R_t_of(R2)
            t_r = self._buf("t_r", (max(R_t, 1),), torch.float32)
            self._t_head = None
            if R_t > 0:
                self._teacher_forward(R_t, ia_ib[:R_t], ia_ib[R2:R2 + R_t], t_r, defer_head=R_t == BC)
                if grouped and self.side_grouping:
                    ev_t = self._side_event(side)
            if grouped and self.side_grouping:
                self._hadamard_group_nodes(R2, ia_ib, dh_out)
            return self._t_head

        def dh_target():   # where the per-node sums go: this rank's f32 rows of all nodes, or dh itself
            return (self._buf("fb_dhfull", (s_world * n_loc, H), torch.float32)[:N] if shard is not None
                    else self._buf("gS0", (N, H), dt))

        main = torch.cuda.current_stream(self.dev)
        # without a row-sharded student (no collective before the backward) the teacher and the
        # grouping follow the pairs on the side stream at once, beside the student forward; with
        # one, they start after the all-gather (the streams are joined before a collective)
        early = side is not None and shard is None and self.early_pair_work
        ev_pairs = None
        if side is not None:
            # the samples, the negatives and the pairs need only the step's inputs: on the side
            # stream from the step's start, while the main stream runs the student forward
            self._fork(side)
            with torch.cuda.stream(side):
                if side_samp:
                    samp = sample()
                neg_res = negatives_and_pairs()
                if early:
                    ev_pairs = self._side_event(side)
                    t_head_early = pair_work(neg_res[3], neg_res[4], dh_target() if grouped else None)

        # ---- a4: student MLP over all nodes (src/main.py:173), queued before the dense negatives'
        # count is read back (one host sync), so the GPU runs it while the host waits; at several ranks each rank
        # runs it on its own slice of the nodes and the slices are all-gathered (_fb_shard)
        x_loc = self.x if shard is None else self.x[r0:r0 + n_rows]
        acts = []
        A = K.operand(x_loc)
        for l, lin in enumerate(self.stu):
            last = l == len(self.stu) - 1
            out = self._buf(f"H{l}", (n_loc, lin.out_f), dt)
            hm = None if last else self._mask(f"Hm{l}", n_rows, lin.out_f, lin.k_in, self.stu[l + 1].out_f)
            self._act_mask[id(out)] = hm
            act = K.ACT_NONE if last else K.ACT_RELU
            normed = not last and bool(self.stu_norms)
            if normed:   # Linear, then norm + ReLU + dropout (src/models.py:48-53)
                hm, act = None, K.ACT_NONE
                self._act_mask[id(out)] = None
                dst = self._buf(f"Y{l}", (n_loc, lin.out_f), dt)
            else:
                dst = out
            sparse = l == 0 and self.xs is not None and (p_drop == 0.0 or normed)
            splits = self._splitk_plan(n_rows, lin.out_f, lin.k_in) if (p_drop == 0.0 or normed) and not sparse else 1
            if sparse:       # bag-of-words x: gather W^T rows by its nonzeros (no dropout here)
                K.spmm_rows(self.xs, n_rows, r0, lin.Wt, lin.b, dst, act=act, mask=hm)
            elif splits > 1:   # few output tiles over a long K (the first layer at 8,448 features)
                ws = self._ws("ws_splitk", K.gemm_nt_splitk_ws_bytes(n_rows, lin.out_f, splits))
                K.gemm_nt_splitk(A, K.operand(lin.Wcomp), n_rows, lin.out_f, lin.k_in, dst, splits, ws, bias=lin.b,
                                 act=act, mask=hm)
            else:
                K.gemm_nt(A, K.operand(lin.Wcomp), n_rows, lin.out_f, lin.k_in, dst, dc, bias=lin.b, act=act, aux=hm,
                          dropout=None if (last or normed) else self._dropout(p_drop, DROP_ENCODER, l))
            if normed:
                # the student is replicated (or row-sharded, LayerNorm only) over the ranks: BatchNorm's
                # statistics are over all N nodes on every rank, no exchange
                self._norm_forward(self.stu_norms[l], f"s{l}", dst[:n_rows], out[:n_rows], p_drop, DROP_ENCODER, l,
                                   count=n_rows)
            acts.append(out)
            A = K.operand(out)
        if early:
            self._wait_side(ev_pairs)            # the pairs (the side stream goes on)
        elif side is not None:
            self._join(side)                     # joined before any collective cut (graph segments)
        else:
            neg_res = negatives_and_pairs()
        n_neg, n_neg_total, cnt, R2, ia_ib = neg_res
        n_lab = P + n_neg
        n_lab_total = P_total + n_neg_total if cnt is None else 0.0
        ia, ib = ia_ib[:R2], ia_ib[R2:]
        if shard is None:
            h = acts[-1]
        else:
            h_full = self._buf("fb_hfull", (s_world * n_loc, H), dt)
            h_loc = acts[-1]
            self._collective(lambda: self._all_gather_rows(h_full, h_loc, s_world, s_rank))
            h = h_full[:N]

        # ---- a6: teacher on the context pairs (+ label pairs for KD_LM, src/main.py:187,215) and the
        # node grouping: with the side stream beside the student forward (early) or the predictor forward
        R_t = R_t_of(R2)
        if early:
            t_head = t_head_early
        elif side is not None and (R_t > 0 or (grouped and self.side_grouping)):
            self._fork(side)
            with torch.cuda.stream(side):
                t_head = pair_work(R2, ia_ib, dh_target() if grouped else None)
        else:
            t_r = self._buf("t_r", (max(R_t, 1),), torch.float32)
            self._t_head = None
            t_head = None

        # ---- a5: predictor over context + label pairs (src/main.py:186,213)
        logit = self._buf("logit", (R2,), torch.float32)
        A0, zacts = self._predictor_forward(h, ia, ib, R2, logit, p_drop, defer_head=True)
        if side is not None and R_t > 0:
            if ev_t is not None:
                self._wait_side(ev_t)            # the teacher (the grouping may still run)
            else:
                self._join(side)
            self._t_head = t_head
        elif R_t > 0:   # (KD_LM reads the label pairs' probabilities: finished here, not in the loss)
            self._teacher_forward(R_t, ia[:R_t], ib[:R_t], t_r, defer_head=R_t == BC)

        # ---- a7-a9: LLP_D + LLP_R + BCE, then KD_RM / KD_LM (src/main.py:217-222)
        dlogit = self._buf("dlogit", (R2,), torch.float32)
        ws = self._ws("ws_loss", K.llp_loss_ws_bytes(Bc, n_lab))
        K.llp_loss(Bc, C, logit, t_r, n_lab, P, logit[BC:], B_total if use_llp else 1, n_lab_total,
                   float(a.margin), 1.0, float(a.True_label), float(a.LLP_D) if use_llp else 0.0,
                   float(a.LLP_R) if use_llp else 0.0, dlogit, dlogit[BC:], self.terms, ws, neg_count=cnt,
                   neg_offset=p_offset, pos_total=P_total, s_head=self._s_head, t_head=self._t_head,
                   ticket=self.loss_ticket)
        self._logit_layout = (Bc, C, n_lab)
        if not grouped:   # in fp32 mode dh32 IS the student backward's first gradient buffer
            dh32 = self._buf("gS0" if dt == torch.float32 else "dh32", (N, H), torch.float32)
            dh32.zero_()
        if w_rm != 0.0 or w_lm != 0.0:
            if w_rm != 0.0 and self.t_h.shape[1] != H:
                raise ValueError("KD_RM needs the student width to equal the teacher's (src/main.py:218)")
            wsk = self._ws("ws_kd", K.kd_terms_ws_bytes(B, n_lab))
            K.kd_terms(self.terms, wsk, n_lab=n_lab if w_lm != 0.0 else 0, out_logit=logit[BC:],
                       t_prob_lab=t_r[BC:R2] if w_lm != 0.0 else None, n_lab_total=n_lab_total, w_lm=w_lm,
                       dlogit_lab=dlogit[BC:], B_rm=B if w_rm != 0.0 else 0, h=h, t_h=self.t_h, idx_rm=anchors,
                       B_rm_total=B_total, w_rm=w_rm, dh=None if grouped else dh32)
            self._kd_clear = False
        elif not getattr(self, "_kd_clear", False):   # no KD terms: cleared once, not every step
            self.terms[4:6].zero_()
            self._kd_clear = True

        # ---- a10: backward
        dZ0 = self._predictor_backward(dlogit, R2, A0, zacts, p_drop)
        mlp = self.predictor_kind == "mlp"
        pre = side is not None and grouped and self.side_grouping
        if side is not None:
            self._join(side)                     # the node grouping; every side branch joined
        if grouped and shard is not None:
            # every rank's d(h) over all nodes as unrounded f32 per-node sums, summed in f32
            # onto the owners' slices (reduce-scatter), then rounded once to the compute dtype
            dh_full = self._buf("fb_dhfull", (s_world * n_loc, H), torch.float32)
            self._hadamard_bwd_nodes(R2, ia_ib, dZ0 if mlp else None, None if mlp else dlogit, h, dh_full[:N],
                                     grouped_in=pre)
            if s_world * n_loc > N:
                dh_full[N:].zero_()
            if dt == torch.float32:
                dh = self._buf("gS0", (n_loc, H), dt)
                self._collective(lambda: self._reduce_scatter_rows(dh, dh_full, s_world, s_rank))
            else:
                dh32 = self._buf("fb_dh32", (n_loc, H), torch.float32)
                self._collective(lambda: self._reduce_scatter_rows(dh32, dh_full, s_world, s_rank))
                dh = self._buf("gS0", (n_loc, H), dt)
                K.convert(dh32, dh)
        elif grouped:
            dh = self._buf("gS0", (N, H), dt)
            self._hadamard_bwd_nodes(R2, ia_ib, dZ0 if mlp else None, None if mlp else dlogit, h, dh,
                                     grouped_in=pre)
        else:
            if mlp:
                K.hadamard_bwd_scatter(R2, H, dZ0, ia, ib, h, dh32)
            else:
                K.hadamard_bwd_scatter(R2, H, None, ia, ib, h, dh32, drow=dlogit)
            if dt == torch.float32:
                dh = dh32
            else:
                dh = self._buf("gS0", (N, H), dt)
                K.convert(dh32, dh)
        sp = (r0, n_rows) if self.xs is not None and (p_drop == 0.0 or bool(self.stu_norms)) else None
        self._student_backward(dh, n_rows, None, acts, p_drop, x_rows=None if shard is None else x_loc,
                               norm_count=n_rows, sparse_rows=sp,
                               side=self._side_stream() if self.overlap_streams and self.side_wgrad else None)
        self._allreduce_and_update()
        K.step_end(self.terms[:1], float(P_total), self.loss_sum, self.step_ctr, adam_step=self.adam_step)
        return n_neg if cnt is None else cnt

    def _fb_shard(self, p_drop, grouped):
        """(first row, rows, rows per rank, world, rank) of this rank's slice of the full-batch student,
        or None: the student over all N nodes on every rank, as in the reference
        (src/main.py:173).  On (``shard_student``, default) with several ranks, no dropout
        (the GEMM's dropout draws are keyed by the row within the call)
        and the node-grouped d(h) (``grouped``: no KD_RM, whose f32 scatter target covers
        all rows, and rows the grouping kernels take).  The slices are all-gathered
        after the forward; d(h) of all nodes is reduce-scattered onto them before the
        student backward, whose weight gradients the usual all-reduce sums.
        ``emulate_shard = (rank, world)`` on a one-rank engine times that rank's slice
        with the collectives replaced by local copies (tools/physics_bench.py)."""
        world, rank = self.world, self.rank
        if world <= 1 and self.emulate_shard is not None:
            rank, world = self.emulate_shard
        if world <= 1 or not self.shard_student or p_drop > 0.0 or not grouped or self._batch_norm:
            return None   # (BatchNorm: statistics over all N nodes, so the student stays replicated)
        n_loc = -(-self.N // world)
        if self.N - (world - 1) * n_loc <= 0:   # a rank without rows: off on every rank alike
            return None
        r0 = rank * n_loc
        n_rows = min(self.N, r0 + n_loc) - r0
        return r0, n_rows, n_loc, world, rank

    def _all_gather_rows(self, full, part, world, rank):
        """full [world * n, H] <- every rank's part [n, H] in rank order."""
        if self.world <= 1:   # emulated shard (timing): this rank's rows stand in for every slice
            full.view(world, *part.shape).copy_(part.unsqueeze(0).expand(world, *part.shape))
        elif dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(full, part, group=self.group)
        else:   # gloo (CPU rehearsal / tests): all_reduce is its one CUDA collective; exact in f32
            t = torch.zeros(full.shape, dtype=_acc_dtype(full), device=full.device)
            t.view(self.world, *part.shape)[self.rank].copy_(part)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            full.copy_(t)

    def _reduce_scatter_rows(self, part, full, world, rank):
        """part [n, H] <- rows [rank * n, (rank + 1) * n) of the SUM over ranks of full."""
        if self.world <= 1:   # emulated shard: this rank's own contribution (timing)
            part.copy_(full.view(world, *part.shape)[rank])
        elif dist.get_backend(self.group) == "nccl":
            dist.reduce_scatter_tensor(part, full, op=dist.ReduceOp.SUM, group=self.group)
        else:
            t = full.to(_acc_dtype(full))
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            part.copy_(t.view(self.world, *part.shape)[self.rank])

    def capture_minibatch(self, anchors, link_ids, pairs, segmented=None, debug_cuts=False, mode="thread_local",
                          batches=None, **kw):
        """Capture one step_minibatch into a hipGraph (torch.cuda.CUDAGraph).

        ``anchors`` / ``link_ids`` must be persistent device buffers: refill them
        (e.g. ``anchors.copy_(node_perm[i*B:(i+1)*B])``) before each ``replay()``.
        Every random draw is keyed by device counters (Philox stream = STREAMS_PER_STEP *
        step_ctr + offset; Adam's step), so each replay is a fresh step.  Call
        after at least one eager step (kernels and buffers already loaded).
        With several ranks the step is captured as segments cut at the gradient
        all-reduces, which run eagerly between them at replay (_SegmentedGraph);
        the returned object has the same ``replay()``.  ``segmented=True`` takes the
        segmented capture on one rank too, ``debug_cuts`` adds a synchronising cut after
        each stage, ``mode`` is the segments' capture mode (tests, tools/seg_diag.py).
        ``batches = (node_perm, b_stride, b_offset, link_perm, p_stride, p_offset, n_batches)``: the
        graph fills ``anchors`` / ``link_ids`` itself with the step's batch of those epoch
        permutations, j = step_ctr mod n_batches (llp_batch_slices), so a replay needs no host
        copy; refresh the permutation buffers in place once per epoch."""
        fill = self._batch_fill(batches, anchors, link_ids)
        return self._capture(lambda: (fill(), self.step_minibatch(anchors, link_ids, pairs, **kw))[1], segmented,
                             debug_cuts, mode)

    def _batch_fill(self, batches, anchors, link_ids):
        if batches is None:
            return lambda: None
        node_perm, b_stride, b_off, link_perm, p_stride, p_off, n_batches = batches
        return lambda: K.batch_slices(node_perm, b_stride, b_off, anchors, link_perm, p_stride, p_off, link_ids,
                                      n_batches, self.step_ctr)

    def capture_fullbatch(self, anchors, link_ids, pairs, segmented=None, mode="thread_local", batches=None, **kw):
        """Capture one step_fullbatch (train, src/main.py:167-235) into a hipGraph, as
        capture_minibatch does: persistent ``anchors`` / ``link_ids`` buffers, refilled
        before each ``replay()`` or by the graph itself (``batches``, capture_minibatch);
        segments between the collectives at several ranks.
        The PyG-dense negatives keep their count on the device (step_fullbatch), so
        the step has no host read; KD_LM, whose kernel takes the host count, cannot
        be captured and raises here."""
        if float(self.args.KD_LM) != 0.0 and kw.get("dense_negatives", True) and kw.get("neg") is None:
            raise NotImplementedError("capture_fullbatch: KD_LM reads the dense negatives' count on the host; "
                                      "run the step eagerly")
        fill = self._batch_fill(batches, anchors, link_ids)
        return self._capture(lambda: (fill(), self.step_fullbatch(anchors, link_ids, pairs, **kw))[1], segmented,
                             False, mode)

    def _capture(self, step, segmented, debug_cuts, mode):
        if segmented is None:
            segmented = self.world > 1
        if segmented:
            # RCCL stays outside the graphs: one segment per stretch between collectives
            torch.cuda.synchronize(self.dev)
            seg = _SegmentedGraph(self.dev, mode)
            seg.stream.wait_stream(torch.cuda.current_stream(self.dev))
            self._seg = seg
            self._seg_debug = bool(debug_cuts)
            try:
                seg.begin()
                step()
            finally:
                self._seg = None
                self._seg_debug = False
                seg.end()
            torch.cuda.current_stream(self.dev).wait_stream(seg.stream)
            return seg
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.graph(g, stream=s):
            step()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        return g

    def _teacher_forward(self, R, t_ia, t_ib, t_r, defer_head=False):
        """The frozen teacher predictor's probabilities t_r over R pairs; with ``defer_head``
        and the fused head GEMM, left as head partials in ``self._t_head`` (the loss launch
        finishes them, see _predictor_forward)."""
        dt, dc = self.dtype, self.dc
        self._t_head = None
        if self.t_kind == "inner":
            K.head_fwd(self.t_h, R, self.t_h.shape[1], None, None, prob=t_r, Z2=self.t_h, iz=t_ia, iz2=t_ib)
            return
        Ht = self.t_h.shape[1]
        if len(self.t_hidden) == 1 and self._fusable(Ht, self.t_hidden[0][0].shape[0], self.t_dropout):
            # t_h[a] * t_h[c] materialised, then hidden layer + head in one GEMM; the bf16
            # hidden activations are never stored (no backward through the teacher); the f32
            # kernel's head epilogue stores them (one pass instead of the head's second read)
            tin = self._buf("Tin", (R, Ht), dt)
            K.hadamard_rows(self.t_h, t_ia, self.t_h, t_ib, tin)
            W, b = self.t_hidden[0]
            w2, b2 = self.t_head
            parts = K.head_parts(W.shape[0])
            tpart = self._buf("tpart", (parts, R), torch.float32)
            if dt == torch.float32:
                K.gemm_nt_head_f32(K.operand(tin), K.operand(W), R, W.shape[0], W.shape[1],
                                   self._buf("T0", (R, W.shape[0]), dt), w2, tpart, bias=b)
            else:
                K.gemm_nt_head(K.operand(tin), K.operand(W), R, W.shape[0], W.shape[1], None, w2, tpart, bias=b,
                               act=K.ACT_RELU, dropout=self._dropout(self.t_dropout, DROP_TEACHER_PRED, 0))
            if defer_head:
                self._t_head = K.head_in(tpart, parts, R, b2)
            else:
                K.head_finish(parts, R, tpart, b2, prob=t_r)
            return
        if self.dtype == torch.float32 and not self.t_dropout:
            # t_h[a] * t_h[c] materialised: plain rows take the persistent f32 kernel (§4.8), the
            # on-load Hadamard operand only the 128-tile one (0.81 ms, 76 TF/s at the collab shape)
            tin = self._buf("Tin", (R, Ht), self.dtype)
            K.hadamard_rows(self.t_h, t_ia, self.t_h, t_ib, tin)
            A = K.operand(tin)
        else:
            A = K.operand(self.t_h, t_ia, self.t_h, t_ib)
        out = None
        for l, (W, b) in enumerate(self.t_hidden):
            out = self._buf(f"T{l}", (R, W.shape[0]), dt)
            K.gemm_nt(A, K.operand(W), R, W.shape[0], W.shape[1], out, dc, bias=b, act=K.ACT_RELU,
                      dropout=self._dropout(self.t_dropout, DROP_TEACHER_PRED, l))
            A = K.operand(out)
        w, b = self.t_head
        K.head_fwd(out, R, out.shape[1], w, b, prob=t_r)

    def _student_backward(self, dh, R1, target, acts, p_drop, count=None, x_rows=None, norm_count=0.0,
                          norm_sync=False, sparse_rows=None, side=None):
        """count: int32 device row count (unique-node student) or None.  dh lives in
        buffer 'gS0'.  x_rows: x[target] materialised by the forward (else the first
        layer's input is gathered).  norm_count / norm_sync: BatchNorm's batch row count
        and whether its sums are all-reduced across ranks (_norm_backward).  sparse_rows:
        (first row, rows) of the sparse x the forward's first layer ran on (llp_spmm_rows):
        its weight gradient by llp_spmm_tn over the same rows, the bias gradient by llp_colsum."""
        dt, dc = self.dtype, self.dc
        alpha = 1.0 / (1.0 - p_drop) if p_drop > 0 else 1.0
        names = ["gS0", "gS1"]
        k = 0
        for l in range(len(self.stu) - 1, -1, -1):
            lin = self.stu[l]
            gcur = self._buf(names[k % 2], (R1, lin.out_f), dt)
            if l > 0:
                A_in = K.operand(acts[l - 1], count=count)
            elif x_rows is not None:
                A_in = K.operand(x_rows, count=count)
            else:
                A_in = K.operand(self.x, target, count=count)
            if l == 0 and sparse_rows is not None:
                if side is not None:   # the bias gradient's column sums beside the sparse weight gradient
                    self._fork(side)
                with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                    K.colsum(gcur, R1, lin.out_f, lin.lin.bias.grad,
                             self._ws("ws_colsum", K.colsum_ws_bytes(R1, lin.out_f)))
                K.spmm_tn(self.xs, sparse_rows[0], sparse_rows[1], gcur, lin.lin.weight.grad)
                if side is not None:
                    self._join(side)
                continue
            wsb = K.gemm_tn_ws_bytes(dc, R1, lin.out_f, lin.k_in)
            padded = lin.k_in != lin.in_f
            dW = self._buf("dW_pad", (lin.out_f, lin.k_in), torch.float32) if padded else lin.lin.weight.grad
            # a data-gradient GEMM of at most half a wave of tiles (the full-batch student at small
            # shards: 31-122 tiles) leaves most CUs idle: the weight gradient runs beside it on the
            # side stream (both only read gcur and the activations)
            par = (side is not None and l > 0 and not self.stu_norms
                   and -(-R1 // 256) * -(-lin.in_f // 256) <= self._cu_count() // 2)
            if par:
                self._fork(side)
            with torch.cuda.stream(side) if par else contextlib.nullcontext():
                K.gemm_tn(K.operand(gcur, count=count), A_in, R1, lin.out_f, lin.k_in, dW, dc, self._ws("ws_tn", wsb),
                          colsum_a=lin.lin.bias.grad)
                if padded:   # the zero-padded input columns' gradient is dropped
                    lin.lin.weight.grad.copy_(dW[:, :lin.in_f])
            if l > 0:    # this layer's gradients are final: all-reduce them under the next layers' GEMMs
                if not par:
                    self._allreduce_bucket(*self._grad_slice(lin.lin.weight, lin.lin.bias))
                k += 1
                gnext = self._buf(names[k % 2], (R1, lin.in_f), dt)
                if self.stu_norms:
                    # d(post-ReLU/dropout activations), then through the norm into d(pre-norm output)
                    graw = self._buf("gN", (R1, lin.in_f), dt)
                    K.gemm_nt(K.operand(gcur, count=count), K.operand(lin.Wt), R1, lin.in_f, lin.out_f, graw, dc)
                    y = self._buf(f"Y{l - 1}", (R1, lin.in_f), dt)
                    self._norm_backward(self.stu_norms[l - 1], f"s{l - 1}", graw, acts[l - 1], alpha, y, gnext,
                                        rows=count, count=norm_count, sync=norm_sync)
                else:
                    K.gemm_nt(K.operand(gcur, count=count), K.operand(lin.Wt), R1, lin.in_f, lin.out_f, gnext, dc,
                              act=K.ACT_RELU_BWD, aux=self._relu_aux(acts[l - 1]), alpha=alpha)
                if par:   # joined before the bucket's all-reduce reads the weight gradient
                    self._join(side)
                    self._allreduce_bucket(*self._grad_slice(lin.lin.weight, lin.lin.bias))
