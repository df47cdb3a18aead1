"""MI355X GraphSAGE teacher engine: one link batch of the teacher's ``train``
(src/train_teacher_gnn.py:21-73) — full-graph SAGE encoder forward/backward,
LinkPredictor on h[train_edges], BCE, clip_grad_norm_ per module, Adam — as a
fixed sequence of hand-written gfx950 kernels.

Encoder layer l (in F, out O), both conv flavours the reference uses:

  SAGEConv (PyG 2.2.0, aggr='mean', src/train_teacher_gnn.py:381-383)
      out = mean_j x_j . W_l^T + b + x . W_r^T
      HBM layout: XA_l = [agg | x] (N x 2F, one buffer): the CSR aggregate
      writes the left half, the previous layer's GEMM epilogue (bias, ReLU,
      dropout) writes x into the right half, and ONE K-concatenated MFMA GEMM
      against Wcat = [W_l | W_r] (O x 2F) produces the layer.
  SAGEConv_updated (src/sageconv_updated.py:65-81, coauthor-physics)
      out = mean_j (x_j . W_l^T + b) + x . W_r^T
      ONE GEMM against Wst = [W_l ; W_r] (2O x F) gives [U | R] (N x 2O); the
      aggregate of U accumulates into R in place.

  GCNConv (PyG 2.2.0, cached=True; the GCN encoder, src/models.py:56-80)
      out = D^-1/2 (A - loops + I) D^-1/2 (x W^T) + b
      ONE GEMM Y = x W^T, then the normalised aggregate of Y over the
      self-loop CSR with the bias fused (llp_gcn_aggregate); ReLU/dropout by
      act_2d.  Backward: db = colsum(dZ), dY = the same aggregate over the
      transposed CSR, dW = dY^T x (TN), dX = dY W with the previous layer's
      mask in the GEMM epilogue.

Backward (SAGE flavours): with dOut the layer's output gradient and
G = mean-backward(dOut) over the transposed CSR, dX = [G | dOut] . [W_l^T | W_r^T]
is ONE K-concatenated GEMM whose epilogue applies the previous layer's
ReLU/dropout mask; weight gradients are TN GEMMs with the bias gradient fused.
The weight copies (Wcat / Wst and the shared [W_l^T | W_r^T]) are shadows the
Adam kernel refreshes through descriptor leading dimensions.

Aggregation follows PyG: messages flow edge_index[0] -> edge_index[1],
duplicates counted, isolated nodes get 0.
"""
from __future__ import annotations

import numpy as np
import torch

import llp_hip as K
from llp_engine import DROP_ENCODER, EngineBase, _norms_of, _resets_on_error
from llp_sage import GCNConv, Graph, SAGEConv_updated, locality_order


class TeacherEngine(EngineBase):
    """``model``: models.SAGE (convs of SAGEConv or SAGEConv_updated, root_weight,
    norm_type 'none' / 'layer' / 'batch') or models.GCN (GCNConv with bias); ``predictor``: LinkPredictor;
    ``x``: node features;
    ``edge_index``: the message-passing graph (data.adj_t / data.edge_index,
    src/train_teacher_gnn.py:23-27,43-46); ``optimizer``: Adam over
    model.parameters() + predictor.parameters()."""

    def __init__(self, model, predictor, x, edge_index, num_nodes, optimizer, dtype="fp32", seed=0, group=None,
                 device=None, reorder=True):
        self._init_device(x.device, device, dtype, seed, group, "TeacherEngine")
        self.N = int(num_nodes)
        N = self.N
        dt = self.dtype
        self.model, self.predictor = model, predictor
        self.convs = list(model.convs)
        self.gcn = isinstance(self.convs[0], GCNConv)
        self.updated = isinstance(self.convs[0], SAGEConv_updated)
        if self.gcn:
            if any(not isinstance(c, GCNConv) or c.bias is None for c in self.convs):
                raise NotImplementedError("all convs GCNConv with bias")
        elif any(isinstance(c, SAGEConv_updated) != self.updated or not c.root_weight for c in self.convs):
            raise NotImplementedError("all convs of one flavour, with root_weight")
        # norm_type 'layer' / 'batch' (src/models.py:90-101,114-115): conv, norm, ReLU, dropout.  The
        # encoder runs on the whole graph on every rank, so BatchNorm's statistics need no exchange.
        self.norms = _norms_of(model, len(self.convs) - 1, self._conv_out(self.convs[0]))
        self.p_drop = float(model.dropout)
        ei = edge_index.cpu().numpy() if torch.is_tensor(edge_index) else np.asarray(edge_index)
        # Node order inside the engine (``reorder``): a locality order (llp_sage.locality_order,
        # label propagation) under which most of a node's neighbours sit next to it, so the CSR
        # aggregate's neighbour rows are L2 hits; node v lives in row pi[v] of every node table
        # (x, activations, h), the edges are relabelled with their order kept (so every row's
        # neighbour sum runs in the same order: the same values), link and negative pairs are
        # drawn on the original ids and mapped, and embed() returns rows in the original order
        self._pi = self._order = None
        ei_int = ei
        if reorder and N > 1:
            order, pi = locality_order(ei, N)
            self._order = torch.from_numpy(order.astype(np.int32)).to(self.dev)   # engine row -> node
            self._pi = torch.from_numpy(pi.astype(np.int32)).to(self.dev)         # node -> engine row
            ei_int = pi[ei]
        self.graph = Graph(ei_int, N, self.dev, gcn=self.gcn)
        self._neg_rc = (ei[0], ei[1])        # row, col = data.adj_t (src/train_teacher_gnn.py:23), original ids
        self.num_edges = int(ei.shape[1])

        # ---------------- per-layer weights and shadows
        self.layers = []
        for l, conv in enumerate(self.convs):
            if self.gcn:
                W = conv.lin.weight
                O, F = W.shape
                Wc = torch.empty(O, F, dtype=dt, device=self.dev)
                WT = torch.empty(F, O, dtype=dt, device=self.dev)
                self._set_shadow(W, Wc, WT)
                self.layers.append(dict(F=F, O=O, conv=conv, Wf=Wc, WT=WT, bias=conv.bias.data))
                continue
            Wl, bl, Wr = conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight
            O, F = Wl.shape
            L = dict(F=F, O=O, conv=conv)
            WT = torch.empty(F, 2 * O, dtype=dt, device=self.dev)          # [W_l^T | W_r^T]
            if self.updated:
                Wst = torch.empty(2 * O, F, dtype=dt, device=self.dev)      # [W_l ; W_r]
                self._set_shadow(Wl, Wst[:O], WT[:, :O], 0, 2 * O)
                self._set_shadow(Wr, Wst[O:], WT[:, O:], 0, 2 * O)
                bias2 = torch.zeros(2 * O, dtype=torch.float32, device=self.dev)
                bias2[:O].copy_(bl.data)
                bl.data = bias2[:O]                                         # the module's bias now lives here
                L.update(Wf=Wst, bias=bias2)
            else:
                Wcat = torch.empty(O, 2 * F, dtype=dt, device=self.dev)     # [W_l | W_r]
                self._set_shadow(Wl, Wcat[:, :F], WT[:, :O], 2 * F, 2 * O)
                self._set_shadow(Wr, Wcat[:, F:], WT[:, O:], 2 * F, 2 * O)
                L.update(Wf=Wcat, bias=bl.data)
            L["WT"] = WT
            self.layers.append(L)
        enc_params = [p for p in model.parameters()]
        prd_params = self._setup_predictor(predictor, predictor.predictor)
        self.pred_drop = float(predictor.dropout)
        self._init_params(enc_params + prd_params, [0] * len(enc_params) + [1] * len(prd_params), optimizer)

        # ---------------- activations (HBM-resident for the whole run)
        x = x.to(self.dev)
        if self._order is not None:
            x = x.index_select(0, self._order.long())
        for l, L in enumerate(self.layers):
            F, O = L["F"], L["O"]
            if self.gcn:
                L["X"] = x.to(dt).contiguous() if l == 0 else torch.empty(N, F, dtype=dt, device=self.dev)
                L["G"] = torch.empty(N, O, dtype=dt, device=self.dev)          # dZ of the layer
                continue
            if self.updated:
                L["X"] = x.to(dt).contiguous() if l == 0 else torch.empty(N, F, dtype=dt, device=self.dev)
                L["YY"] = torch.empty(N, 2 * O, dtype=dt, device=self.dev)
            else:
                XA = torch.empty(N, 2 * F, dtype=dt, device=self.dev)
                if l == 0:
                    XA[:, F:].copy_(x.to(dt))
                L["XA"] = XA
                L["X"] = XA[:, F:]
            L["G"] = torch.empty(N, 2 * O, dtype=dt, device=self.dev)        # [mean-bwd(dOut) | dOut]
        # ReLU(+dropout) bit masks of the SAGEConv layer inputs (bf16): layer l-1's forward GEMM
        # writes bit (output > 0) of layer l's input, layer l's data-gradient GEMM reads it in
        # place of the bf16 activations (16x less epilogue traffic); both on the 256-tile path
        if not (self.gcn or self.updated or self.norms) and dt == torch.bfloat16:
            for l in range(1, len(self.layers)):
                P_, L = self.layers[l - 1], self.layers[l]
                if L["F"] % 32 == 0 and (2 * P_["F"]) % 64 == 0 and (2 * L["O"]) % 64 == 0:
                    L["M"] = torch.empty(N, L["F"] // 8, dtype=torch.uint8, device=self.dev)
        # SAGEConv's two weight gradients as one GEMM over [agg(x) | x] (False: two, the A/B baseline)
        self.fused_wgrad = True
        self._agg0_done = False   # mean aggregate of the input features (first SAGEConv layer) formed
        self.out_dim = self.layers[-1]["O"]
        self.h = torch.empty(N, self.out_dim, dtype=dt, device=self.dev)
        self._build_descs()

    @staticmethod
    def _conv_out(conv):
        return conv.lin.weight.shape[0] if isinstance(conv, GCNConv) else conv.lin_l.weight.shape[0]

    # ------------------------------------------------------------------ encoder
    def _encode(self, training: bool):
        """SAGE.forward (src/models.py:110-119): conv, ReLU, dropout between layers."""
        g = self.graph
        dc = self.dc
        N = self.N
        nl = len(self.layers)
        for l, L in enumerate(self.layers):
            F, O = L["F"], L["O"]
            last = l == nl - 1
            drop = None if (last or not training) else self._dropout(self.p_drop, DROP_ENCODER, l)
            act = K.ACT_NONE if last else K.ACT_RELU
            nxt = None if last else self.layers[l + 1]
            if self.gcn:
                Y = self._buf("gcn_Y", (N, O), self.dtype)
                K.gemm_nt(K.operand(L["X"]), K.operand(L["Wf"]), N, O, F, Y, dc)
                if last:
                    K.gcn_aggregate(N, O, g.rowptr, g.col, Y, g.dinv, self.h, bias=L["bias"])
                else:
                    Z = self._buf("gcn_Z", (N, O), self.dtype)
                    K.gcn_aggregate(N, O, g.rowptr, g.col, Y, g.dinv, Z, bias=L["bias"])
                    K.act_2d(Z, nxt["X"], act=act, dropout=drop)
            elif self.updated:
                YY = L["YY"]
                K.gemm_nt(K.operand(L["X"]), K.operand(L["Wf"]), N, 2 * O, F, YY, dc, bias=L["bias"])
                K.csr_aggregate(N, O, g.rowptr, g.col, YY[:, :O], None, 0, YY[:, O:], accumulate=True)
                if self.norms and not last:
                    self._norm_forward(self.norms[l], f"t{l}", YY[:, O:], nxt["X"], self.p_drop, DROP_ENCODER, l,
                                       count=N, training=training)
                else:
                    K.act_2d(YY[:, O:], self.h if last else nxt["X"], act=act, dropout=drop)
            else:
                XA = L["XA"]
                # the first layer aggregates the raw features (no dropout before it,
                # src/models.py:113-118): the same every step, so formed once
                if l > 0 or not self._agg0_done:
                    K.csr_aggregate(N, F, g.rowptr, g.col, XA[:, F:], None, 0, XA[:, :F])
                    self._agg0_done = l == 0 or self._agg0_done
                out = self.h if last else nxt["X"]
                if self.norms and not last:
                    Y = self._buf(f"tY{l}", (N, O), self.dtype)
                    K.gemm_nt(K.operand(XA), K.operand(L["Wf"]), N, O, 2 * F, Y, dc, bias=L["bias"])
                    self._norm_forward(self.norms[l], f"t{l}", Y, out, self.p_drop, DROP_ENCODER, l, count=N,
                                       training=training)
                else:
                    K.gemm_nt(K.operand(XA), K.operand(L["Wf"]), N, O, 2 * F, out, dc, bias=L["bias"], act=act,
                              aux=None if last else nxt.get("M"), dropout=drop)
        return self.h

    def _pre_norm(self, l):
        """Layer l's pre-norm output (its conv output) [N, O]."""
        L = self.layers[l]
        return L["YY"][:, L["O"]:] if self.updated else self._buf(f"tY{l}", (self.N, L["O"]), self.dtype)

    def _dh_slot(self):
        """The last layer's output-gradient slot [N, O] (compute dtype): d(loss)/dh lands here."""
        last = self.layers[-1]
        return last["G"] if self.gcn else last["G"][:, last["O"]:]

    def _encode_backward(self):
        """Backward of _encode from d(loss)/dh, already in _dh_slot()."""
        g = self.graph
        dt, dc = self.dtype, self.dc
        N = self.N
        alpha = 1.0 / (1.0 - self.p_drop) if self.p_drop > 0 else 1.0
        nl = len(self.layers)
        if self.gcn:
            return self._gcn_backward(alpha)
        for l in range(nl - 1, -1, -1):
            L = self.layers[l]
            F, O = L["F"], L["O"]
            G = L["G"]
            dOut = G[:, O:]
            conv = L["conv"]
            # G = mean-backward(dOut) over the transposed CSR (scale 1/deg of the destination);
            # SAGEConv's first layer needs no input gradient, and its weight gradients read dOut
            # and the stored forward aggregate, so G is not formed there
            if l > 0 or self.updated:
                K.csr_aggregate(N, O, g.rowptr_t, g.col_t, dOut, g.inv_deg, 1, G[:, :O])
            if self.updated:
                # U = x W_l^T + b is aggregated: dW_l = G^T x, db = colsum(G); dW_r = dOut^T x
                ws = self._ws("ws_tn", K.gemm_tn_ws_bytes(dc, N, O, F))
                K.gemm_tn(K.operand(G[:, :O]), K.operand(L["X"]), N, O, F, conv.lin_l.weight.grad, dc, ws,
                          colsum_a=conv.lin_l.bias.grad)
                K.gemm_tn(K.operand(dOut), K.operand(L["X"]), N, O, F, conv.lin_r.weight.grad, dc, ws)
            elif not self.fused_wgrad:   # A/B: the two GEMMs of round 4
                ws = self._ws("ws_tn", K.gemm_tn_ws_bytes(dc, N, O, F))
                K.gemm_tn(K.operand(dOut), K.operand(L["XA"][:, :F]), N, O, F, conv.lin_l.weight.grad, dc, ws,
                          colsum_a=conv.lin_l.bias.grad)
                K.gemm_tn(K.operand(dOut), K.operand(L["X"]), N, O, F, conv.lin_r.weight.grad, dc, ws)
            else:
                # dW_l = dOut^T agg(x), db = colsum(dOut); dW_r = dOut^T x: ONE weight-gradient GEMM over
                # the layer's [agg(x) | x] (XA, the forward's K-concatenated operand), so dOut is read
                # once and one launch + one slab reduce go (round 5); the [O, 2F] result is split
                # into the two modules' gradients by the GEMM's column-split output
                # (llp_gemm_tn_split, round 6: no [O, 2F] buffer, no two strided copies per layer)
                ws = self._ws("ws_tn", K.gemm_tn_ws_bytes(dc, N, O, 2 * F))
                K.gemm_tn(K.operand(dOut), K.operand(L["XA"]), N, O, 2 * F, conv.lin_l.weight.grad, dc, ws,
                          colsum_a=conv.lin_l.bias.grad, split=(F, conv.lin_r.weight.grad))
            if l > 0:
                # dX = [G | dOut] . [W_l^T | W_r^T]^T, ReLU/dropout mask of layer l-1 in the epilogue,
                # written straight into layer l-1's output-gradient slot
                prev = self.layers[l - 1]
                if self.norms:
                    # d(layer l's input) = d(dropout(relu(norm(y_{l-1})))), then through the norm
                    graw = self._buf("tgN", (N, F), dt)
                    K.gemm_nt(K.operand(G), K.operand(L["WT"]), N, F, 2 * O, graw, dc)
                    self._norm_backward(self.norms[l - 1], f"t{l - 1}", graw, L["X"], alpha, self._pre_norm(l - 1),
                                        prev["G"][:, prev["O"]:], count=N)
                    continue
                mask = L.get("M")
                K.gemm_nt(K.operand(G), K.operand(L["WT"]), N, F, 2 * O, prev["G"][:, prev["O"]:], dc,
                          act=K.ACT_RELU_BWD, aux=L["X"] if mask is None else mask, alpha=alpha)

    def _gcn_backward(self, alpha):
        g = self.graph
        dt, dc = self.dtype, self.dc
        N = self.N
        for l in range(len(self.layers) - 1, -1, -1):
            L = self.layers[l]
            F, O = L["F"], L["O"]
            dZ, conv = L["G"], L["conv"]
            K.colsum(dZ, N, O, conv.bias.grad, self._ws("ws_colsum", K.colsum_ws_bytes(N, O)))
            dY = self._buf("gcn_dY", (N, O), dt)
            K.gcn_aggregate(N, O, g.rowptr_t, g.col_t, dZ, g.dinv, dY)
            ws = self._ws("ws_tn", K.gemm_tn_ws_bytes(dc, N, O, F))
            K.gemm_tn(K.operand(dY), K.operand(L["X"]), N, O, F, conv.lin.weight.grad, dc, ws)
            if l > 0:
                prev = self.layers[l - 1]
                K.gemm_nt(K.operand(dY), K.operand(L["WT"]), N, F, O, prev["G"], dc, act=K.ACT_RELU_BWD,
                          aux=L["X"], alpha=alpha)

    # ------------------------------------------------------------------ the step
    @_resets_on_error
    def step(self, link_ids, pairs, p_offset=0, P_total=None, neg=None, dense_negatives=True):
        """One batch of train() (src/train_teacher_gnn.py:33-71).

        link_ids int32[P]   this rank's slice of the DataLoader permutation
        pairs    int32[E,2] pos_train_edge (src/train_teacher_gnn.py:25,28)
        dense_negatives: PyG dense sampler (non-collab) else randint (collab).
        Returns the number of negatives used: a host int (injected / randint), or the
        PyG-dense count as an int32 device tensor (no host read in the step)."""
        P = int(link_ids.numel())
        P_total = P if P_total is None else int(P_total)
        N, O = self.N, self.out_dim
        h = self._encode(training=True)
        # PyG-dense negatives: their count stays on the device (slots past it inert), no host read
        negb, n_neg, n_neg_total, cnt = self._negatives(P, P_total, p_offset, neg, dense_negatives,
                                                        device_count=True)
        R = P + n_neg
        tgt = self._buf("t_tgt", (max(2 * R, 1),), torch.int32)[:2 * R]   # [ia | ib]: endpoint rows
        ia, ib = tgt[:R], tgt[R:]
        K.fullbatch_pairs(0, 0, None, pairs, link_ids, P, negb if n_neg > 0 else None, n_neg, ia, ib, neg_count=cnt,
                          neg_offset=p_offset)
        if self._pi is not None:   # node ids -> the engine's rows (in place)
            K.gather_i32(tgt, self._pi, tgt)
        logit = self._buf("logit", (R,), torch.float32)
        A0, zacts = self._predictor_forward(h, ia, ib, R, logit, self.pred_drop, defer_head=True)
        dlogit = self._buf("dlogit", (R,), torch.float32)
        ws = self._ws("ws_loss", K.llp_loss_ws_bytes(0, R))
        # BCE only (src/train_teacher_gnn.py:56-58), the head's finish in the same launch
        K.llp_loss(0, 1, None, None, R, P, logit, 1, P_total + n_neg_total if cnt is None else 0.0, 0.0, 1.0, 1.0,
                   0.0, 0.0, None, dlogit, self.terms, ws, neg_count=cnt, neg_offset=p_offset, pos_total=P_total,
                   s_head=self._s_head, ticket=self.loss_ticket)
        dZ0 = self._predictor_backward(dlogit, R, A0, zacts, self.pred_drop)
        if self.predictor_kind == "mlp":
            self._hadamard_bwd_nodes(R, tgt, dZ0, None, h, self._dh_slot())
        else:
            self._hadamard_bwd_nodes(R, tgt, None, dlogit, h, self._dh_slot())
        self._encode_backward()
        self._allreduce_and_update()
        K.step_end(self.terms[:1], float(P_total), self.loss_sum, self.step_ctr, adam_step=self.adam_step)
        return n_neg if cnt is None else cnt

    @torch.no_grad()
    def embed(self):
        """model(x, adj_t) in eval mode (src/train_teacher_gnn.py:87) -> f32 [N, O], rows in the
        original node order."""
        h = self._encode(training=False)
        if self._pi is not None:
            out = torch.empty_like(h)
            K.gather_rows(h, self._pi, out)     # node v <- engine row pi[v]
            h = out
        return h.float()
