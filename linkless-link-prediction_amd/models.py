"""Model classes with the reference's constructor signatures and state_dict keys
(src/models.py), computing on MI355X through libllp_hip (llp_ops.py).

  MLP(num_layers, input_dim, hidden_dim, output_dim, dropout_ratio, norm_type='none')   src/models.py:6-54
  GCN(in, hidden, out, num_layers, dropout)                                             src/models.py:56-80
  SAGE(data_name, in, hidden, out, num_layers, dropout, conv_layer, norm_type='none')   src/models.py:82-119
  LinkPredictor(predictor, in, hidden, out, num_layers, dropout)                        src/models.py:121-150

State-dict keys match (``layers.{i}.weight``, ``lins.{i}.weight``,
``convs.{i}.lin_l.weight`` ...), so teacher/student checkpoints written by the
reference load here and vice versa.  Forward/backward run as HIP kernels; a CPU
tensor raises (no fallback).  norm_type 'batch' / 'layer' (never set by the
reference's scripts or CLIs, but part of its Python API) builds nn.BatchNorm1d /
nn.LayerNorm after every hidden layer, as the reference does, and runs them as the
fused norm + ReLU + dropout kernels (csrc/norm.hip).
"""
import torch
import torch.nn as nn

import llp_ops as ops


class MLP(nn.Module):
    def __init__(self, num_layers, input_dim, hidden_dim, output_dim, dropout_ratio, norm_type="none"):
        super().__init__()
        self.num_layers = num_layers
        self.norm_type = norm_type
        self.dropout = nn.Dropout(dropout_ratio)
        self.layers = nn.ModuleList()
        self.norms = nn.ModuleList()
        if num_layers == 1:
            self.layers.append(nn.Linear(input_dim, output_dim))
        else:
            self.layers.append(nn.Linear(input_dim, hidden_dim))
            _add_norm(self.norms, norm_type, hidden_dim)
            for _ in range(num_layers - 2):
                self.layers.append(nn.Linear(hidden_dim, hidden_dim))
                _add_norm(self.norms, norm_type, hidden_dim)
            self.layers.append(nn.Linear(hidden_dim, output_dim))

    def reset_parameters(self):
        for layer in self.layers:
            layer.reset_parameters()

    def forward(self, feats):
        # Linear, then (norm +) ReLU + dropout on every layer but the last (src/models.py:45-54),
        # ReLU and dropout fused into the GEMM epilogue, or into the norm kernel.
        h = feats
        for l, layer in enumerate(self.layers):
            last = l == self.num_layers - 1
            if not last and self.norm_type != "none":
                h = ops.linear(h, layer.weight, layer.bias)
                h = ops.norm_act(h, self.norms[l], p=self.dropout.p, training=self.training)
                continue
            h = ops.linear(h, layer.weight, layer.bias, relu=not last,
                           dropout=0.0 if last else self.dropout.p, training=self.training)
        return h


def _add_norm(norms, norm_type, width):
    """src/models.py:27-30,34-37,90-93,98-101: BatchNorm1d / LayerNorm per hidden layer."""
    if norm_type == "batch":
        norms.append(nn.BatchNorm1d(width))
    elif norm_type == "layer":
        norms.append(nn.LayerNorm(width))


class GCN(nn.Module):
    """src/models.py:56-80: GCNConv(cached=True) layers (llp_sage.GCNConv),
    ReLU + dropout between them.  Trained by llp_teacher.TeacherEngine."""

    def __init__(self, in_channels, hidden_channels, out_channels, num_layers, dropout):
        super().__init__()
        from llp_sage import GCNConv
        self.convs = nn.ModuleList()
        self.convs.append(GCNConv(in_channels, hidden_channels, cached=True))
        for _ in range(num_layers - 2):
            self.convs.append(GCNConv(hidden_channels, hidden_channels, cached=True))
        self.convs.append(GCNConv(hidden_channels, out_channels, cached=True))
        self.dropout = dropout

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, adj_t):
        for conv in self.convs[:-1]:
            x = conv(x, adj_t)
            x = ops.relu_dropout(x, self.dropout, self.training)
        return self.convs[-1](x, adj_t)


class SAGE(nn.Module):
    """src/models.py:82-119: conv_layer is llp_sage.SAGEConv (PyG SAGEConv
    semantics) or llp_sage.SAGEConv_updated.  The training hot path is
    llp_teacher.TeacherEngine; this module is the eval / autograd surface."""

    def __init__(self, data_name, in_channels, hidden_channels, out_channels, num_layers, dropout, conv_layer,
                 norm_type="none"):
        super().__init__()
        self.data_name = data_name
        self.convs = nn.ModuleList()
        self.norms = nn.ModuleList()
        self.norm_type = norm_type
        _add_norm(self.norms, norm_type, hidden_channels)
        self.convs.append(conv_layer(in_channels, hidden_channels))
        for _ in range(num_layers - 2):
            self.convs.append(conv_layer(hidden_channels, hidden_channels))
            _add_norm(self.norms, norm_type, hidden_channels)
        self.convs.append(conv_layer(hidden_channels, out_channels))
        self.dropout = dropout

    def reset_parameters(self):
        for conv in self.convs:
            conv.reset_parameters()

    def forward(self, x, adj_t):
        for l, conv in enumerate(self.convs[:-1]):
            x = conv(x, adj_t)
            if self.norm_type != "none":
                x = ops.norm_act(x, self.norms[l], self.dropout, self.training)
            else:
                x = ops.relu_dropout(x, self.dropout, self.training)
        return self.convs[-1](x, adj_t)


class LinkPredictor(nn.Module):
    def __init__(self, predictor, in_channels, hidden_channels, out_channels, num_layers, dropout):
        super().__init__()
        self.predictor = predictor
        self.lins = nn.ModuleList()
        self.lins.append(nn.Linear(in_channels, hidden_channels))
        for _ in range(num_layers - 2):
            self.lins.append(nn.Linear(hidden_channels, hidden_channels))
        self.lins.append(nn.Linear(hidden_channels, out_channels))
        self.dropout = dropout

    def reset_parameters(self):
        for lin in self.lins:
            lin.reset_parameters()

    def forward(self, x_i, x_j):
        # sigmoid(Lin_L(...ReLU/dropout(Lin_1(x_i * x_j)))) (src/models.py:139-150);
        # x_i * x_j is formed while the first GEMM stages its A tile.
        if x_i.shape != x_j.shape:
            x_i, x_j = torch.broadcast_tensors(x_i, x_j)
        if self.predictor == "mlp":
            if self.lins[-1].out_features != 1:
                raise NotImplementedError("LinkPredictor out_channels != 1")
            x = None
            for l, lin in enumerate(self.lins[:-1]):
                if l == 0:
                    x = ops.linear(x_i, lin.weight, lin.bias, relu=True, dropout=self.dropout,
                                   training=self.training, x2=x_j)
                else:
                    x = ops.linear(x, lin.weight, lin.bias, relu=True, dropout=self.dropout, training=self.training)
            if x is None:
                raise NotImplementedError("LinkPredictor with num_layers < 2")
            return ops.head(x, self.lins[-1].weight, self.lins[-1].bias)
        elif self.predictor == "inner":
            return ops.head(x_i, z2=x_j)
        raise ValueError(self.predictor)
