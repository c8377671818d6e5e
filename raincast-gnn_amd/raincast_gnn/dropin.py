"""The reference's model with only the GINEConv import swapped: the drop-in path.

models/gnn.py imports ``GINEConv`` from torch_geometric (gnn.py:5) and everything else
from torch.  :class:`ReferenceStructGNN` is that module tree -- ``DeepSetEncoder`` (gnn.py:
48-68), ``dim_red`` (gnn.py:112-113), ``ResGnn`` (gnn.py:10-45) calling ``conv(x,
edge_index, edge_attr)`` then applying ReLU / the residual in torch (gnn.py:41,44),
``aggr`` and ``PostProcess`` (gnn.py:123-125, 139-141) -- built from plain
``torch.nn.Linear`` / ``BatchNorm1d`` modules, with :class:`raincast_gnn.nn.GINEConv` in
place of PyG's.  Same state_dict keys as the reference and as :class:`raincast_gnn.models.
GNN`.  The loss is the torch formulation of models/loss.py (``fused=False``), the optimizer
``torch.optim.AdamW``: what train.py:55-74 runs once PyG's layer is replaced, and nothing
more.  bench.py ``--dropin`` times it with ``batch.to(device)`` every step (a fresh
``edge_index`` tensor each time, train.py:62); the engine's graph cache recognises the
static station graph by content, so the CSRs and window plans are not rebuilt per step.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .models import make_loss
from .nn import GINEConv
from .postprocess import PostProcess


class ResGnn(nn.Module):
    """models/gnn.py:10-45 verbatim in structure: the activation and residual stay in torch."""

    def __init__(self, in_channels: int, out_channels: int, num_layers: int,
                 hidden_channels: int):
        super().__init__()
        self.convolutions = nn.ModuleList()
        for _ in range(num_layers):
            mlp = nn.Sequential(nn.Linear(in_channels, hidden_channels),
                                nn.BatchNorm1d(hidden_channels), nn.ReLU(),
                                nn.Linear(hidden_channels, hidden_channels))
            self.convolutions.append(GINEConv(nn=mlp, train_eps=True, edge_dim=1))
        self.relu = nn.ReLU()

    def forward(self, x, edge_index, edge_attr):
        x = x.float()
        edge_attr = edge_attr.float()
        for i, conv in enumerate(self.convolutions):
            if i == 0:
                x = self.relu(conv(x, edge_index, edge_attr))
            else:
                x = x + self.relu(conv(x, edge_index, edge_attr))
        return x


class DeepSetEncoder(nn.Module):
    """models/gnn.py:48-68: phi per member, sum over members, rho (plain torch)."""

    def __init__(self, ensemble_in_dim, hidden_channels, out_channels):
        super().__init__()
        self.phi = nn.Sequential(nn.Linear(ensemble_in_dim, hidden_channels), nn.ReLU(),
                                 nn.Linear(hidden_channels, hidden_channels))
        self.rho = nn.Sequential(nn.Linear(hidden_channels, hidden_channels), nn.ReLU(),
                                 nn.Linear(hidden_channels, out_channels))

    def forward(self, ensemble_feats):
        return self.rho(self.phi(ensemble_feats).sum(dim=1))


class ReferenceStructGNN(nn.Module):
    """models/gnn.py:70-141 with torch layers and the engine's GINEConv."""

    def __init__(self, in_channels, hidden_channels_gnn, out_channels_gnn, num_layers_gnn,
                 loss="MixedLoss", grad_u=False, u=0.5, xi=0.5):
        super().__init__()
        self.loss_fn, self.out_channels = make_loss(loss, grad_u, u, xi)
        self.loss_fn.fused = False   # the reference's torch loss, not the fused kernel
        self.deepset = DeepSetEncoder(in_channels, hidden_channels_gnn, hidden_channels_gnn)
        self.dim_red = nn.Linear(in_channels + hidden_channels_gnn, hidden_channels_gnn)
        self.conv = ResGnn(in_channels=hidden_channels_gnn, hidden_channels=hidden_channels_gnn,
                           out_channels=hidden_channels_gnn, num_layers=num_layers_gnn)
        self.aggr = nn.Linear(out_channels_gnn, self.out_channels)
        self.postprocess = PostProcess(loss, grad_u)

    def forward(self, data):
        emb = self.deepset(data.ensemble)
        h = self.dim_red(torch.cat([data.x, emb], dim=1))
        h = self.conv(h, data.edge_index, data.edge_attr)
        return self.postprocess(self.aggr(h))


def reference_struct_from_params(params: dict, in_channels: int = 35) -> ReferenceStructGNN:
    """train.py:168-179's construction from a params.json dict."""
    return ReferenceStructGNN(in_channels, params["gnn_hidden"], params["gnn_hidden"],
                              params["gnn_layers"], loss=params["loss"],
                              grad_u=params["grad_u"], u=params["u"], xi=params["xi"])
