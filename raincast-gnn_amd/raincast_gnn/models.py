"""The station-graph GNN of models/gnn.py on the MI355X GINE engine.

Structure, constructor arguments and state_dict keys follow models/gnn.py exactly, so a
checkpoint saved by the reference (train.py:203) loads here and vice versa; the only change
is that ``GINEConv`` comes from this package instead of torch_geometric (gnn.py:5), and
ResGnn's outer ReLU / residual add are fused into the last GEMM of each GINE layer.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn import Linear, ModuleList, ReLU

from . import chain as fused_chain
from . import deepset
from . import head as fused_head
from . import options
from .linear import Linear as RowLinear
from .loss import MixedLoss, MixedNormalCRPS, NormalCRPS
from .nn import GINEConv
from .postprocess import PostProcess


class ResGnn(nn.Module):
    """models/gnn.py:10-45: a stack of GINEConv(Linear-BN-ReLU-Linear) with residuals."""

    def __init__(self, in_channels: int, out_channels: int, num_layers: int,
                 hidden_channels: int):
        super().__init__()
        assert num_layers > 0, "num_layers must be > 0."
        self.convolutions = ModuleList()
        out = hidden_channels
        for layer in range(num_layers):
            mlp = nn.Sequential(Linear(in_channels, hidden_channels),
                                nn.BatchNorm1d(hidden_channels), ReLU(),
                                Linear(hidden_channels, out))
            self.convolutions.append(GINEConv(nn=mlp, train_eps=True, edge_dim=1))
            if layer == num_layers - 1:  # kept for parity; has no effect
                out = out_channels
        self.relu = ReLU()

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor,
                edge_attr: torch.Tensor, head=None) -> torch.Tensor:
        """``head``: a head.HeadPlan for the output head that follows (GNN.forward), handed
        to the last layer, whose launch runs it where it can."""
        x = x.float()
        edge_attr = edge_attr.float()
        last = len(self.convolutions) - 1
        for i, conv in enumerate(self.convolutions):
            hp = head if i == last else None
            if i == 0:
                x = conv.forward_relu(x, edge_index, edge_attr, head=hp)        # relu(conv(x))
            else:
                x = conv.forward_residual_relu(x, edge_index, edge_attr, head=hp)  # x + relu(.)
        return x


class DeepSetEncoder(nn.Module):
    """models/gnn.py:48-68: phi per member, sum over members, rho.

    phi's last layer is affine, so ``sum_m (W2 r_m + b2) = W2 (sum_m r_m) + M b2``: the
    member sum is taken before that Linear (same function, same parameters and state_dict
    keys), which shrinks its GEMM -- and its weight-gradient GEMM -- from N*M rows to N rows
    (176,000 -> 16,000 at the 24h_mixed benchmark shape).  On the GPU the remaining
    ``sum_m relu(phi[0](ens_m))`` runs on the fused kernel pair of :mod:`.deepset`.
    """

    def __init__(self, ensemble_in_dim, hidden_channels, out_channels):
        super().__init__()
        self.phi = nn.Sequential(RowLinear(ensemble_in_dim, hidden_channels), nn.ReLU(),
                                 RowLinear(hidden_channels, hidden_channels))
        self.rho = nn.Sequential(RowLinear(hidden_channels, hidden_channels), nn.ReLU(),
                                 RowLinear(hidden_channels, out_channels))

    def forward(self, ensemble_feats):
        lin1, act, lin2 = self.phi
        if isinstance(act, nn.ReLU) and deepset.fusable(ensemble_feats, lin1.weight, lin1.bias):
            r = deepset.phi_sum(ensemble_feats, lin1)                  # fused HIP kernels
        else:
            r = act(lin1(ensemble_feats)).sum(dim=1)                   # [N, H]
        phi_sum = lin2(r, bias_scale=ensemble_feats.size(1))           # = sum_m lin2(r_m)
        return self.rho(phi_sum)


def make_loss(loss: str, grad_u, u, xi):
    """gnn.py:91-103: loss object and number of distribution parameters."""
    if loss == "NormalCRPS":
        return NormalCRPS(), 2
    if loss == "MixedNormalCRPS":
        return MixedNormalCRPS(), 3
    if loss == "MixedLoss":
        if grad_u == "True":
            return MixedLoss(grad_u=True, xi=xi), 5
        return MixedLoss(grad_u=False, u=u, xi=xi), 4
    raise ValueError(f"unknown loss '{loss}'")


class GNN(nn.Module):
    """models/gnn.py:70-141 (the Lightning-style helpers at gnn.py:143-168 are dead code in
    the reference -- nn.Module has no ``log`` -- and are not reproduced)."""

    def __init__(self, in_channels, hidden_channels_gnn, out_channels_gnn, num_layers_gnn,
                 optimizer_class=None, optimizer_params=None, loss="MixedLoss", grad_u=False,
                 u=0.5, xi=0.5):
        super().__init__()
        self.loss, self.grad_u, self.u, self.xi = loss, grad_u, u, xi
        self.loss_fn, self.out_channels = make_loss(loss, grad_u, u, xi)
        self.deepset = DeepSetEncoder(ensemble_in_dim=in_channels,
                                      hidden_channels=hidden_channels_gnn,
                                      out_channels=hidden_channels_gnn)
        self.dim_red = RowLinear(in_channels + hidden_channels_gnn, hidden_channels_gnn)
        self.conv = ResGnn(in_channels=hidden_channels_gnn, hidden_channels=hidden_channels_gnn,
                           out_channels=hidden_channels_gnn, num_layers=num_layers_gnn)
        self.aggr = RowLinear(out_channels_gnn, self.out_channels)
        self.postprocess = PostProcess(self.loss, self.grad_u)
        self.optimizer_class = optimizer_class
        self.optimizer_params = optimizer_params

    def _front(self, data):
        """``dim_red(cat([x, deepset(ensemble)]))`` (gnn.py:132-135); on a HIP device with
        the reference's layer types, the fused member-sum kernels plus the fused dense
        chain (raincast_gnn/chain.py)."""
        ds = self.deepset
        ens, x = data.ensemble, data.x
        lin1, act, lin2 = ds.phi
        rho0, rho_act, rho1 = ds.rho
        lins = (lin2, rho0, rho1, self.dim_red)
        if (isinstance(act, nn.ReLU) and isinstance(rho_act, nn.ReLU)
                and deepset.fusable(ens, lin1.weight, lin1.bias)):
            if (fused_chain.FOLD and fused_chain.F3
                    and (fused_chain.FOLD2 or ens.size(0) <= fused_chain.F3_MAX_NODES)
                    and fused_chain.fusable_dims(lin1.out_features, x, lins)):
                # the DeepSet launch also folds dim_red; the chain forward is one launch
                fold = ((rho1, self.dim_red, rho0, lin2) if fused_chain.FOLD2
                        else (rho1, self.dim_red))
                r, wfold = deepset.phi_sum(ens, lin1, fold=fold)
                return fused_chain.chain(r, x, lins, ens.size(1), wfold=wfold)
            r = deepset.phi_sum(ens, lin1)
            if fused_chain.fusable(r, x, lins):
                return fused_chain.chain(r, x, lins, ens.size(1))
            emb = ds.rho(lin2(r, bias_scale=ens.size(1)))
            return self.dim_red(torch.cat([x, emb], dim=1))
        emb = ds(ens)
        return self.dim_red(torch.cat([x, emb], dim=1))

    def forward(self, data):
        h = self._front(data)
        kind = fused_head.loss_kind(self.postprocess.loss, self.postprocess.grad_u)
        y = getattr(data, "y", None)
        hplan = None
        if (options.HEAD_FOLD and self.training and type(self.aggr) in (RowLinear, Linear)
                and fused_head.fusable(h, self.aggr, kind)):
            # the head's forward folded into the last GINE layer's launch (gine_layer_head;
            # training mode: the one-launch layer runs on batch statistics only)
            hplan = fused_head.plan(h, self.aggr, kind, y)
        h = self.conv(h, data.edge_index, data.edge_attr, head=hplan)
        if type(self.aggr) in (RowLinear, Linear) and fused_head.fusable(h, self.aggr, kind):
            # aggr + PostProcess in one kernel, which also counts the loss's valid targets
            return fused_head.head(h, self.aggr, kind, y, hplan)
        return self.postprocess(self.aggr(h))

    def configure_optimizers(self):
        return self.optimizer_class(self.parameters(), **self.optimizer_params)


def gnn_from_params(params: dict, in_channels: int = 35, **overrides) -> GNN:
    """Build the model the way train.py:168-179 does from a params.json dict."""
    cfg = dict(params)
    cfg.update(overrides)
    return GNN(in_channels=in_channels, hidden_channels_gnn=cfg["gnn_hidden"],
               out_channels_gnn=cfg["gnn_hidden"], num_layers_gnn=cfg["gnn_layers"],
               optimizer_class=torch.optim.AdamW, optimizer_params={"lr": cfg["lr"]},
               loss=cfg["loss"], grad_u=cfg["grad_u"], u=cfg["u"], xi=cfg["xi"])
