"""ORACLE -- test infrastructure only.  CPU restatement of the reference's hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``raincast_gnn``) never imports it and has no CPU fallback.

What is restated, and from where
--------------------------------
* GINEConv (torch_geometric, NOT vendored in /root/reference and not installed here;
  environment.yml:31 leaves it unpinned, README.md:73 says "2.3.1+"; the semantics below
  are identical across 2.3-2.6).  Its published algorithm, in the ATen ops PyG dispatches
  to on CPU for a plain-Tensor ``edge_index`` and ``aggr='add'``:
    - ``MessagePassing._collect``:   ``x_j = x.index_select(0, edge_index[0])``
    - ``GINEConv.message``:          ``(x_j + self.lin(edge_attr)).relu()``, lin = Linear(1, D)
    - ``SumAggregation`` -> ``utils.scatter(reduce='sum')``:
                                     ``x.new_zeros(N, D).scatter_add_(0, index.expand, m)``
    - ``GINEConv.forward``:          ``out = out + (1 + self.eps) * x_r; return self.nn(out)``
  Call sites anchoring it: models/gnn.py:5 (import), :28 (construction), :41,44 (calls).
* ResGnn / DeepSetEncoder / GNN: models/gnn.py:10-141.
* PostProcess: models/model_utils.py:42-113.   Losses: models/loss.py:6-68, 71-272, 335-369.
* Graph layout: utils/data.py:261-284 (``build_edge_index_and_attr``).

Pinning
-------
* GINE path: **parity unpinned** -- the reference ships no test, fixture or golden vector
  for GINEConv and torch_geometric cannot be imported here.  The
  restatement is cross-checked against an independent per-edge Python loop
  (:func:`gine_aggregate_loops`) and its CPU summation order is verified in tests.
* PostProcess and the CRPS losses: pinned -- ``tests/golden/reference_heads.npz`` holds
  outputs of the reference's own models/model_utils.py and models/loss.py, generated in the
  build container by ``tests/golden/make_reference_heads.py``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------
# GINEConv (PyG semantics)
# ---------------------------------------------------------------------------------------


def tie_relu(v, decide=None, **ctx):
    """relu(v); with ``decide`` (a callable ``decide(v, **ctx) -> bool mask``) the ReLU keeps
    ``v`` where the mask is set instead of where ``v > 0``.  The hook of the tie-break oracle
    (tests/helpers.EngineTies): an fp64 restatement that follows another implementation's
    ReLU decisions after checking that each one that differs from ``v > 0`` lies within that
    implementation's forward rounding bound of zero -- the exact gradient of the branch the
    implementation took.  ``ctx`` carries the operands the bound is computed from."""
    if decide is None:
        return v.relu()
    keep = decide(v, **ctx)
    return v * keep.to(v.dtype)


def gine_aggregate(x, edge_index, edge_attr, lin_w, lin_b, eps, decide=None, record=None):
    """z = scatter_add(relu(x[src] + lin(a)), dst) + (1 + eps) * x  (PyG op sequence).
    ``record`` (tests): a dict that receives "dpre" = d loss / d (x_j + lin(a)) in backward."""
    src, dst = edge_index[0], edge_index[1]
    x_j = x.index_select(0, src)
    e = F.linear(edge_attr.reshape(-1, lin_w.size(1)), lin_w, lin_b)
    pre = x_j + e
    if record is not None and pre.requires_grad:
        pre.register_hook(lambda g: record.__setitem__("dpre", g.detach()))
    m = tie_relu(pre, decide, x=x, src=src, edge_attr=edge_attr)
    agg = x.new_zeros(x.size(0), m.size(1)).scatter_add_(0, dst.view(-1, 1).expand_as(m), m)
    return agg + (1 + eps) * x


def gine_aggregate_loops(x, edge_index, edge_attr, lin_w, lin_b, eps, rounding="fma"):
    """Independent per-edge restatement (small inputs only): sequential float32 sums in
    original edge order (np.float32 arithmetic per element).  ``rounding`` is how the host's
    CPU Linear(1, D) rounds a*w+b: "fma" (one rounding; MKL on Intel) or "muladd" (two;
    MKL on AMD EPYC) -- see tools/probe_cpu_rounding.py."""
    xn = x.detach().numpy().astype(np.float32)
    ei = edge_index.numpy()
    a = edge_attr.detach().reshape(-1).numpy().astype(np.float32)
    w = lin_w.detach().reshape(-1).numpy().astype(np.float32)
    b = lin_b.detach().reshape(-1).numpy().astype(np.float32)
    ope = np.float32(1) + np.float32(eps.detach().reshape(-1)[0].item())
    N, D = xn.shape
    agg = np.zeros((N, D), dtype=np.float32)
    for e in range(ei.shape[1]):
        s, d = ei[0, e], ei[1, e]
        if rounding == "fma":
            lin = (np.float64(a[e]) * np.float64(w) + np.float64(b)).astype(np.float32)
        else:
            lin = ((a[e] * w).astype(np.float32) + b).astype(np.float32)
        pre = (xn[s] + lin).astype(np.float32)
        m = np.where(pre > 0, pre, np.float32(0)).astype(np.float32)
        agg[d] = (agg[d] + m).astype(np.float32)
    return torch.from_numpy((agg + (ope * xn).astype(np.float32)).astype(np.float32))


class OracleGINEConv(nn.Module):
    """CPU GINEConv with PyG's attributes and state_dict keys (nn.*, eps, lin.*)."""

    def __init__(self, nn_module, eps=0.0, train_eps=False, edge_dim=None):
        super().__init__()
        self.nn = nn_module
        self.initial_eps = eps
        if train_eps:
            self.eps = nn.Parameter(torch.empty(1))
        else:
            self.register_buffer("eps", torch.empty(1))
        self.lin = None
        if edge_dim is not None:
            first = self.nn[0] if isinstance(self.nn, nn.Sequential) else self.nn
            self.lin = nn.Linear(edge_dim, first.in_features)
        self.eps.data.fill_(eps)

    record = None  # tests may set a dict: "z" -> (x, d z), "a1" -> d a1, "dpre" -> d message
    #                pre-activation, filled during backward
    decide = None  # tests may set {"msg" | "bn" | "res": callable} (see tie_relu)
    last_r = None  # the ReLU output of the node MLP (the "res" hook's operand)

    def _decide(self, key):
        return None if self.decide is None else self.decide.get(key)

    def aggregate(self, x, edge_index, edge_attr):
        z = gine_aggregate(x, edge_index, edge_attr, self.lin.weight, self.lin.bias, self.eps,
                           self._decide("msg"), self.record)
        if self.record is not None and z.requires_grad:
            xd = x.detach()
            z.register_hook(lambda g: self.record.__setitem__("z", (xd, g.detach())))
        return z

    def forward(self, x, edge_index, edge_attr):
        z = self.aggregate(x, edge_index, edge_attr)
        if self.decide is None and self.record is None:
            return self.nn(z)
        l1, bn, _, l2 = self.nn
        a1 = l1(z)
        if self.record is not None and a1.requires_grad:
            a1.register_hook(lambda g: self.record.__setitem__("a1", g.detach()))
        r = tie_relu(bn(a1), self._decide("bn"), a1=a1, z=z)
        self.last_r = r
        return l2(r)


class OracleResGnn(nn.Module):
    """models/gnn.py:10-45 on OracleGINEConv."""

    def __init__(self, in_channels, out_channels, num_layers, hidden_channels):
        super().__init__()
        self.convolutions = nn.ModuleList()
        for _ in range(num_layers):
            mlp = nn.Sequential(nn.Linear(in_channels, hidden_channels),
                                nn.BatchNorm1d(hidden_channels), nn.ReLU(),
                                nn.Linear(hidden_channels, hidden_channels))
            self.convolutions.append(OracleGINEConv(mlp, train_eps=True, edge_dim=1))
        self.relu = nn.ReLU()

    def forward(self, x, edge_index, edge_attr):
        # models/gnn.py:36-37 casts to fp32; the fp64 tie-break copy keeps its own dtype
        dt = self.convolutions[0].lin.weight.dtype
        x = x.to(dt)
        edge_attr = edge_attr.to(dt)
        for i, conv in enumerate(self.convolutions):
            o = conv(x, edge_index, edge_attr)
            h = tie_relu(o, conv._decide("res"), r=conv.last_r)
            x = h if i == 0 else x + h
        return x


class OracleDeepSet(nn.Module):
    decide = None  # tests may set {"phi" | "rho": callable} (see tie_relu)

    def __init__(self, d_in, hidden, out):
        super().__init__()
        self.phi = nn.Sequential(nn.Linear(d_in, hidden), nn.ReLU(), nn.Linear(hidden, hidden))
        self.rho = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU(), nn.Linear(hidden, out))

    def forward(self, ens):
        if self.decide is None:
            return self.rho(self.phi(ens).sum(dim=1))
        p0, _, p2 = self.phi
        r0, _, r2 = self.rho
        hp = tie_relu(p0(ens), self.decide.get("phi"))
        s = p2(hp).sum(dim=1)
        # r (the member sum of phi's hidden layer): the doubly folded engine's rho[0] input
        return r2(tie_relu(r0(s), self.decide.get("rho"), s=s, r=hp.sum(dim=1)))


# ---------------------------------------------------------------------------------------
# Heads: PostProcess and CRPS losses (reference semantics, boolean-mask NaN handling)
# ---------------------------------------------------------------------------------------
_EPS = 1e-6


def postprocess(x, loss, grad_u):
    cols = list(torch.split(x, 1, dim=-1))
    if loss == "NormalCRPS":
        cols[1] = F.softplus(cols[1]) + _EPS
    elif loss == "MixedNormalCRPS":
        cols[1] = F.softplus(cols[1]) + _EPS
        cols[2] = torch.sigmoid(cols[2])
    elif loss == "MixedLoss":
        cols[1] = F.softplus(cols[1]) + _EPS
        cols[2] = torch.sigmoid(cols[2])
        cols[3] = F.softplus(cols[3]) + _EPS
        if grad_u == "True":
            cols[4] = torch.sigmoid(cols[4]) * 2.12
    return torch.cat(cols, dim=-1)


def _Phi(v):
    return torch.distributions.Normal(loc=0, scale=1).cdf(v)


def _phi(v):
    return torch.distributions.Normal(loc=0, scale=1).log_prob(v).exp()


def crps_normal(pred, y):
    keep = ~torch.isnan(y)
    mu, sigma = (t[keep] for t in torch.split(pred, 1, dim=1))
    yy = y.unsqueeze(1)[keep]
    z = (yy - mu) / sigma
    inv_sqrt_pi = 1 / torch.sqrt(torch.tensor(np.pi))
    dist = torch.distributions.Normal(loc=0.0, scale=1.0)
    val = sigma * (z * (2.0 * dist.cdf(z) - 1.0) + 2.0 * torch.exp(dist.log_prob(z)) - inv_sqrt_pi)
    return val.mean()


def crps_mixed_normal(pred, y, c=np.log(0.01)):
    keep = ~torch.isnan(y)
    mu, sigma, p = (t[keep] for t in torch.split(pred, 1, dim=1))
    yy = y.unsqueeze(1)[keep]
    ct = (torch.tensor([c]) - mu) / sigma
    yt = (yy - mu) / sigma
    mass_c = p + (1 - p) * _Phi(ct)
    body = (yt * (2 * (p + (1 - p) * _Phi(yt)) - 1) - ct * mass_c ** 2
            - 2 * (1 - p) * _phi(ct) * mass_c + 2 * (1 - p) * _phi(yt)
            - (1 - p) ** 2 / math.sqrt(math.pi) * (1 - _Phi(math.sqrt(2) * ct)))
    return (sigma * body).mean()


def _gpd_crps(y, u, m, s, xi):
    t = (y - u) / s
    G = torch.where(t <= 0, 0, 1 - (1 + xi * t).pow(-1 / xi))
    return s * (t.abs() - 2 * (1 - m) / (1 - xi) * (1 - (1 - G).pow(1 - xi))
                + (1 - m) ** 2 / (2 - xi))


def crps_mixed(pred, y, grad_u, u=None, xi=0.5, t=5, c=np.log(0.01)):
    keep = ~torch.isnan(y)
    cols = torch.split(pred, 1, dim=1)
    if grad_u:
        mu, sigma, p, su, uu = (v[keep] for v in cols)
    else:
        mu, sigma, p, su = (v[keep] for v in cols)
        uu = torch.tensor([u])
    yy = y.unsqueeze(1)[keep].to(pred.dtype)
    xit = torch.tensor([xi])
    ct = (torch.tensor([c]) - mu) / sigma
    ut = (uu - mu) / sigma
    yt = (yy - mu) / sigma
    m_u = p + (1 - p) * _Phi(ut)
    mass_c = p + (1 - p) * _Phi(ct)
    mass_u = (1 - p) * (1 - _Phi(ut))
    shared = (-ct * mass_c ** 2 + ut * mass_u ** 2
              - 2 * (1 - p) * _phi(ct) * mass_c - 2 * (1 - p) * _phi(ut) * mass_u
              - (1 - p) ** 2 / math.sqrt(math.pi) * (_Phi(math.sqrt(2) * ut)
                                                      - _Phi(math.sqrt(2) * ct)))
    below = sigma * (yt * (2 * (p + (1 - p) * _Phi(yt)) - 1) + 2 * (1 - p) * _phi(yt) + shared)
    above = sigma * (ut + 2 * ((1 - p) * _phi(ut) - ut * mass_u) + shared)
    loss_1 = below + _gpd_crps(uu, uu, m_u, su, xit)
    loss_2 = _gpd_crps(yy, uu, m_u, su, xit) + above
    if grad_u:
        val = torch.sigmoid((uu - yy) * t) * (loss_1 - loss_2) + loss_2
    else:
        val = torch.where(yy < uu, loss_1, loss_2)
    return val.mean()


def make_crps(loss, grad_u, u, xi):
    if loss == "NormalCRPS":
        return crps_normal, 2
    if loss == "MixedNormalCRPS":
        return crps_mixed_normal, 3
    if grad_u == "True":
        return (lambda pr, y: crps_mixed(pr, y, True, xi=xi)), 5
    return (lambda pr, y: crps_mixed(pr, y, False, u=u, xi=xi)), 4


class OracleGNN(nn.Module):
    """models/gnn.py:70-141 on CPU; state_dict keys identical to the reference."""

    def __init__(self, in_channels, hidden, num_layers, loss="MixedLoss", grad_u="False",
                 u=1.71, xi=0.5):
        super().__init__()
        self.loss, self.grad_u = loss, grad_u
        self.crps, out = make_crps(loss, grad_u, u, xi)
        self.deepset = OracleDeepSet(in_channels, hidden, hidden)
        self.dim_red = nn.Linear(in_channels + hidden, hidden)
        self.conv = OracleResGnn(hidden, hidden, num_layers, hidden)
        self.aggr = nn.Linear(hidden, out)

    def forward(self, data):
        h = self.dim_red(torch.cat([data.x, self.deepset(data.ensemble)], dim=1))
        h = self.conv(h, data.edge_index, data.edge_attr)
        return postprocess(self.aggr(h), self.loss, self.grad_u)
