"""GPU: the one-launch layer forward with LDS staging of every tile's neighbour rows
(gine_mp_fwd_layer with the layer window plan, csrc/gine_mpmlp.hip WIN; north star:
"per-destination-node LDS staging of neighbour features") against the same launch gathering
from L2 and against the two-launch pair.

The window form sums the same messages in the same edge order (gine_edge.hpp), splits z into
the same planes and runs the same chains and epilogues, so every output is the same bits: y,
the ReLU mask, z, a1, bn_save, the running statistics and the gradients of the backward that
follows -- also with non-finite inputs (the fp32 redo of a NaN tile reads z back from HBM).
Reference: models/gnn.py:41,44 (GINEConv.propagate + nn), PyG's x.index_select per edge.
"""
import ctypes

import numpy as np
import pytest
import torch

from raincast_gnn import GINEConv, _lib, options
from raincast_gnn.data import relabel_edges, station_order
from raincast_gnn.graph import GineGraph

from helpers import knn_batch_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _python_binding(monkeypatch):
    from raincast_gnn import nn as rnn
    monkeypatch.setattr(rnn, "USE_TORCH_EXT", False)


def _local_graph(nodes, k, graphs, seed):
    """``graphs`` copies of one station graph, stations in the locality order (what
    raincast_gnn.data.DeviceDataset / bench.py run)."""
    ei, ea, n = knn_batch_graph(nodes, k, graphs, seed=seed)
    ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // graphs], nodes))
    return ei, ea, n


def _plan_numpy(ei, n):
    src, dst = ei[0].numpy(), ei[1].numpy()
    tiles = (n + 31) // 32
    own_lo = np.arange(tiles) * 32
    own_hi = np.minimum(own_lo + 31, n - 1)
    lo, hi = own_lo.copy(), own_hi.copy()
    t = dst // 32
    np.minimum.at(lo, t, src)
    np.maximum.at(hi, t, src)
    edges = np.bincount(t, minlength=tiles)
    return np.stack([lo, hi - lo + 1], 1), int((hi - lo + 1).max()), int(edges.max())


@pytest.mark.parametrize("nodes,k,graphs", [(500, 10, 32), (120, 6, 3), (97, 5, 1)],
                         ids=["cfg2", "small", "odd-N"])
def test_layer_window_plan_matches_numpy(nodes, k, graphs):
    ei, ea, n = _local_graph(nodes, k, graphs, seed=7)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    want, rows, edges = _plan_numpy(ei, n)
    ok = ctypes.c_int32(0)
    _lib.call("gine_mp_fwd_layer_windows_fit", rows, g.max_in_degree, ctypes.byref(ok))
    if not ok.value:  # a tile's window beyond the launch's LDS: no plan, the L2 gather
        assert g.layer_windows is None
        return
    win, r, e = g.layer_windows
    assert (r, e) == (rows, edges)
    assert np.array_equal(win.cpu().numpy(), want)
    if nodes == 500:
        assert edges == 32 * (k + 1)


def test_layer_window_plan_refused_when_it_does_not_fit():
    # dataset order: a tile's neighbours span the whole 500-station graph
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=3)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    assert g.layer_windows is None


def _conv(seed):
    torch.manual_seed(seed)
    D = 128
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    with torch.no_grad():
        mlp[1].weight.uniform_(0.5, 1.5)
        mlp[1].bias.uniform_(-0.2, 0.2)
    return conv.to(DEV).train()


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t


def _run(conv, state, x, ei, ea, epilogue, form, monkeypatch):
    """One forward + backward in `form`: "win" (layer, windows), "l2" (layer, gather from
    L2) or "pair" (two launches)."""
    conv.load_state_dict(state)
    monkeypatch.setattr(options, "LAYER_FWD", form != "pair")
    monkeypatch.setattr(options, "LAYER_WIN", form == "win")
    fn = {"none": conv.forward, "relu": conv.forward_relu,
          "residual": conv.forward_residual_relu}[epilogue]
    xi = x.clone().requires_grad_(True)
    y = fn(xi, ei, ea)
    saved = [t.detach().clone() for t in y.grad_fn.saved_tensors[:6] if t is not None]
    (torch.nan_to_num(y) * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum() \
        .backward()
    grads = [xi.grad.clone()] + [p.grad.clone() for p in conv.parameters()]
    conv.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    bn = conv.nn[1]
    return ([y.detach().clone()] + saved + grads
            + [bn.running_mean.clone(), bn.running_var.clone()])


@pytest.mark.parametrize("nodes,k,graphs", [(500, 10, 32), (120, 6, 3)], ids=["cfg2", "small"])
@pytest.mark.parametrize("epilogue", ["none", "relu", "residual"])
def test_layer_window_form_same_bits_as_gather_and_pair(nodes, k, graphs, epilogue,
                                                        monkeypatch):
    ei, ea, n = _local_graph(nodes, k, graphs, seed=nodes + k)
    eid, ead = ei.to(DEV), ea.to(DEV)
    conv = _conv(seed=k)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    x = torch.randn(n, 128, device=DEV) * 1.5 + 0.2
    from raincast_gnn.graph import get_graph
    assert get_graph(eid, ead, n).layer_windows is not None
    ref = _run(conv, state, x, eid, ead, epilogue, "pair", monkeypatch)
    for form in ("win", "l2", "win"):   # interleaved on one accumulator (pairing carries)
        got = _run(conv, state, x, eid, ead, epilogue, form, monkeypatch)
        for a, b in zip(got, ref):
            assert torch.equal(_bits(a), _bits(b)), form


def test_layer_window_form_nonfinite_inputs(monkeypatch):
    """+-inf and NaN feature entries: the tiles that see them take the fp32 redo in both
    forms (the window form reads z back from memory); NaN / inf land in the same places with
    the same bits."""
    ei, ea, n = _local_graph(500, 10, 8, seed=21)
    eid, ead = ei.to(DEV), ea.to(DEV)
    conv = _conv(seed=4)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    x = torch.randn(n, 128, device=DEV)
    x[17, 5] = float("inf")
    x[1200, 77] = float("-inf")
    x[3001, 100] = float("nan")
    ref = _run(conv, state, x, eid, ead, "residual", "l2", monkeypatch)
    got = _run(conv, state, x, eid, ead, "residual", "win", monkeypatch)
    assert torch.isnan(got[0]).any()
    for a, b in zip(got, ref):
        assert torch.equal(_bits(a), _bits(b))
