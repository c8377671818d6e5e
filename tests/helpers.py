"""Shared graph builders and comparison helpers for the test-suite."""
from __future__ import annotations

import numpy as np
import torch

from raincast_gnn import data as rdata


def knn_batch_graph(n: int, k: int, batch: int = 1, seed: int = 0):
    ei, ea = rdata.station_graph(n, k=k, seed=seed)
    eis = [ei + g * n for g in range(batch)]
    return torch.cat(eis, 1), torch.cat([ea] * batch), n * batch


def radius_graph(n: int, max_dist: float, seed: int = 0):
    lat, lon = rdata.synthetic_stations(n, seed)
    ei, ea = rdata.build_edge_index_and_attr(rdata.haversine_matrix(lat, lon), max_dist)
    return ei, ea, n


def random_graph(n: int, e: int, seed: int = 0, skew: bool = True):
    """Unsorted multigraph with hub sources (power-law out-degree) and isolated nodes."""
    rng = np.random.default_rng(seed)
    if skew:
        w = 1.0 / np.arange(1, n + 1) ** 1.2
        src = rng.choice(n, size=e, p=w / w.sum())
    else:
        src = rng.integers(0, n, e)
    dst = rng.integers(0, max(n - 2, 1), e)  # last nodes never receive: isolated targets
    ei = torch.tensor(np.stack([src, dst]), dtype=torch.long)
    ea = torch.from_numpy(rng.uniform(0.5, 4.0, (e, 1)).astype(np.float32))
    return ei, ea, n


def special_graphs():
    """(name, edge_index, edge_attr, num_nodes) edge cases the reference can produce."""
    out = []
    ei, ea, n = knn_batch_graph(64, 4, 1, seed=3)
    out.append(("knn64_k4", ei, ea, n))
    ei, ea, n = knn_batch_graph(500, 10, 2, seed=0)
    out.append(("knn500_k10_b2", ei, ea, n))
    # max_dist=1 (trained_models/24h_normal_mixed/params.json:6): self-loops only
    ei, ea, n = radius_graph(50, 1.0, seed=1)
    out.append(("selfloops_only", ei, ea, n))
    ei, ea, n = radius_graph(80, 150.0, seed=2)
    out.append(("radius80_150km", ei, ea, n))
    out.append(("no_edges", torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, 1), 7))
    ei, ea, n = random_graph(200, 3000, seed=4)
    out.append(("hubs_unsorted", ei, ea, n))
    ei, ea, n = random_graph(1, 5, seed=5, skew=False)
    out.append(("single_node_multi_loops", torch.zeros(2, 5, dtype=torch.long), ea, 1))
    return out


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.abs().max().item()
    num = (a - b).abs().max().item()
    if den == 0.0:
        return num
    return num / den


def assert_close_tiebreak(gpu, cpu32, cpu64, tol=1e-5, name="", gpu64=None):
    """GPU vs CPU fp32 oracle within ``tol`` (max-norm relative); if not, the GPU must be at
    least as close to the fp64 oracle as the fp32 CPU oracle is (x2 slack).  ``gpu64``: the
    fp64 oracle on the engine's side of the ReLU ties (check_training_step), which the GPU is
    measured against instead of ``cpu64``."""
    e32 = rel_err(gpu, cpu32)
    if e32 <= tol:
        return e32
    e_gpu = rel_err(gpu, cpu64 if gpu64 is None else gpu64)
    e_cpu = rel_err(cpu32, cpu64)
    assert e_gpu <= max(tol, 2.0 * e_cpu), (
        f"{name}: rel err vs cpu32 {e32:.3e}, gpu vs fp64 {e_gpu:.3e}, cpu32 vs fp64 {e_cpu:.3e}")
    return e32


# ---------------------------------------------------------------------------------------
# full training step vs the oracle (GPU tests)
# ---------------------------------------------------------------------------------------
def _oracle_step(ref, batch, dtype, record=False, decide=None):
    import copy
    r = copy.deepcopy(ref).to(dtype)
    if record:
        for conv in r.conv.convolutions:
            conv.record = []
    if decide is not None:
        for conv, d in zip(r.conv.convolutions, decide):
            conv.decide = d
    b = copy.copy(batch)
    b.x, b.ensemble, b.edge_attr = (t.to(dtype) for t in (batch.x, batch.ensemble,
                                                          batch.edge_attr))
    pred = r(b)
    loss = r.crps(pred, batch.y)
    loss.backward()
    return r, pred, loss


def fro_rel(a: torch.Tensor, b: torch.Tensor) -> float:
    """Frobenius-norm relative error ||a - b|| / ||b||."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.norm().item()
    return (a - b).norm().item() / den if den else (a - b).norm().item()


TIE_BAND = 1e-5


def capture_engine_layers(model):
    """Wrap the engine's GINE layers so that each layer's output (whose autograd node holds
    the layer's saved tensors) is kept until ``engine_decisions`` reads it."""
    outs = []
    for conv in model.conv.convolutions:
        for nm in ("forward_relu", "forward_residual_relu"):
            def wrapped(*a, _fn=getattr(conv, nm), **k):
                y = _fn(*a, **k)
                outs.append(y)
                return y
            setattr(conv, nm, wrapped)
    return outs


def engine_decisions(outs, model, batch, log):
    """The engine's ReLU decisions in each GINE layer, restated exactly from the tensors its
    forward saved (raincast_gnn/functional.py: x, z, a1, y, mask, bn_save): the messages
    x_j + lin(a) > 0 (lin by the host's CPU Linear, whose rounding the kernels match --
    functional.edge_linear_flag), the BatchNorm-ReLU a1 * alpha + shift > 0 (gine_mlpsrc.hpp
    bn_apply) and the output ReLU (the saved residual mask, or y > 0 in layer 0).  As
    ``decide`` dicts for the oracle's tie_relu, with band TIE_BAND."""
    import torch.nn.functional as F
    src = batch.edge_index[0].cpu()
    ea = batch.edge_attr.float().cpu().reshape(-1, 1)
    out = []
    for conv, y in zip(model.conv.convolutions, outs):
        x, _, a1, ys, mask, bn_save = (t.detach().cpu() if t is not None else None
                                       for t in y.grad_fn.saved_tensors[:6])
        lw = conv.lin.weight.detach().float().cpu()
        lb = conv.lin.bias.detach().float().cpu()
        msg = (x.index_select(0, src) + F.linear(ea, lw, lb)) > 0
        bn = (a1 * bn_save[2] + bn_save[3]) > 0
        res = mask.bool() if mask is not None else ys > 0
        out.append({"msg": (msg, TIE_BAND, log), "bn": (bn, TIE_BAND, log),
                    "res": (res, TIE_BAND, log)})
    return out


def engine_order_batch(batch):
    """``batch`` (B collated copies of one station graph) relabelled into the engine's
    locality order (raincast_gnn.data.station_order / relabel_stations)."""
    from raincast_gnn.data import relabel_stations, station_order
    n = batch.num_nodes // batch.num_graphs
    e1 = batch.edge_index.size(1) // batch.num_graphs   # graph 0's edges come first
    return relabel_stations(batch, station_order(batch.edge_index[:, :e1], n))


def check_training_step(params, batch, dev, tol=1e-5, seed=42, envelope_threads=None,
                        relabel=False):
    """One training step (DeepSet + dim_red + GINE stack + head + PostProcess + loss +
    backward) of the engine's GNN on ``dev`` against the CPU oracle with the same weights.

    Predictions, loss and the BatchNorm running statistics: within ``tol`` (max-norm
    relative) of the fp32 oracle, fp64 oracle as tie-break.

    Gradients, default (small batches): every parameter gradient within ``tol`` of the fp32
    oracle, fp64 tie-break.  Linear1's bias gradient is analytically zero (train-mode BN
    follows it), so it always goes through the tie-break.  ``d eps = sum dz*x`` is one
    cancelling reduction over N*D terms, ill-conditioned in any fp32 implementation: it is
    checked as |gpu - exact| <= tol * sum |dz*x| with the fp64 oracle as exact.

    ReLU ties (default mode): a decision whose fp64 pre-activation lies within
    TIE_BAND * max|pre| of zero -- within fp32 rounding -- can go either way in any fp32
    implementation, and one such decision moves one gradient entry by the whole upstream
    gradient (e.g. one message x_j + lin(a) of 3e-7 in a GINE layer: 6e-4 on that layer's
    lin.bias gradient, 2e-5 on the DeepSet's).  The engine's decisions are restated from the
    tensors its forward saved (engine_decisions) and the fp64 tie-break oracle takes the
    engine's side of every tie (oracle.gine_cpu.tie_relu); decisions outside the band stay
    the oracle's own, and at most 1e-5 of all decisions may be adopted.

    Gradients, ``envelope_threads`` given (benchmark-size batches): at 10^4-10^5 nodes a step
    makes ~10^8 ReLU decisions, and the ones whose fp32 pre-activation lies within rounding
    of zero go either way in ANY fp32 implementation -- the forward barely notices (ReLU is
    continuous) but each such decision switches one gradient entry between 0 and the
    upstream gradient.  The reference restatement itself, run with 1 thread and with all
    threads, then differs from the exact gradient by 1e-4..5e-3 (tools/diag_grads.py,
    DESIGN.md 4).  There the bar is the reference's own envelope: for every parameter,
    ||gpu - fp64|| / ||fp64|| <= max(tol, 2 * the largest such error of the fp32 oracle over
    the thread counts ``envelope_threads``).
    ``relabel``: the engine runs the batch in its locality order (engine_order_batch) and
    its predictions are mapped back to the collated order; the oracle runs the reference
    order.
    Returns the worst relative gradient error against the fp32 oracle."""
    from oracle import gine_cpu as O
    from raincast_gnn.models import GNN
    torch.manual_seed(seed)
    model = GNN(35, params["gnn_hidden"], params["gnn_hidden"], params["gnn_layers"],
                loss=params["loss"], grad_u=params["grad_u"], u=params["u"], xi=params["xi"])
    ref = O.OracleGNN(35, params["gnn_hidden"], params["gnn_layers"], params["loss"],
                      params["grad_u"], params["u"], params["xi"])
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()},
                        strict=True)
    model = model.to(dev).train()
    from raincast_gnn.data import restore_node_order
    gb = engine_order_batch(batch) if relabel else batch
    layer_outs = None if relabel else capture_engine_layers(model)
    pred = model(gb.to(dev))
    loss = model.loss_fn.crps(pred, gb.y.to(dev))
    ties = []
    decide = None if relabel else engine_decisions(layer_outs, model, batch, ties)
    layer_outs = None
    loss.backward()
    pred = restore_node_order(pred, gb)
    r32, pred32, loss32 = _oracle_step(ref, batch, torch.float32)
    r64, pred64, loss64 = _oracle_step(ref, batch, torch.float64, record=True)
    # the fp64 oracle on the engine's side of every decision within fp32 rounding of zero
    # (oracle.gine_cpu.tie_relu): the exact gradient of the branch the engine took
    p64e = p64t = None
    if decide is not None:
        r64t = _oracle_step(ref, batch, torch.float64, decide=decide)[0]
        p64t = dict(r64t.named_parameters())
        n_dec = sum(d["msg"][0].numel() + d["bn"][0].numel() + d["res"][0].numel()
                    for d in decide)
        adopted = sum(ties)
        assert adopted <= 1e-5 * n_dec, f"{adopted} tie decisions of {n_dec}"
        if adopted:
            print(f"engine took the other side of {adopted} ReLU ties (|pre| <= "
                  f"{TIE_BAND} max|pre|) of {n_dec} decisions")
    assert loss.dtype == loss32.dtype
    assert pred.shape == pred32.shape
    assert_close_tiebreak(pred.detach().cpu(), pred32.detach(), pred64.detach(), tol, "pred")
    assert_close_tiebreak(loss.detach().cpu().reshape(1), loss32.detach().reshape(1),
                          loss64.detach().reshape(1), tol, "loss")
    p32, p64 = dict(r32.named_parameters()), dict(r64.named_parameters())
    p64e = p64t if p64t is not None else p64
    worst = 0.0
    if envelope_threads:
        runs = [p32]
        nthr = torch.get_num_threads()
        try:
            for t in envelope_threads:
                if t != nthr:
                    torch.set_num_threads(t)
                    runs.append(dict(_oracle_step(ref, batch, torch.float32)[0]
                                     .named_parameters()))
        finally:
            torch.set_num_threads(nthr)
        for name, p in model.named_parameters():
            exact = p64[name].grad
            if name.endswith(".nn.0.bias"):   # analytically zero: compare absolute sizes
                assert p.grad.abs().max() <= 2 * max(r[name].grad.abs().max() for r in runs)
                continue
            env = max(fro_rel(r[name].grad, exact) for r in runs)
            e = fro_rel(p.grad, exact)
            bar = tol
            if name.endswith(".eps"):  # a cancelling reduction: its condition scale too
                i = int(name.split(".")[2])
                x64, dz64 = r64.conv.convolutions[i].record[0]
                bar = tol * (dz64 * x64).abs().sum().item() / max(exact.abs().item(), 1e-300)
            assert e <= max(bar, 2.0 * env), (
                f"{name}: gpu vs fp64 {e:.3e} > max({bar:.3e}, 2 x reference envelope "
                f"{env:.3e})")
            worst = max(worst, rel_err(p.grad, p32[name].grad))
    else:
        for name, p in model.named_parameters():
            if name.endswith(".eps"):
                i = int(name.split(".")[2])
                x64, dz64 = r64.conv.convolutions[i].record[0]
                scale = (dz64 * x64).abs().sum().item()
                err = abs(p.grad.item() - p64e[name].grad.item())
                assert err <= tol * scale, f"{name}: |err| {err:.3e} > {tol} * {scale:.3e}"
                continue
            e = assert_close_tiebreak(p.grad.cpu(), p32[name].grad, p64[name].grad, tol, name,
                                      p64e[name].grad)
            worst = max(worst, e)
    # BatchNorm running statistics after the step (train mode updates them once)
    for (name, buf), (rname, rbuf) in zip(model.named_buffers(), r32.named_buffers()):
        assert name == rname
        if buf.dtype.is_floating_point:
            torch.testing.assert_close(buf.cpu(), rbuf, rtol=tol, atol=tol, msg=name)
        else:
            assert torch.equal(buf.cpu(), rbuf), name
    return worst
