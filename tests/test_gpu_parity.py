"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact: graph build, message-passing forward z, message-passing backward dx (index_add_
order).  Everything with a reduction over nodes or a GEMM: max-norm relative 1e-5 vs the
fp32 CPU oracle, with an fp64 oracle tie-break (tests/helpers.py).
"""
import copy

import numpy as np
import pytest
import torch

from raincast_gnn import options

from helpers import (assert_close_tiebreak, check_training_step, knn_batch_graph, random_graph,
                     rel_err, special_graphs)
from oracle import gine_cpu as O
from raincast_gnn import GINEConv, _lib, functional as Fn
from raincast_gnn.graph import GineGraph
from raincast_gnn.models import GNN, ResGnn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def _mp_params(D, seed=0, eps=0.1):
    g = torch.Generator().manual_seed(seed)
    lw = torch.randn(D, 1, generator=g) * 0.5
    lb = torch.randn(D, generator=g) * 0.5
    return lw, lb, torch.tensor([eps])


# ---------------------------------------------------------------------------------------
# graph build
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", special_graphs(), ids=lambda c: c[0])
def test_graph_build_matches_stable_sort(case):
    _, ei, ea, n = case
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    E = ei.size(1)
    for key, other, rowptr, nbr, attr in ((1, 0, g.in_rowptr, g.in_src, g.in_attr),
                                          (0, 1, g.out_rowptr, g.out_dst, g.out_attr)):
        perm = np.argsort(ei[key].numpy(), kind="stable")
        counts = np.bincount(ei[key].numpy(), minlength=n)
        exp_rowptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        assert np.array_equal(rowptr.cpu().numpy(), exp_rowptr)
        if E:
            assert np.array_equal(nbr.cpu().numpy()[:E], ei[other].numpy()[perm].astype(np.int32))
            assert np.array_equal(attr.cpu().numpy()[:E], ea.reshape(-1).numpy()[perm])


def test_graph_build_rejects_out_of_range():
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]], device=DEV)
    with pytest.raises(IndexError):
        GineGraph(ei, torch.ones(3, 1, device=DEV), 3)
    ei = torch.tensor([[0, -1], [1, 0]], device=DEV)
    with pytest.raises(IndexError):
        GineGraph(ei, torch.ones(2, 1, device=DEV), 3)


# ---------------------------------------------------------------------------------------
# message passing: bit-exact
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", special_graphs(), ids=lambda c: c[0])
@pytest.mark.parametrize("D", [4, 64, 128, 96, 260])
def test_mp_forward_bit_exact(case, D):
    _, ei, ea, n = case
    torch.manual_seed(D)
    x = torch.randn(n, D)
    lw, lb, eps = _mp_params(D, seed=D)
    z_ref = O.gine_aggregate(x, ei, ea, lw, lb, eps)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    z = Fn.mp_forward(x.to(DEV), g, lw.reshape(-1).to(DEV), lb.to(DEV), eps.to(DEV))
    assert torch.equal(z.cpu(), z_ref), f"max diff {(z.cpu() - z_ref).abs().max().item()}"


@pytest.mark.parametrize("rounding,flag", [("fma", 0), ("muladd", _lib.GINE_MP_LIN_MULADD)])
def test_mp_forward_matches_loop_restatement(rounding, flag):
    """Both edge-Linear rounding modes against the independent per-edge restatement."""
    ei, ea, n = random_graph(30, 200, seed=9)
    x = torch.randn(n, 8)
    lw, lb, eps = _mp_params(8, seed=2, eps=-0.3)
    z_loop = O.gine_aggregate_loops(x, ei, ea, lw, lb, eps, rounding)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    z = Fn.mp_forward(x.to(DEV), g, lw.reshape(-1).to(DEV), lb.to(DEV), eps.to(DEV),
                      lin_flag=flag)
    assert torch.equal(z.cpu(), z_loop)
    other = O.gine_aggregate_loops(x, ei, ea, lw, lb, eps,
                                   "muladd" if rounding == "fma" else "fma")
    assert not torch.equal(z_loop, other)  # the two modes really differ on this input


@pytest.mark.parametrize("case", special_graphs(), ids=lambda c: c[0])
@pytest.mark.parametrize("D", [64, 128, 36])
def test_mp_backward(case, D):
    _, ei, ea, n = case
    torch.manual_seed(100 + D)
    x = torch.randn(n, D, requires_grad=True)
    lw, lb, eps = _mp_params(D, seed=D + 1, eps=0.25)
    lw.requires_grad_(True)
    lb.requires_grad_(True)
    eps.requires_grad_(True)
    z = O.gine_aggregate(x, ei, ea, lw, lb, eps)
    dz = torch.randn_like(z)
    z.backward(dz)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    xd = x.detach().to(DEV)
    dx, dlw, dlb, deps = Fn.mp_backward(dz.to(DEV), xd, g, lw.detach().reshape(-1).to(DEV),
                                        lb.detach().to(DEV), eps.detach().to(DEV))
    # index_add_ order + two-term sum with (1+eps)*dz: bit-identical to CPU autograd
    assert torch.equal(dx.cpu(), x.grad), f"max diff {(dx.cpu() - x.grad).abs().max().item()}"
    # fp64 reference for the parameter reductions
    x64 = x.detach().double().requires_grad_(False)
    lw64, lb64, e64 = (t.detach().double().requires_grad_(True) for t in (lw, lb, eps))
    O.gine_aggregate(x64, ei, ea.double(), lw64, lb64, e64).backward(dz.double())
    for name, got, ref32, ref64 in (("dlin_w", dlw, lw.grad.reshape(-1), lw64.grad.reshape(-1)),
                                    ("dlin_b", dlb, lb.grad, lb64.grad),
                                    ("deps", deps, eps.grad, e64.grad)):
        if ref32.abs().max() == 0:
            assert got.abs().max().item() == 0
            continue
        assert_close_tiebreak(got.cpu(), ref32, ref64, TOL, name)


@pytest.mark.parametrize("case", special_graphs(), ids=lambda c: c[0])
@pytest.mark.parametrize("D,tile_nodes", [(128, 128), (64, 8), (32, 1), (16, 128), (256, 64),
                                          (96, 128)])
def test_mp_window_path_matches_gather_and_oracle(case, D, tile_nodes, monkeypatch):
    """LDS-staged window kernels (gine_mp_*_win) vs the gather kernels and the oracle:
    z and dx bit-identical, the parameter reductions at fp32 tolerance."""
    _, ei, ea, n = case
    monkeypatch.setattr(options, "WINDOW_NODES", str(tile_nodes))
    monkeypatch.setattr(options, "MP_WINDOW", "all")
    gw = GineGraph(ei.to(DEV), ea.to(DEV), n)
    monkeypatch.setattr(options, "MP_WINDOW", "0")
    gg = GineGraph(ei.to(DEV), ea.to(DEV), n)
    assert gg.window_plan("in", D) is None and gg.window_plan("out", D) is None
    plan_in, plan_out = gw.window_plan("in", D), gw.window_plan("out", D)
    assert plan_in is not None and plan_out is not None
    assert plan_in.max_nodes <= tile_nodes
    torch.manual_seed(7 + D)
    x = torch.randn(n, D, requires_grad=True)
    dz, dres = torch.randn(n, D), torch.randn(n, D)
    lw, lb, eps = _mp_params(D, seed=D + 3, eps=0.3)
    lw.requires_grad_(True)
    lb.requires_grad_(True)
    eps.requires_grad_(True)
    z_ref = O.gine_aggregate(x, ei, ea, lw, lb, eps)
    (z_ref * dz).sum().backward()
    dev_args = [t.detach().to(DEV) for t in (lw.reshape(-1), lb, eps)]
    xd = x.detach().to(DEV)
    z_w = Fn.mp_forward(xd, gw, *dev_args)
    z_g = Fn.mp_forward(xd, gg, *dev_args)
    assert torch.equal(z_w.cpu(), z_ref.detach())
    assert torch.equal(z_w, z_g)
    rw = Fn.mp_backward(dz.to(DEV), xd, gw, *dev_args, dres=dres.to(DEV))
    rg = Fn.mp_backward(dz.to(DEV), xd, gg, *dev_args, dres=dres.to(DEV))
    assert torch.equal(rw[0].cpu(), x.grad + dres)
    assert torch.equal(rw[0], rg[0])
    x64 = x.detach().double()
    lw64, lb64, e64 = (t.detach().double().requires_grad_(True) for t in (lw, lb, eps))
    O.gine_aggregate(x64, ei, ea.double(), lw64, lb64, e64).backward(dz.double())
    for name, got, ref32, ref64 in (("dlin_w", rw[1], lw.grad.reshape(-1), lw64.grad.reshape(-1)),
                                    ("dlin_b", rw[2], lb.grad, lb64.grad),
                                    ("deps", rw[3], eps.grad, e64.grad)):
        if ref32.abs().max() == 0:
            assert got.abs().max().item() == 0
            continue
        assert_close_tiebreak(got.cpu(), ref32, ref64, TOL, name)
    # deterministic: a second run is bit-identical
    rw2 = Fn.mp_backward(dz.to(DEV), xd, gw, *dev_args, dres=dres.to(DEV))
    for a, b in zip(rw, rw2):
        assert torch.equal(a, b)


def test_mp_window_auto_policy(monkeypatch):
    """Default mode: the backward is staged when the launch has >= 256 workgroups, the
    forward keeps the gather kernel; options.MP_WINDOW "0" disables staging."""
    ei, ea, n = knn_batch_graph(500, 10, 32, seed=0)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    assert g.window_plan("in", 128) is None
    plan = g.window_plan("out", 128)
    assert plan is not None and plan.num_tiles == 128 and plan.slice_channels == 32
    ei1, ea1, n1 = knn_batch_graph(500, 10, 1, seed=0)
    g1 = GineGraph(ei1.to(DEV), ea1.to(DEV), n1)
    assert g1.window_plan("out", 128) is None      # 4 tiles x 4 slices: too few
    monkeypatch.setattr(options, "MP_WINDOW", "0")
    g0 = GineGraph(ei.to(DEV), ea.to(DEV), n)
    assert g0.window_plan("out", 128) is None
    monkeypatch.setattr(options, "MP_WINDOW", "bogus")
    with pytest.raises(ValueError):
        GineGraph(ei.to(DEV), ea.to(DEV), n)


def test_mp_nonfinite_inputs_follow_cpu():
    """NaN / inf node features: relu keeps NaN (clamp_min), its backward passes the
    gradient where relu(pre) is NaN (threshold_backward tests `result <= 0`)."""
    ei, ea, n = knn_batch_graph(64, 4, 1, seed=3)
    D = 64
    torch.manual_seed(5)
    x = torch.randn(n, D)
    x[3, 5] = float("nan")
    x[10, :7] = float("inf")
    x[20, 40:] = float("-inf")
    x[33, 1] = float("nan")
    lw, lb, eps = _mp_params(D, seed=6, eps=0.2)
    z_ref = O.gine_aggregate(x, ei, ea, lw, lb, eps)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    z = Fn.mp_forward(x.to(DEV), g, lw.reshape(-1).to(DEV), lb.to(DEV), eps.to(DEV)).cpu()
    assert torch.equal(z.isnan(), z_ref.isnan())
    fin = ~z_ref.isnan()
    assert torch.equal(z[fin], z_ref[fin])
    xr = x.clone().requires_grad_(True)
    dz = torch.randn(n, D)
    O.gine_aggregate(xr, ei, ea, lw, lb, eps).backward(dz)
    dx = Fn.mp_backward(dz.to(DEV), x.to(DEV), g, lw.reshape(-1).to(DEV), lb.to(DEV),
                        eps.to(DEV))[0].cpu()
    assert torch.equal(dx.isnan(), xr.grad.isnan())
    fin = ~xr.grad.isnan()
    assert torch.equal(dx[fin], xr.grad[fin])


def test_mp_deterministic():
    ei, ea, n = random_graph(3000, 60000, seed=11)
    x = torch.randn(n, 128, device=DEV)
    lw, lb, eps = (t.to(DEV) for t in _mp_params(128))
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    dz = torch.randn(n, 128, device=DEV)
    r1 = Fn.mp_backward(dz, x, g, lw.reshape(-1), lb, eps)
    r2 = Fn.mp_backward(dz, x, g, lw.reshape(-1), lb, eps)
    z1 = Fn.mp_forward(x, g, lw.reshape(-1), lb, eps)
    z2 = Fn.mp_forward(x, g, lw.reshape(-1), lb, eps)
    assert torch.equal(z1, z2)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


# ---------------------------------------------------------------------------------------
# GINE layer with the fused node MLP
# ---------------------------------------------------------------------------------------
def _make_pair(D, seed):
    torch.manual_seed(seed)
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    with torch.no_grad():
        conv.eps.fill_(0.125)
        mlp[1].weight.uniform_(0.5, 1.5)
        mlp[1].bias.uniform_(-0.2, 0.2)
        mlp[1].running_mean.uniform_(-0.1, 0.1)
        mlp[1].running_var.uniform_(0.5, 2.0)
    ref = O.OracleGINEConv(copy.deepcopy(mlp), train_eps=True, edge_dim=1)
    ref.load_state_dict(conv.state_dict())
    return conv.to(DEV), ref


def _oracle_layer(ref, x, ei, ea, epilogue, dtype):
    r = copy.deepcopy(ref).to(dtype)
    xx = x.detach().to(dtype).requires_grad_(True)
    o = r(xx, ei, ea.to(dtype))
    if epilogue == "relu":
        o = torch.relu(o)
    elif epilogue == "residual":
        o = xx + torch.relu(o)
    return r, xx, o


@pytest.mark.parametrize("D", [128, 64, 32, 256])
@pytest.mark.parametrize("epilogue", ["none", "relu", "residual"])
@pytest.mark.parametrize("training", [True, False])
def test_gine_layer_fused(D, epilogue, training):
    ei, ea, n = knn_batch_graph(300, 8, 2, seed=D)
    conv, ref = _make_pair(D, seed=D + len(epilogue))
    conv.train(training)
    ref.train(training)
    x = torch.randn(n, D)
    dy = torch.randn(n, D)
    outs = {}
    for dtype in (torch.float32, torch.float64):
        r, xx, o = _oracle_layer(ref, x, ei, ea, epilogue, dtype)
        o.backward(dy.to(dtype))
        outs[dtype] = (r, xx, o)
    xd = x.to(DEV).requires_grad_(True)
    eid, ead = ei.to(DEV), ea.to(DEV)
    fn = {"none": conv.forward, "relu": conv.forward_relu,
          "residual": conv.forward_residual_relu}[epilogue]
    y = fn(xd, eid, ead)
    y.backward(dy.to(DEV))
    r32, x32, o32 = outs[torch.float32]
    r64, x64, o64 = outs[torch.float64]
    assert_close_tiebreak(y.detach().cpu(), o32.detach(), o64.detach(), TOL, "y")
    assert_close_tiebreak(xd.grad.cpu(), x32.grad, x64.grad, TOL, "dx")
    p_gpu = dict(conv.named_parameters())
    p32, p64 = dict(r32.named_parameters()), dict(r64.named_parameters())
    for name in p32:
        assert_close_tiebreak(p_gpu[name].grad.cpu(), p32[name].grad, p64[name].grad, TOL, name)
    bn_gpu, bn32 = conv.nn[1], r32.nn[1]
    for buf in ("running_mean", "running_var"):
        assert rel_err(getattr(bn_gpu, buf).cpu(), getattr(bn32, buf)) <= TOL, buf
    assert int(bn_gpu.num_batches_tracked) == int(bn32.num_batches_tracked)


def test_generic_nn_path():
    """An nn the fused path does not cover (D=48, GELU): HIP message passing + torch nn."""
    D = 48
    ei, ea, n = knn_batch_graph(100, 6, 1, seed=5)
    torch.manual_seed(0)
    mlp = torch.nn.Sequential(torch.nn.Linear(D, 24), torch.nn.GELU(), torch.nn.Linear(24, 16))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    ref = O.OracleGINEConv(copy.deepcopy(mlp), train_eps=True, edge_dim=1)
    ref.load_state_dict(conv.state_dict())
    conv = conv.to(DEV)
    x = torch.randn(n, D)
    xd = x.to(DEV).requires_grad_(True)
    out = conv(xd, ei.to(DEV), ea.to(DEV))
    xr = x.clone().requires_grad_(True)
    outr = ref(xr, ei, ea)
    assert rel_err(out.cpu(), outr) <= TOL
    g = torch.randn_like(outr)
    out.backward(g.to(DEV))
    outr.backward(g)
    assert rel_err(xd.grad.cpu(), xr.grad) <= TOL


def test_layer_deterministic_and_errors():
    conv, _ = _make_pair(128, seed=1)
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=1)
    x = torch.randn(n, 128, device=DEV, requires_grad=True)
    eid, ead = ei.to(DEV), ea.to(DEV)
    conv.eval()  # no running-stat drift between the two runs
    res = []
    for _ in range(2):
        x.grad = None
        conv.zero_grad()
        y = conv.forward_residual_relu(x, eid, ead)
        y.square().sum().backward()
        res.append([y.detach().clone(), x.grad.clone()] +
                   [p.grad.clone() for p in conv.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)
    with pytest.raises(_lib.GineError):
        conv(x.detach().cpu(), ei, ea)
    conv.train()
    with pytest.raises(ValueError):
        conv(x[:1].detach(), torch.zeros(2, 0, dtype=torch.long, device=DEV),
             torch.zeros(0, 1, device=DEV))


# ---------------------------------------------------------------------------------------
# full models
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("experiment", ["24h_mixed", "72h_mixed_u", "120h_normal_mixed",
                                        "24h_normal"])
def test_training_step_matches_oracle(experiment):
    """Full train-step gradients (DeepSet + 4 GINE layers + head + loss) vs the oracle
    (tests/helpers.py: check_training_step; the benchmark shapes are in
    tests/test_gpu_configs.py)."""
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.params import EXPERIMENTS
    worst = check_training_step(dict(EXPERIMENTS[experiment]),
                                synthetic_batch(500, 2, k=10, seed=7), DEV, TOL)
    print(f"{experiment}: worst grad rel err vs fp32 oracle {worst:.2e}")


def test_resgnn_stack_matches_oracle():
    ei, ea, n = knn_batch_graph(500, 10, 3, seed=2)
    torch.manual_seed(3)
    net = ResGnn(128, 128, 4, 128)
    ref = O.OracleResGnn(128, 128, 4, 128)
    ref.load_state_dict(net.state_dict())
    net = net.to(DEV)
    x = torch.randn(n, 128)
    y = net(x.to(DEV), ei.to(DEV), ea.to(DEV))
    yr = ref(x, ei, ea)
    ref64 = copy.deepcopy(ref).double()
    y64 = ref64(x.double(), ei, ea.double())
    assert_close_tiebreak(y.detach().cpu(), yr.detach(), y64.detach(), TOL, "resgnn")


def test_graph_capture_replay_matches_eager():
    """Whole training step (fwd + loss + bwd + AdamW) captured in one HIP graph: replays
    follow the same trajectory as eager steps from the same initial state."""
    from raincast_gnn.data import synthetic_batch
    torch.manual_seed(0)
    base = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(500, 4, k=10, seed=1).to(DEV)

    def make():
        m = copy.deepcopy(base).to(DEV)
        return m, torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True)

    def step(m, opt):
        opt.zero_grad(set_to_none=False)
        loss = m.loss_fn.crps(m(batch), batch.y)
        loss.backward()
        opt.step()
        return loss

    m_e, o_e = make()
    eager = [step(m_e, o_e).item() for _ in range(5)]

    m_g, o_g = make()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        warm = [step(m_g, o_g).item() for _ in range(2)]
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_loss = step(m_g, o_g)
    replayed = []
    for _ in range(3):
        g.replay()
        replayed.append(static_loss.item())
    got = warm + replayed
    for a, b in zip(got, eager):
        assert abs(a - b) <= 1e-6 * abs(b), (got, eager)


def test_eval_mode_prediction_and_ensemble_match_oracle(tmp_path):
    """eval.py's path: after training steps (non-trivial BatchNorm running statistics) the
    eval-mode forward under no_grad matches the oracle's eval forward, and the
    checkpoint-ensemble average matches averaging the oracle's predictions."""
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.evaluate import ensemble_crps, predict_ensemble
    from raincast_gnn.optim import FlatAdamW
    torch.manual_seed(5)
    batches = [synthetic_batch(300, 2, k=8, seed=s) for s in (11, 12)]
    states = []
    for seed in (1, 2):
        torch.manual_seed(seed)
        model = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5).to(DEV)
        opt = FlatAdamW(model.parameters(), lr=1e-3)
        model.train()
        for b in batches:
            opt.zero_grad()
            bb = b.to(DEV)
            model.loss_fn.crps(model(bb), bb.y).backward()
            opt.step()
        path = str(tmp_path / f"ck{seed}.pth")
        torch.save(model.state_dict(), path)
        states.append(path)

    def make():
        return GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)

    preds = predict_ensemble(make, states, batches, DEV)
    refs = []
    for path in states:
        ref = O.OracleGNN(35, 128, 4, "MixedLoss", "False", 1.71, 0.5)
        ref.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        ref.eval()
        with torch.no_grad():
            refs.append(torch.cat([ref(b) for b in batches], 0))
    ref_mean = torch.stack(refs, 0).mean(0)
    assert preds.shape == ref_mean.shape
    assert rel_err(preds, ref_mean) <= 1e-5, rel_err(preds, ref_mean)
    y = torch.cat([b.y for b in batches])
    c = ensemble_crps(make(), preds, y)
    c_ref = ensemble_crps(make(), ref_mean, y)
    assert abs(c.item() - c_ref.item()) <= 1e-5 * abs(c_ref.item())


# ---------------------------------------------------------------------------------------
# fused message passing + first Linear (gine_mp_fwd_mlp1)
# ---------------------------------------------------------------------------------------
def _fused_cases():
    out = [c for c in special_graphs()]
    ei, ea, n = knn_batch_graph(500, 10, 32, seed=5)        # cfg2: ~2 tiles per workgroup
    out.append(("knn500_k10_b32", ei, ea, n))
    ei, ea, n = knn_batch_graph(2000, 16, 16, seed=6)       # 1000 tiles: 4 per workgroup
    out.append(("knn2000_k16_b16", ei, ea, n))
    ei, ea, n = knn_batch_graph(37, 31, 3, seed=7)          # in-degree 32: the limit
    out.append(("knn37_k31_b3", ei, ea, n))
    return out


@pytest.mark.parametrize("case", _fused_cases(), ids=lambda c: c[0])
@pytest.mark.parametrize("rounding", [0, _lib.GINE_MP_LIN_MULADD], ids=["fma", "muladd"])
def test_mp_fwd_mlp1_fused_matches_unfused(case, rounding, monkeypatch):
    """One-launch gather + Linear1 + BN partials == gine_mp_fwd then gine_mlp_fwd1, bit for
    bit (z, a1 and every partial row); above the degree limit it refuses."""
    monkeypatch.setattr(options, "MP_FUSED", "all")
    _, ei, ea, n = case
    D = 128
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    torch.manual_seed(n)
    x = torch.randn(n, D, device=DEV)
    lw, lb, eps = (t.to(DEV) for t in _mp_params(D, seed=n, eps=0.25))
    lw = lw.reshape(-1).contiguous()
    w1 = (torch.randn(D, D) / 11).to(DEV)
    b1 = torch.randn(D).to(DEV)
    P = Fn._count("gine_mlp_num_partials", n, D)
    z1, a1f = torch.full_like(x, 7.0), torch.full_like(x, 7.0)
    part1 = torch.full((P, 2, D), 7.0, dtype=torch.float64, device=DEV)
    args = (Fn.ptr(x), Fn.ptr(g.in_rowptr), Fn.ptr(g.in_src), Fn.ptr(g.in_attr), Fn.ptr(lw),
            Fn.ptr(lb), Fn.ptr(eps), Fn.ptr(w1), Fn.ptr(b1), Fn.ptr(z1), Fn.ptr(a1f),
            Fn.ptr(part1), n, D)
    stream = _lib.stream_handle(DEV)
    if g.max_in_degree > _lib.MP_FUSED_MAX_DEGREE:
        with pytest.raises(_lib.GineError):
            _lib.call("gine_mp_fwd_mlp1", *args, g.max_in_degree, rounding, stream)
        assert not Fn.fused_forward_ok(g, n, D)
        return
    assert Fn.fused_forward_ok(g, n, D)
    _lib.call("gine_mp_fwd_mlp1", *args, g.max_in_degree, rounding, stream)
    z0 = Fn.mp_forward(x, g, lw, lb, eps, lin_flag=rounding)
    a10 = torch.empty_like(x)
    part0 = torch.empty(P, 2, D, dtype=torch.float64, device=DEV)
    _lib.call("gine_mlp_fwd1", Fn.ptr(z0), Fn.ptr(w1), Fn.ptr(b1), Fn.ptr(a10), Fn.ptr(part0),
              n, D, stream)
    torch.cuda.synchronize()
    assert torch.equal(z1, z0)
    assert torch.equal(a1f, a10)
    assert torch.equal(part1, part0)


def test_mp_fwd_mlp1_rejects_bad_arguments():
    ei, ea, n = knn_batch_graph(64, 4, 1, seed=3)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    D = 128
    x = torch.randn(n, D, device=DEV)
    t = torch.zeros(D, device=DEV)
    P = Fn._count("gine_mlp_num_partials", n, D)
    part = torch.zeros(P, 2, D, dtype=torch.float64, device=DEV)
    base = [Fn.ptr(x), Fn.ptr(g.in_rowptr), Fn.ptr(g.in_src), Fn.ptr(g.in_attr), Fn.ptr(t),
            Fn.ptr(t), Fn.ptr(t), Fn.ptr(x), Fn.ptr(t), Fn.ptr(x), Fn.ptr(x), Fn.ptr(part)]
    s = _lib.stream_handle(DEV)
    for bad in ([*base, n, 64, 5, 0, s], [*base, n, D, 33, 0, s], [*base, n, D, 5, 8, s],
                [*base[:3], None, *base[4:], n, D, 5, 0, s], [*base, 0, D, 5, 0, s]):
        with pytest.raises(_lib.GineError):
            _lib.call("gine_mp_fwd_mlp1", *bad)


def test_layer_fused_forward_equals_unfused(monkeypatch):
    """A training GINE layer (forward + backward) gives identical bits with the fused
    forward on and off."""
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=9)
    assert n <= Fn.FUSED_MAX_NODES
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setattr(options, "MP_FUSED", flag)
        torch.manual_seed(0)
        net = ResGnn(128, 128, 2, 128).to(DEV).train()
        x = torch.randn(n, 128, device=DEV, requires_grad=True)
        y = net(x, ei.to(DEV), ea.to(DEV))
        y.backward(torch.ones_like(y))
        outs.append([y.detach(), x.grad] + [p.grad for p in net.parameters()]
                    + [b for b in net.buffers()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
