"""GPU: the training-step pieces around the GINE stack (flat AdamW, DeepSet restructure,
captured step) against their reference formulations."""
import copy

import pytest
import torch

from raincast_gnn import options

from helpers import rel_err
from oracle import gine_cpu as O
from raincast_gnn.models import DeepSetEncoder
from raincast_gnn.optim import FlatAdamW

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_flat_adamw_matches_torch_adamw():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(35, 64), torch.nn.ReLU(),
                              torch.nn.Linear(64, 5)).to(DEV)
    ref = copy.deepcopy(net)
    opt = FlatAdamW(net.parameters(), lr=3e-3, weight_decay=0.01)
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=3e-3, weight_decay=0.01, foreach=False)
    x = torch.randn(256, 35, device=DEV)
    for _ in range(6):
        # identical gradients on both sides: only the optimizer arithmetic is compared
        opt_ref.zero_grad()
        ref(x).square().mean().backward()
        opt.zero_grad(set_to_none=False)
        for p, q in zip(net.parameters(), ref.parameters()):
            p.grad.copy_(q.grad)
        opt.step()
        opt_ref.step()
    assert opt.views_intact()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert rel_err(p.detach(), q.detach()) <= 2e-6
    st = opt_ref.state[next(ref.parameters())]
    assert opt.step_count.item() == st["step"].item() == 6


@pytest.mark.parametrize("numel", [64, 3 * 1024, 8 * 1024, 13 * 1024 - 40, 900_000])
def test_flat_adamw_step_count_across_grid_sizes(numel):
    """The step counter sits behind a two-level ticket (gine_adamw_step: 8 sub-tickets, then
    the top word): grids of 1, 3, 8, 13 and the capped 512 workgroups (ragged groups) bump it
    exactly once per step and leave every ticket word at 0, and the update follows torch."""
    torch.manual_seed(1)
    p = torch.nn.Parameter(torch.randn(numel, device=DEV))
    q = torch.nn.Parameter(p.detach().clone())
    opt = FlatAdamW([p], lr=1e-3, weight_decay=0.01)
    opt_ref = torch.optim.AdamW([q], lr=1e-3, weight_decay=0.01, foreach=False)
    for _ in range(5):
        g = torch.randn(numel, device=DEV)
        opt.zero_grad(set_to_none=False)
        p.grad.copy_(g)
        q.grad = g.clone()
        opt.step()
        opt_ref.step()
    torch.cuda.synchronize()
    assert opt.step_count.item() == 5
    state = opt._step_state.view(torch.int32).cpu()
    assert int(state[1:].abs().sum()) == 0      # top and sub-tickets re-armed
    assert rel_err(p.detach(), q.detach()) <= 2e-6


def test_deepset_restructure_matches_reference_form():
    torch.manual_seed(1)
    enc = DeepSetEncoder(35, 128, 128)
    ref = O.OracleDeepSet(35, 128, 128)
    ref.load_state_dict(enc.state_dict())
    ens = torch.randn(3000, 11, 35)
    out = enc.to(DEV)(ens.to(DEV))
    exp = ref(ens)
    exp64 = copy.deepcopy(ref).double()(ens.double())
    assert rel_err(out.detach().cpu(), exp64) <= 2 * rel_err(exp.detach(), exp64) + 1e-6
    assert rel_err(out.detach().cpu(), exp.detach()) <= 1e-5


def test_bench_trainer_graph_step_runs():
    import bench
    from raincast_gnn.params import BENCH_CONFIGS
    tr = bench.Trainer(BENCH_CONFIGS[1], DEV, 0, 1, 2)
    losses = [tr.eager_step().item() for _ in range(3)]
    tr.capture()
    for _ in range(3):
        losses.append(tr.step().item())
    assert all(map(lambda v: v == v, losses))  # finite / not NaN
    assert losses[-1] < losses[0]              # training makes progress (lr 1e-4, 6 steps)


CASES = [("normal", "NormalCRPS", "False"), ("normal_mixed", "MixedNormalCRPS", "False"),
         ("mixed", "MixedLoss", "False"), ("mixed_u", "MixedLoss", "True")]


@pytest.mark.parametrize("name,loss,grad_u", CASES)
def test_fused_crps_matches_reference_golden(name, loss, grad_u):
    """The fused HIP loss (value + gradient through PostProcess) vs outputs of the
    reference's own models/loss.py + models/model_utils.py (tests/golden/)."""
    import os

    import numpy as np

    from conftest import GOLDEN
    from raincast_gnn.models import make_loss
    from raincast_gnn.postprocess import PostProcess
    d = np.load(os.path.join(GOLDEN, "reference_heads.npz"))
    raw = torch.from_numpy(d[f"{name}_raw"]).to(DEV).requires_grad_(True)
    y = torch.from_numpy(d[f"{name}_y"]).to(DEV)
    fn, _ = make_loss(loss, grad_u, 1.71, 0.5)
    val = fn.crps(PostProcess(loss, grad_u)(raw), y)
    assert str(val.dtype) == str(d[f"{name}_loss_dtype"][0])
    ref = d[f"{name}_loss"][0]
    assert abs(val.item() - ref) <= 1e-6 * abs(ref), (val.item(), ref)
    val.backward()
    g, gr = raw.grad.cpu().numpy(), d[f"{name}_grad"]
    assert np.abs(g - gr).max() <= 1e-5 * np.abs(gr).max()


@pytest.mark.parametrize("name,loss,grad_u", CASES)
def test_fused_crps_matches_torch_formulation(name, loss, grad_u):
    from raincast_gnn.models import make_loss
    from raincast_gnn.postprocess import PostProcess
    from raincast_gnn.data import synthetic_targets
    import numpy as np
    torch.manual_seed(3)
    K = {"NormalCRPS": 2, "MixedNormalCRPS": 3, "MixedLoss": 4 + (grad_u == "True")}[loss]
    raw = torch.randn(20000, K)
    y = torch.from_numpy(synthetic_targets(np.random.default_rng(1), 20000, nan_frac=0.05))
    fn, _ = make_loss(loss, grad_u, 1.71, 0.5)
    pp = PostProcess(loss, grad_u)
    xg = raw.to(DEV).requires_grad_(True)
    v = fn.crps(pp(xg), y.to(DEV))          # fused HIP path
    v.backward()
    xc = raw.clone().requires_grad_(True)
    vc = fn.crps(pp(xc), y)                  # torch formulation (CPU)
    vc.backward()
    assert v.dtype == vc.dtype
    assert abs(v.item() - vc.item()) <= 1e-6 * abs(vc.item())
    assert rel_err(xg.grad.cpu(), xc.grad) <= 1e-5


def test_fused_crps_nan_handling():
    from raincast_gnn.loss import MixedLoss
    fn = MixedLoss(grad_u=False, u=1.71, xi=0.5)
    pred = torch.rand(50, 4, device=DEV) + 0.1
    y = torch.full((50,), float("nan"), device=DEV)
    y[7] = 0.3
    pred.requires_grad_(True)
    v = fn.crps(pred, y)
    v.backward()
    assert torch.isfinite(v)
    assert torch.count_nonzero(pred.grad.abs().sum(1)) == 1  # only row 7 has a gradient
    assert torch.isnan(fn.crps(pred.detach(), torch.full((50,), float("nan"), device=DEV)))


@pytest.mark.parametrize("rows,O,I", [(176000, 128, 35), (16000, 128, 163), (16000, 4, 128),
                                      (1000, 128, 128), (37, 5, 3), (0, 8, 8)])
def test_linear_wgrad_kernel(rows, O, I):
    from raincast_gnn.linear import Linear
    torch.manual_seed(rows + O)
    lin = Linear(I, O).to(DEV)
    x = torch.randn(rows, I, device=DEV)
    dy = torch.randn(rows, O, device=DEV)
    lin(x).backward(dy)
    dw64 = dy.double().T @ x.double()
    db64 = dy.double().sum(0)
    scale_w = (dy.double().abs().T @ x.double().abs()).max().item() or 1.0
    assert (lin.weight.grad.double() - dw64).abs().max().item() <= 1e-6 * scale_w
    if rows:
        assert (lin.bias.grad.double() - db64).abs().max().item() <= 1e-6 * dy.abs().sum(0).max().item()
    else:
        assert torch.count_nonzero(lin.weight.grad) == 0


def test_linear_wgrad_nonfinite_operands():
    """The weight-gradient engine's split-bf16 chain turns an inf operand into NaN planes;
    such a tile is redone on the fp32 chain, so inf / NaN land where fp32 puts them (torch's
    dy^T x): +-inf columns for an inf in x, NaN columns for a NaN, the rest unchanged."""
    from raincast_gnn.linear import Linear
    torch.manual_seed(5)
    rows, O, I = 5000, 64, 200
    lin = Linear(I, O).to(DEV)
    x = torch.randn(rows, I, device=DEV)
    x[17, 3] = float("inf")
    x[4000, 150] = float("nan")
    dy = torch.randn(rows, O, device=DEV)
    lin(x).backward(dy)
    got, ref = lin.weight.grad.cpu(), (dy.T @ x).cpu()
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(torch.isinf(got), torch.isinf(ref))
    assert torch.equal(got[torch.isinf(ref)], ref[torch.isinf(ref)])
    fin = torch.isfinite(ref)
    assert int(fin.sum()) == O * (I - 2)
    ref64 = (dy.double().T @ torch.nan_to_num(x.double(), nan=0.0, posinf=0.0)).cpu()
    scale = (dy.double().abs().T @ torch.nan_to_num(x.double(), nan=0.0, posinf=0.0).abs())
    assert ((got.double() - ref64).abs()[fin] <= 1e-6 * scale.cpu().max()).all()


def test_grads_land_in_flat_buffer_without_copies():
    """Backward kernels write every parameter gradient straight into its FlatAdamW slice,
    and the resulting training trajectory equals torch.optim.AdamW's on ordinary grads."""
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    torch.manual_seed(5)
    base = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(300, 2, k=8, seed=2).to(DEV)
    m1, m2 = copy.deepcopy(base).to(DEV), copy.deepcopy(base).to(DEV)
    opt1 = FlatAdamW(m1.parameters(), lr=1e-3)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-3, foreach=False)
    for step in range(3):
        opt1.zero_grad()
        m1.loss_fn.crps(m1(batch), batch.y).backward()
        base_ptr = opt1.flat_grad.data_ptr()
        for p, off in zip(opt1.params, opt1._offsets):
            assert p.grad.data_ptr() == base_ptr + 4 * off   # adopted, not copied
        opt1.step()
        if step == 0:
            # one step from identical weights: same gradients, same AdamW arithmetic.  (Later
            # steps are not comparable elementwise: Adam turns ulp-level gradient differences
            # on near-zero components into +-lr steps.)
            opt2.zero_grad()
            m2.loss_fn.crps(m2(batch), batch.y).backward()
            opt2.step()
            for (n, p), q in zip(m1.named_parameters(), m2.parameters()):
                assert rel_err(p.detach(), q.detach()) <= 1e-6, n


def test_device_loader_training_builds_graph_once():
    """With the device-resident batcher every batch of one size shares one edge list, so
    the engine's CSR build runs once for the whole epoch."""
    from raincast_gnn.batching import DeviceDataset, DeviceLoader
    from raincast_gnn.data import synthetic_samples
    from raincast_gnn.graph import graph_cache
    from raincast_gnn.models import GNN
    from raincast_gnn.optim import FlatAdamW
    graph_cache.clear()
    ds = DeviceDataset(synthetic_samples(80, 12, k=6, seed=2), DEV)
    torch.manual_seed(0)
    model = GNN(35, 128, 128, 2, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5).to(DEV)
    opt = FlatAdamW(model.parameters(), lr=1e-3)
    losses = []
    for batch in DeviceLoader(ds, batch_size=4, shuffle=True, seed=1):
        opt.zero_grad()
        loss = model.loss_fn.crps(model(batch), batch.y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert len(losses) == 3 and all(l == l for l in losses)
    assert len(graph_cache._entries) == 1


def test_batched_grad_finish_matches_per_kernel_reductions(monkeypatch):
    """The end-of-backward batch (gine_grad_finalize_batch: dW_e/db_e/eps of every layer, the
    head / chain / DeepSet slabs) gives the gradients of the per-kernel reductions, complete
    when backward() returns, in fewer launches."""
    from raincast_gnn import gradbuf
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    torch.manual_seed(9)
    base = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(500, 32, k=10, seed=4).to(DEV)   # window backward active
    grads = {}
    for on in (False, True):
        monkeypatch.setattr(gradbuf, "BATCH_ENABLED", on)
        m = copy.deepcopy(base).to(DEV)
        opt = FlatAdamW(m.parameters(), lr=1e-3)
        opt.zero_grad()
        m.loss_fn.crps(m(batch), batch.y).backward()
        assert not gradbuf._pending
        grads[on] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for n, g in grads[False].items():
        assert rel_err(grads[True][n], g) <= 1e-6, n
    # a second backward accumulates onto complete gradients (nothing deferred then)
    monkeypatch.setattr(gradbuf, "BATCH_ENABLED", True)
    m = copy.deepcopy(base).to(DEV)
    opt = FlatAdamW(m.parameters(), lr=1e-3)
    opt.zero_grad()
    for _ in range(2):
        m.loss_fn.crps(m(batch), batch.y).backward()
    for n, p in m.named_parameters():
        assert rel_err(p.grad, 2 * grads[True][n]) <= 1e-6, n


def test_mlp_weight_grads_in_message_passing_launch(monkeypatch):
    """The node-MLP weight-gradient engine run by extra workgroups of the window
    message-passing backward (gine_mp_bwd_win_mlp_wgrad) gives the gradients of the engine
    run beside the dz GEMM (gine_mlp_bwd1_wgrad): dW bit for bit (same MFMA order), the
    bias sums to fp32 rounding."""
    from raincast_gnn import functional as Fn
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    torch.manual_seed(11)
    base = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(500, 32, k=10, seed=5).to(DEV)   # window backward active
    grads = {}
    for flag in ("0", "1"):
        monkeypatch.setattr(options, "ENGINE_IN_MP", flag == "1")
        m = copy.deepcopy(base).to(DEV)
        opt = FlatAdamW(m.parameters(), lr=1e-3)
        opt.zero_grad()
        m.loss_fn.crps(m(batch), batch.y).backward()
        grads[flag] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for n, gref in grads["0"].items():
        got = grads["1"][n]
        if n.endswith("nn.0.weight") or n.endswith("nn.3.weight"):
            assert torch.equal(got, gref), n
        assert rel_err(got, gref) <= 1e-6, n


@pytest.mark.parametrize("graphs,stations,k", [(1, 64, 4), (3, 500, 10), (2, 37, 36)])
def test_mlp_weight_grads_in_mp_launch_small_graphs(graphs, stations, k, monkeypatch):
    """The combined launch at sizes where the engine has few row chunks and the window plan
    is forced (options.MP_WINDOW "all"): same gradients as the engine beside the dz GEMM."""
    from raincast_gnn import functional as Fn
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    monkeypatch.setattr(options, "MP_WINDOW", "all")
    torch.manual_seed(graphs + stations)
    base = GNN(35, 128, 128, 2, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(stations, graphs, k=k, seed=6).to(DEV)
    grads = {}
    for flag in ("0", "1"):
        monkeypatch.setattr(options, "ENGINE_IN_MP", flag == "1")
        m = copy.deepcopy(base).to(DEV)
        opt = FlatAdamW(m.parameters(), lr=1e-3)
        opt.zero_grad()
        m.loss_fn.crps(m(batch), batch.y).backward()
        grads[flag] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    from raincast_gnn.graph import get_graph
    g = get_graph(batch.edge_index, batch.edge_attr.float(), batch.num_nodes)
    assert Fn.engine_in_mp_ok(g, 128)   # the combined launch really ran
    for n, gref in grads["0"].items():
        got = grads["1"][n]
        if n.endswith("nn.0.weight") or n.endswith("nn.3.weight"):
            assert torch.equal(got, gref), n
        assert rel_err(got, gref) <= 1e-6, n


@pytest.mark.parametrize("name,loss,grad_u", CASES)
def test_head_backward_in_crps_pass_matches_separate_launch(name, loss, grad_u):
    """gine_crps_head_fwd_grad: for a unit-seeded backward (gradbuf.loss_backward) the CRPS
    pass also runs the head's backward.  dh and so every gradient below the head are
    bit-identical to the separate gine_head_bwd launch (plain backward(), whose seed is not
    the cached unit, so the head falls back to it); the head's own
    dW / db differ only in the grouping of their fixed-order partial sums."""
    from raincast_gnn import gradbuf, head
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    torch.manual_seed(3)
    base = GNN(35, 128, 128, 2, loss=loss, grad_u=grad_u, u=1.71, xi=0.5)
    batch = synthetic_batch(700, 2, k=10, seed=4).to(DEV)
    batch.y[::7] = float("nan")  # masked targets: zero rows of d raw

    def grads(unit):
        m = copy.deepcopy(base).to(DEV)
        pred = m(batch)
        loss_v = m.loss_fn.crps(pred, batch.y)
        rec = head.record_of(pred)
        assert rec is not None and rec.pre is not None  # computed; used for the unit seed only
        if unit:
            gradbuf.loss_backward(loss_v)
        else:
            loss_v.backward()
        return loss_v.item(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}

    l_sep, g_sep = grads(False)
    l_fus, g_fus = grads(True)
    assert l_sep == l_fus
    for n, g in g_sep.items():
        if n.startswith("aggr."):
            assert rel_err(g_fus[n], g) <= 1e-6, n
        else:
            assert torch.equal(g_fus[n], g), n
