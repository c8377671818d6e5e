"""GPU: the one-launch layer forward (gine_mp_fwd_layer: fused gather + Linear1 + BatchNorm
sums, grid barrier, BatchNorm finish + Linear2 + ResGnn epilogue; csrc/gine_mpmlp.hip) against
the two-launch pair it replaces (gine_mp_fwd_mlp1_acc + gine_mlp_fwd2_bn).

Same tile -> workgroup map, integer BatchNorm totals and the row GEMM's MFMA chain and
epilogue: every output must be the same bits -- y, the ReLU mask, z, a1, bn_save, the
running statistics -- over several steps on one accumulator, with the two forms interleaved
(the pairing protocol of csrc/gine_bnacc.hpp must carry across them), and the backward that
follows must give the same gradients.
"""
import ctypes

import pytest
import torch

from raincast_gnn import GINEConv, _lib, functional as Fn, options

from helpers import knn_batch_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _python_binding(monkeypatch):
    """These tests read the Python autograd Function's saved tensors; the C++ binding (the
    drop-in default) issues the same launches (tests/test_gpu_dropin.py)."""
    from raincast_gnn import nn as rnn
    monkeypatch.setattr(rnn, "USE_TORCH_EXT", False)


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


def _saved(y):
    x, z, a1, ys, mask, bn_save = y.grad_fn.saved_tensors[:6]
    return [t.detach().clone() for t in (z, a1, bn_save) if t is not None] + (
        [mask.clone()] if mask is not None else [])


def _steps(conv, state, x, ei, ea, epilogue, forms, monkeypatch):
    conv.load_state_dict(state)
    fn = {"none": conv.forward, "relu": conv.forward_relu,
          "residual": conv.forward_residual_relu}[epilogue]
    outs = []
    for use_layer in forms:
        monkeypatch.setattr(options, "LAYER_FWD", use_layer)
        xi = x.clone().requires_grad_(True)
        y = fn(xi, ei, ea)
        sv = _saved(y)
        (y * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
        grads = [xi.grad.clone()] + [p.grad.clone() for p in conv.parameters()]
        conv.zero_grad(set_to_none=True)
        outs.append([y.detach().clone()] + sv + grads)
    torch.cuda.synchronize()
    bn = conv.nn[1]
    return outs, bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked)


@pytest.mark.parametrize("nodes,graphs,k", [(500, 32, 10), (120, 3, 6), (2000, 4, 16)],
                         ids=["cfg2", "small", "cfg3-b4"])
@pytest.mark.parametrize("epilogue", ["none", "relu", "residual"])
def test_layer_forward_equals_pair(nodes, graphs, k, epilogue, monkeypatch):
    ei, ea, n = knn_batch_graph(nodes, k, graphs, seed=nodes + k)
    ok = ctypes.c_int32(0)
    _lib.call("gine_mp_fwd_layer_ok", n, 128, k + 1, ctypes.byref(ok))
    assert ok.value == 1, "the layer form must apply at this size"
    conv = _conv(seed=k)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    x = torch.randn(n, 128, device=DEV) * 1.5 + 0.2
    eid, ead = ei.to(DEV), ea.to(DEV)
    pair = _steps(conv, state, x, eid, ead, epilogue, [False, False, False], monkeypatch)
    mixed = _steps(conv, state, x, eid, ead, epilogue, [True, False, True], monkeypatch)
    for a_step, b_step in zip(mixed[0], pair[0]):
        for a, b in zip(a_step, b_step):
            assert torch.equal(a, b)
    assert torch.equal(mixed[1], pair[1]) and torch.equal(mixed[2], pair[2])
    assert mixed[3] == pair[3] == 3
    from test_gpu_bnacc import BAR_WORDS, phase_index
    acc = Fn._BN_ACC[conv.nn[1]][(DEV, "fwd")]
    ph = phase_index(128)
    assert int(acc[ph]) == 6 and int(acc[ph + 1 + (6 & 1)]) == 6   # phase / consumed
    bar = acc[ph + 3:].view(-1, 16)[:, 0]                 # one word per 128-byte line
    assert bar.numel() == BAR_WORDS // 16
    assert int(bar[:10].abs().sum()) == 0                 # every arrival count back at zero
    gens = bar[10:18]                                     # per-XCD generations: one per launch
    assert int(gens.max()) == 2 and int(gens.min()) >= 0


def test_layer_forward_ok_limits():
    ok = ctypes.c_int32(7)
    for n, D, deg, want in [(16000, 128, 11, 1), (16000, 64, 11, 0), (16000, 128, 33, 0),
                            (128000, 128, 11, 0), (1, 128, 0, 1)]:
        _lib.call("gine_mp_fwd_layer_ok", n, D, deg, ctypes.byref(ok))
        assert ok.value == want, (n, D, deg)


@pytest.mark.parametrize("hidden", [128, 64])
def test_model_step_same_bits_with_and_without_layer_launches(hidden, monkeypatch):
    """The benchmark's training step (cfg2: 32 x 500 stations in the locality order, where the
    window backward carries the weight-gradient engine and the BatchNorm backward sums go
    through the accumulator): predictions, loss and every gradient are the same bits with the
    one-launch forward / backward layers on or off, over two steps."""
    import copy
    from helpers import engine_order_batch
    from raincast_gnn import functional as F
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import gnn_from_params
    from raincast_gnn.params import BENCH_CONFIGS
    c = BENCH_CONFIGS[2].with_hidden(hidden)
    batch = engine_order_batch(synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k,
                                               seed=11)).to(DEV)
    torch.manual_seed(5)
    base = gnn_from_params(c.params()).to(DEV).train()

    def run(fwd):
        monkeypatch.setattr(options, "LAYER_FWD", fwd)
        m = copy.deepcopy(base)
        out = []
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            pred = m(batch)
            loss = m.loss_fn.crps(pred, batch.y)
            loss.backward()
            out.append([pred.detach().clone(), loss.detach().clone()]
                       + [p.grad.clone() for p in m.parameters()]
                       + [b.clone() for b in m.buffers()])
        torch.cuda.synchronize()
        return out

    n = batch.num_nodes
    monkeypatch.setattr(options, "LAYER_FWD", True)
    if hidden == 128:
        assert F.layer_forward_ok(n, hidden, c.k + 1)
    ref = run(False)
    got = run(True)
    for a_step, b_step in zip(got, ref):
        for a, b in zip(a_step, b_step):
            assert torch.equal(a, b)


def test_layer_barrier_failure_is_loud(monkeypatch):
    """A grid the device cannot hold at once (gine_testing_layer_extra_workgroups adds one
    workgroup per CU beyond the resident limit): the resident workgroups' barrier times out
    (~2 s), their rows come out NaN, the running statistics stay untouched, and
    check_grid_barriers raises GineError and resets the accumulator -- after which the
    production grid gives the pair's bits again."""
    ei, ea, n = knn_batch_graph(500, 10, 32, seed=510)
    conv = _conv(seed=3)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    x = torch.randn(n, 128, device=DEV) * 1.5 + 0.2
    eid, ead = ei.to(DEV), ea.to(DEV)
    monkeypatch.setattr(options, "LAYER_FWD", True)
    assert Fn.layer_forward_ok(n, 128, 11)
    Fn.check_grid_barriers()  # nothing pending from earlier tests
    bn = conv.nn[1]
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    _lib.call("gine_testing_layer_extra_workgroups", cus)
    try:
        with torch.no_grad():
            y = conv.forward_residual_relu(x, eid, ead)
        torch.cuda.synchronize()
    finally:
        _lib.call("gine_testing_layer_extra_workgroups", 0)
    assert torch.isnan(y).any(), "the workgroups whose barrier failed must poison their rows"
    assert torch.equal(bn.running_mean, rm0) and torch.equal(bn.running_var, rv0)
    nbt0 = bn.num_batches_tracked.clone()
    # the failure is sticky on the device: production launches on the same
    # accumulator before the host's check -- the one-launch layer and the pair -- give NaN
    # everywhere and leave the running statistics alone, never finite-but-wrong statistics
    for layer in (True, False):
        monkeypatch.setattr(options, "LAYER_FWD", layer)
        with torch.no_grad():
            y2 = conv.forward_residual_relu(x, eid, ead)
        torch.cuda.synchronize()
        assert torch.isnan(y2).all(), layer
        assert torch.equal(bn.running_mean, rm0) and torch.equal(bn.running_var, rv0), layer
        assert torch.equal(bn.num_batches_tracked, nbt0), layer
    monkeypatch.setattr(options, "LAYER_FWD", True)
    with pytest.raises(_lib.GineError, match="grid barrier timed out"):
        Fn.check_grid_barriers()
    acc = Fn._BN_ACC[bn][(DEV, "fwd")]
    assert int(acc.abs().sum()) == 0                      # reset for a fresh pairing
    assert torch.equal(bn.running_mean, rm0) and torch.equal(bn.running_var, rv0)
    Fn.check_grid_barriers()                              # reported once
    # the production grid afterwards: the layer launch and the pair agree bit for bit again
    got = _steps(conv, state, x, eid, ead, "residual", [True], monkeypatch)
    ref = _steps(conv, state, x, eid, ead, "residual", [False], monkeypatch)
    for a, b in zip(got[0][0], ref[0][0]):
        assert torch.equal(a, b)
    Fn.check_grid_barriers()


def test_layer_forward_refused_when_ranks_share_the_device(monkeypatch):
    from raincast_gnn import distributed
    monkeypatch.setattr(options, "LAYER_FWD", True)
    assert Fn.layer_forward_ok(16000, 128, 11)
    monkeypatch.setattr(distributed, "_SHARED_DEVICE", True)
    assert not Fn.layer_forward_ok(16000, 128, 11)
