"""GPU: the one-launch node-MLP backward (gine_mlp_bwd_layer: dbn GEMM + BatchNorm-backward
sums, grid barrier, BatchNorm-backward finish + dz GEMM; csrc/gine_mlpbwd.hip) against the
two-launch pair it replaces (gine_mlp_bwd2_acc + gine_mlp_bwd1_bn).

Same tile -> workgroup map, integer BatchNorm totals, the row GEMM's chains, prologues and
epilogue: every output must be the same bits -- dbn, dz, coef, dgamma, dbeta -- over several
steps on one accumulator with the two forms interleaved (the pairing protocol of
csrc/gine_bnacc.hpp must carry across them), and the model's training step must give the same
bits with the layer backward on or off.
"""
import copy
import ctypes

import pytest
import torch

from raincast_gnn import _lib, functional as Fn, options

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
D = 128


def _inputs(N, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    a1 = (torch.randn(N, D, generator=g) * 1.3 + 0.1).to(DEV)
    gamma = (torch.rand(D, generator=g) + 0.5).to(DEV)
    beta = (torch.rand(D, generator=g) * 0.4 - 0.2).to(DEV)
    mean = a1.double().mean(0)
    var = a1.double().var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    alpha = gamma.double() * invstd
    bn_save = torch.stack([mean.float(), invstd.float(), alpha.float(),
                           (beta.double() - mean * alpha).float()]).contiguous()
    dy = torch.randn(N, D, generator=g).to(DEV)
    y = torch.randn(N, D, generator=g).to(DEV)
    mask = (torch.rand(N, D, generator=g) > 0.4).to(torch.uint8).to(DEV)
    w1 = (torch.randn(D, D, generator=g) / 11).to(DEV)
    w2 = (torch.randn(D, D, generator=g) / 11).to(DEV)
    return dict(a1=a1, gamma=gamma, bn_save=bn_save, dy=dy, y=y, mask=mask, w1=w1, w2=w2)


def _run(form, t, acc, N, epi):
    c, p = _lib.call, _lib.ptr
    s = _lib.stream_handle(DEV)
    dbn, dz = torch.empty(N, D, device=DEV), torch.empty(N, D, device=DEV)
    coef = torch.empty(3, D, device=DEV)
    dg, db = torch.empty(D, device=DEV), torch.empty(D, device=DEV)
    y = p(t["y"]) if epi == 1 else None
    mask = p(t["mask"]) if epi == 2 else None
    if form == "layer":
        c("gine_mlp_bwd_layer", p(t["dy"]), y, mask, p(t["a1"]), p(t["bn_save"]), p(t["w2"]),
          p(dbn), p(acc), p(t["gamma"]), p(dg), p(db), p(coef), p(t["w1"]), p(dz), N, D, epi, s)
    else:
        c("gine_mlp_bwd2_acc", p(t["dy"]), y, mask, p(t["a1"]), p(t["bn_save"]), p(t["w2"]),
          p(dbn), None, p(acc), N, D, epi, s)
        c("gine_mlp_bwd1_bn", p(dbn), p(t["a1"]), p(t["bn_save"]), p(acc), p(t["gamma"]), p(dg),
          p(db), p(coef), p(t["w1"]), p(dz), N, D, s)
    return [dbn, dz, coef, dg, db]


@pytest.mark.parametrize("N", [16000, 5000, 7777, 33], ids=["cfg2", "1tile", "ragged", "tiny"])
@pytest.mark.parametrize("epi", [0, 1, 2], ids=["none", "relu", "residual"])
def test_layer_backward_equals_pair(N, epi):
    ok = ctypes.c_int32(0)
    _lib.call("gine_mlp_bwd_layer_ok", N, D, ctypes.byref(ok))
    assert ok.value == 1, "the one-launch backward must apply at this size"
    t = _inputs(N, seed=N + epi)
    words = Fn._count64("gine_bn_acc_words", D)
    acc_a = torch.zeros(words, dtype=torch.int64, device=DEV)
    acc_b = torch.zeros(words, dtype=torch.int64, device=DEV)
    for step, form in enumerate(["layer", "pair", "layer"]):
        ref = _run("pair", t, acc_a, N, epi)
        got = _run(form, t, acc_b, N, epi)
        torch.cuda.synchronize()
        for i, (a, b) in enumerate(zip(got, ref)):
            assert torch.equal(a, b), (step, form, ["dbn", "dz", "coef", "dgamma", "dbeta"][i])
        assert torch.isfinite(got[1]).all()
    from test_gpu_bnacc import phase_index
    ph = phase_index(D)
    assert torch.equal(acc_a[:ph + 3], acc_b[:ph + 3])  # totals, snapshots, phase, consumed
    assert int(acc_b[ph]) == 3 and int(acc_b[ph + 1 + (3 & 1)]) == 3
    bar = acc_b[ph + 3:].view(-1, 16)[:, 0]           # one word per 128-byte line
    assert int(bar[:10].abs().sum()) == 0              # arrival counts back at zero, no failure
    assert int(bar[10:18].max()) == 2                  # per-XCD generations: two layer launches


def test_layer_backward_ok_limits():
    ok = ctypes.c_int32(7)
    for n, d, want in [(16000, 128, 1), (16000, 64, 0), (128000, 128, 0), (1, 128, 1)]:
        _lib.call("gine_mlp_bwd_layer_ok", n, d, ctypes.byref(ok))
        assert ok.value == want, (n, d)
    with pytest.raises(_lib.GineError):
        t = _inputs(128000, seed=1)
        acc = torch.zeros(Fn._count64("gine_bn_acc_words", D), dtype=torch.int64, device=DEV)
        _run("layer", t, acc, 128000, 2)


def test_layer_backward_barrier_failure_is_loud():
    """A grid the device cannot hold at once: the resident workgroups' barrier times out
    (~2 s), the failure word counts them and their dz rows come out NaN; after the grid is
    restored (and the accumulator re-zeroed, as check_grid_barriers does) the layer and the
    pair agree again."""
    N, epi = 16000, 2
    t = _inputs(N, seed=3)
    words = Fn._count64("gine_bn_acc_words", D)
    acc = torch.zeros(words, dtype=torch.int64, device=DEV)
    idx = ctypes.c_int64(0)
    _lib.call("gine_bn_acc_barrier_failures_index", D, ctypes.byref(idx))
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    _lib.call("gine_testing_bwd_layer_extra_workgroups", cus)
    try:
        out = _run("layer", t, acc, N, epi)
        torch.cuda.synchronize()
    finally:
        _lib.call("gine_testing_bwd_layer_extra_workgroups", 0)
    assert int(acc[idx.value]) > 0, "the barrier failure must be counted"
    assert torch.isnan(out[1]).any(), "the workgroups whose barrier failed must poison dz"
    acc.zero_()
    acc_ref = torch.zeros_like(acc)
    got = _run("layer", t, acc, N, epi)
    ref = _run("pair", t, acc_ref, N, epi)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_layer_backward_refused_when_ranks_share_the_device(monkeypatch):
    from raincast_gnn import distributed
    monkeypatch.setattr(options, "LAYER_BWD", True)
    assert Fn.layer_backward_ok(16000, 128)
    monkeypatch.setattr(distributed, "_SHARED_DEVICE", True)
    assert not Fn.layer_backward_ok(16000, 128)


def test_model_step_same_bits_with_and_without_layer_backward(monkeypatch):
    """The benchmark's training step (cfg2, the locality order: the window backward carries
    the weight-gradient engine and the BatchNorm-backward sums go through the accumulator):
    predictions, loss, every gradient and buffer are the same bits with the one-launch
    backward on or off, over two steps, through the Python autograd Function and the C++
    binding alike."""
    from helpers import engine_order_batch
    from raincast_gnn import nn as rnn
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import gnn_from_params
    from raincast_gnn.params import BENCH_CONFIGS
    c = BENCH_CONFIGS[2]
    batch = engine_order_batch(synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k,
                                               seed=13)).to(DEV)
    torch.manual_seed(6)
    base = gnn_from_params(c.params()).to(DEV).train()
    assert Fn.layer_backward_ok(batch.num_nodes, 128)

    def run(bwd, ext):
        monkeypatch.setattr(options, "LAYER_BWD", bwd)
        monkeypatch.setattr(rnn, "USE_TORCH_EXT", ext)
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

    ref = run(False, False)
    for ext in (False, True):
        got = run(True, ext)
        for a_step, b_step in zip(got, ref):
            for a, b in zip(a_step, b_step):
                assert torch.equal(a, b), ext
    Fn.check_grid_barriers()


@pytest.mark.parametrize("bad", [float("inf"), float("nan"), float("-inf")],
                         ids=["inf", "nan", "-inf"])
def test_layer_kernels_nonfinite_follow_oracle(bad, monkeypatch):
    """D = 128 train-mode layer with a non-finite input value through the one-launch forward
    and backward (their split-plane chains redo a non-finite tile on the fp32 chain): the
    NaN / Inf pattern of y, of the running statistics and of every gradient equals the CPU
    oracle's."""
    import copy
    from oracle import gine_cpu as O
    from helpers import knn_batch_graph
    from test_gpu_bnacc import _cls, _conv
    from raincast_gnn import nn as rnn
    monkeypatch.setattr(rnn, "USE_TORCH_EXT", False)
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=21)
    assert Fn.layer_forward_ok(n, D, 11) and Fn.layer_backward_ok(n, D)
    conv = _conv(D, seed=4)
    ref = O.OracleGINEConv(copy.deepcopy(conv.nn).cpu(), train_eps=True, edge_dim=1)
    ref.load_state_dict({k: v.cpu() for k, v in conv.state_dict().items()})
    ref.train()
    x = torch.randn(n, D)
    x[321, 17] = bad
    xg = x.to(DEV).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = conv.forward_residual_relu(xg, ei.to(DEV), ea.to(DEV))
    yr = xr + torch.relu(ref(xr, ei, ea))
    w = torch.linspace(-1, 1, y.numel()).view_as(yr)
    (y * w.to(DEV)).sum().backward()
    (yr * w).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(_cls(y.detach().cpu()), _cls(yr.detach()))
    for buf in ("running_mean", "running_var"):
        assert torch.equal(_cls(getattr(conv.nn[1], buf).cpu()), _cls(getattr(ref.nn[1], buf)))
    assert torch.equal(_cls(xg.grad.cpu()), _cls(xr.grad))
    refp = dict(ref.named_parameters())
    for name, p in conv.named_parameters():
        assert torch.equal(_cls(p.grad.cpu()), _cls(refp[name].grad)), name
    Fn.check_grid_barriers()
