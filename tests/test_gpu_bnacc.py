"""GPU: BatchNorm statistics summed by fixed-point integer atomics and finished inside the
second node-MLP GEMM (gine_mlp_fwd1_acc / gine_mp_fwd_mlp1_acc + gine_mlp_fwd2_bn,
csrc/gine_bnacc.hpp) against the finish-launch path (partials -> gine_bn_fwd_finalize ->
gine_mlp_fwd2).  The layer uses it by default in training mode (options.BN_ACC = False turns it
off), so test_gpu_parity.py's test_gine_layer_fused also checks it against the oracle.

Tolerance: the fixed-point sums round each workgroup's fp64 partial to 2^-64, so mean and
variance agree with the fp64 partials path to ~1e-15 relative; alpha / shift may differ in
their last fp32 bit, y by a few ulp (1e-5 relative bound written below).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from raincast_gnn import options

from helpers import knn_batch_graph
from raincast_gnn import GINEConv, _lib, functional as Fn
from raincast_gnn.graph import GineGraph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def _words(D):
    w = ctypes.c_int64(0)
    assert _lib.load().gine_bn_acc_words(D, ctypes.byref(w)) == 0
    return w.value


BAR_WORDS = (2 + 2 * 8) * 16  # gine_bnacc.hpp kBarWords: the grid-barrier lines at the end


def _replicas(D):
    """Replica count of the accumulator layout (gine_bnacc.hpp): words = (3R + 9) 2D + 3 +
    BAR_WORDS (phase, two consumed words, then the grid-barrier words)."""
    return ((_words(D) - 3 - BAR_WORDS) // (2 * D) - 9) // 3


def phase_index(D):
    """Offset of the phase word (consumed[2] follow it)."""
    return _words(D) - 3 - BAR_WORDS


def _conv(D, seed):
    torch.manual_seed(seed)
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    with torch.no_grad():
        mlp[1].weight.uniform_(0.5, 1.5)
        mlp[1].bias.uniform_(-0.2, 0.2)
    return conv.to(DEV).train()


def _run(conv, state, x, ei, ea, steps, epilogue):
    conv.load_state_dict(state)
    fn = {"none": conv.forward, "relu": conv.forward_relu,
          "residual": conv.forward_residual_relu}[epilogue]
    ys = [fn(x, ei, ea) for _ in range(steps)]
    torch.cuda.synchronize()
    bn = conv.nn[1]
    return ys, bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked)


@pytest.mark.parametrize("D", [32, 64, 128, 256])
@pytest.mark.parametrize("epilogue", ["none", "relu", "residual"])
def test_bn_acc_matches_finish_launch(D, epilogue, monkeypatch):
    ei, ea, n = knn_batch_graph(400, 8, 3, seed=D)
    conv = _conv(D, seed=D)
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    x = torch.randn(n, D, device=DEV) * 2 + 0.5
    eid, ead = ei.to(DEV), ea.to(DEV)
    monkeypatch.setattr(options, "BN_ACC", False)
    ref = _run(conv, state, x, eid, ead, 3, epilogue)
    monkeypatch.setattr(options, "BN_ACC", True)
    got = _run(conv, state, x, eid, ead, 3, epilogue)
    for a, b in zip(got[0], ref[0]):   # three steps: each consumer differences against the snapshot of the last
        assert ((a - b).abs() <= TOL * (1 + b.abs())).all()
    torch.testing.assert_close(got[1], ref[1], rtol=TOL, atol=TOL)
    torch.testing.assert_close(got[2], ref[2], rtol=TOL, atol=TOL)
    assert got[3] == ref[3] == 3
    acc = Fn._BN_ACC[conv.nn[1]][(DEV, "fwd")]
    ph = phase_index(D)
    assert acc.numel() == _words(D) and int(acc[ph]) == 3   # phase: one per producer launch
    assert int(acc[ph + 1 + (3 & 1)]) == 3                   # consumed: the last consumer


def test_bn_acc_deterministic(monkeypatch):
    monkeypatch.setattr(options, "BN_ACC", True)
    ei, ea, n = knn_batch_graph(2000, 16, 4, seed=7)
    conv = _conv(128, seed=3)
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    x = torch.randn(n, 128, device=DEV)
    eid, ead = ei.to(DEV), ea.to(DEV)
    runs = [_run(conv, state, x, eid, ead, 2, "residual") for _ in range(3)]
    for r in runs[1:]:
        for a, b in zip(r[0], runs[0][0]):
            assert torch.equal(a, b)
        assert torch.equal(r[1], runs[0][1]) and torch.equal(r[2], runs[0][2])


def test_bn_acc_eval_and_momentum_none_use_finish_launch(monkeypatch):
    monkeypatch.setattr(options, "BN_ACC", True)
    conv = _conv(64, seed=1)
    bn = Fn.BnConfig(conv.nn[1])
    assert Fn.bn_accumulator(bn, 64, DEV) is not None
    conv.eval()
    assert Fn.bn_accumulator(Fn.BnConfig(conv.nn[1]), 64, DEV) is None
    conv.train()
    conv.nn[1].momentum = None
    assert Fn.bn_accumulator(Fn.BnConfig(conv.nn[1]), 64, DEV) is None


@pytest.mark.parametrize("n,max_deg", [(33, 3), (2049, 7), (16000, 11)])
def test_fused_forward_acc_equals_unfused(n, max_deg):
    """gine_mp_fwd_mlp1_acc and gine_mlp_fwd1_acc add the same workgroup sums: the integer
    accumulators agree word for word; z / a1 as the partials forms."""
    rng = np.random.default_rng(n)
    deg = rng.integers(0, max_deg + 1, n)
    dst = np.repeat(np.arange(n), deg)
    src = rng.integers(0, n, dst.size)
    ei = torch.tensor(np.stack([src, dst]), dtype=torch.long, device=DEV)
    ea = torch.from_numpy(rng.uniform(0.2, 5.0, (dst.size, 1)).astype(np.float32)).to(DEV)
    g = GineGraph(ei, ea, n)
    D = 128
    x = torch.randn(n, D, device=DEV)
    lw, lb = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    eps = torch.tensor([0.1], device=DEV)
    w1, b1 = torch.randn(D, D, device=DEV) / 11, torch.randn(D, device=DEV)
    p, s = _lib.ptr, _lib.stream_handle(DEV)
    acc1 = torch.zeros(_words(D), dtype=torch.int64, device=DEV)
    acc0 = torch.zeros_like(acc1)
    z1, a11 = torch.empty_like(x), torch.empty_like(x)
    _lib.call("gine_mp_fwd_mlp1_acc", p(x), p(g.in_rowptr), p(g.in_src), p(g.in_attr), p(lw),
              p(lb), p(eps), p(w1), p(b1), p(z1), p(a11), None, p(acc1), n, D,
              g.max_in_degree, 0, s)
    z0 = Fn.mp_forward(x, g, lw, lb, eps, lin_flag=0)
    a10 = torch.empty_like(x)
    _lib.call("gine_mlp_fwd1_acc", p(z0), p(w1), p(b1), p(a10), None, p(acc0), n, D, s)
    torch.cuda.synchronize()
    assert torch.equal(z1, z0) and torch.equal(a11, a10)
    assert torch.equal(acc1, acc0)
    # the totals are the column sums of a1 and a1^2
    a64 = a10.double()
    W = 2 * D
    R = _replicas(D)
    rep = acc0[:R * 3 * W].view(R, 3, W).sum(0)   # replicas: [hi | mid | lo] x (sum | sumsq)
    tot = (rep[0].double() + rep[1].double() * 2.0**-32 + rep[2].double() * 2.0**-64).view(2, D)
    torch.testing.assert_close(tot[0], a64.sum(0), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(tot[1], (a64 * a64).sum(0), rtol=1e-12, atol=1e-9)
    ph = phase_index(D)
    assert int(acc0[R * 3 * W:ph].abs().sum()) == 0       # no non-finite counts, no snapshot
    assert int(acc0[ph]) == 1 and int(acc0[ph + 1:].abs().sum()) == 0


def test_bn_acc_entry_points_validate():
    p, s = _lib.ptr, _lib.stream_handle(DEV)
    a = torch.zeros(64, 64, device=DEV)
    words = ctypes.c_int64(0)
    assert _lib.load().gine_bn_acc_words(64, ctypes.byref(words)) == 0
    # [R replicas x 3 words | 1 packed count word | 2 snapshots x 4 words] x 2D + 3 + barrier
    assert words.value == (3 * _replicas(64) + 1 + 8) * 128 + 3 + BAR_WORDS
    assert _replicas(64) == 4
    acc = torch.zeros(words.value, dtype=torch.int64, device=DEV)
    save = torch.empty(4, 64, device=DEV)
    w = torch.zeros(64, 64, device=DEV)
    b = torch.zeros(64, device=DEV)
    lib = _lib.load()
    # momentum=None (negative) and a missing accumulator are refused
    assert lib.gine_mlp_fwd2_bn(p(a), p(acc), None, None, None, None, None, p(save), -1.0,
                                1e-5, 0, p(w), p(b), None, p(a), None, 64, 64, 0, s) != 0
    assert lib.gine_mlp_fwd2_bn(p(a), None, None, None, None, None, None, p(save), 0.1,
                                1e-5, 0, p(w), p(b), None, p(a), None, 64, 64, 0, s) != 0
    assert lib.gine_mlp_fwd1_acc(p(a), p(w), p(b), p(a), None, None, 64, 64, s) != 0


@pytest.mark.parametrize("epilogue", ["none", "relu", "residual"])
def test_bn_acc_backward_matches_finish_launch(epilogue, monkeypatch):
    """gine_mlp_bwd2_acc + gine_mlp_bwd1_bn (taken with the window-plan backward, D = 128)
    against gine_mlp_bwd2 + gine_bn_bwd_finalize + gine_mlp_bwd1, over two steps."""
    monkeypatch.setattr(options, "MP_WINDOW", "all")
    monkeypatch.setattr(options, "BN_ACC_BWD", True)
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=11)
    conv = _conv(128, seed=5)
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    eid, ead = ei.to(DEV), ea.to(DEV)
    x0 = torch.randn(n, 128, device=DEV)
    dy = torch.randn(n, 128, device=DEV)
    fn = {"none": "forward", "relu": "forward_relu", "residual": "forward_residual_relu"}
    grads = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(options, "BN_ACC", mode == "1")
        conv.load_state_dict(state)
        out = []
        for _ in range(2):
            conv.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            getattr(conv, fn[epilogue])(x, eid, ead).backward(dy)
            out.append([x.grad.clone()] + [p.grad.clone() for p in conv.parameters()])
        torch.cuda.synchronize()
        grads[mode] = out
    for a_step, b_step in zip(grads["1"], grads["0"]):
        for a, b in zip(a_step, b_step):
            assert ((a - b).abs() <= 1e-4 * (1 + b.abs())).all()


def _fwd_pair(x, acc, bn, D, N, w1=None):
    """gine_mlp_fwd1_acc (a1 = x W1^T, W1 = I by default so a1 = x exactly), then
    gine_mlp_fwd2_bn; returns a1 and bn_save [mean | invstd | alpha | shift]."""
    p, s = _lib.ptr, _lib.stream_handle(DEV)
    eye, zero = torch.eye(D, device=DEV), torch.zeros(D, device=DEV)
    w1 = eye if w1 is None else w1
    a1 = torch.empty_like(x)
    _lib.call("gine_mlp_fwd1_acc", p(x), p(w1), p(zero), p(a1), None, p(acc), N, D, s)
    save = torch.empty(4, D, device=DEV)
    y = torch.empty_like(x)
    _lib.call("gine_mlp_fwd2_bn", p(a1), p(acc), p(bn["g"]), p(bn["b"]), p(bn["rm"]),
              p(bn["rv"]), None, p(save), 0.1, 1e-5, 1, p(eye), p(zero), None, p(y), None,
              N, D, 0, s)
    torch.cuda.synchronize()
    return a1, save


def _cls(t):
    """NaN / +Inf / -Inf classification of a tensor (for exact pattern comparisons)."""
    return torch.stack([t.isnan(), t == float("inf"), t == float("-inf")])


def _bn_state(D):
    return {"g": torch.rand(D, device=DEV) + 0.5, "b": torch.randn(D, device=DEV),
            "rm": torch.zeros(D, device=DEV), "rv": torch.ones(D, device=DEV)}


@pytest.mark.parametrize("case", ["nan", "+inf", "-inf", "both_inf"])
def test_bn_acc_nonfinite_follows_aten(case):
    """Non-finite column sums (csrc/gine_bnacc.hpp counts them): mean and the running
    statistics come out NaN / +Inf / -Inf exactly where ATen's train-mode batch_norm (CPU,
    on the same a1) puts them, finite entries within 1e-5; the next step is clean again."""
    N, D = 1000, 64
    x = torch.randn(N, D, device=DEV) * 3 + 1
    bad = {"nan": [(17, 0, float("nan"))], "+inf": [(5, 1, float("inf"))],
           "-inf": [(900, 2, float("-inf"))],
           "both_inf": [(3, 3, float("inf")), (600, 5, float("-inf"))]}[case]
    for r, c, v in bad:
        x[r, c] = v
    # W1 > 0 everywhere: a non-finite entry spreads over its a1 row with one sign
    w1 = torch.eye(D, device=DEV) + 1e-3
    bn = _bn_state(D)
    acc = torch.zeros(_words(D), dtype=torch.int64, device=DEV)
    a1, save = _fwd_pair(x, acc, bn, D, N, w1)
    a64 = a1.cpu().double()
    rm, rv = torch.zeros(D, dtype=torch.float64), torch.ones(D, dtype=torch.float64)
    torch.nn.functional.batch_norm(a64, rm, rv, training=True, momentum=0.1, eps=1e-5)
    assert not bool(torch.isfinite(a64.sum(0)).any())          # the case reached every column
    assert torch.equal(_cls(save[0].cpu()), _cls(a64.mean(0).float()))
    assert torch.equal(_cls(bn["rm"].cpu()), _cls(rm.float()))
    assert torch.equal(_cls(bn["rv"].cpu()), _cls(rv.float()))
    # the accumulator carries nothing into the next step
    bn2 = _bn_state(D)
    x2 = torch.randn(N, D, device=DEV)
    _, save2 = _fwd_pair(x2, acc, bn2, D, N)
    torch.testing.assert_close(save2[0].cpu().double(), x2.cpu().double().mean(0),
                               rtol=TOL, atol=TOL)


def test_bn_acc_out_of_range_column_is_nan():
    """The documented divergence: a finite workgroup column sum of 2^52 or more is counted as
    NaN (no silent fixed-point wrap); other columns are unaffected."""
    N, D = 1000, 64
    x = torch.randn(N, D, device=DEV)
    x[:, 4] = 3e16
    bn = _bn_state(D)
    acc = torch.zeros(_words(D), dtype=torch.int64, device=DEV)
    a1, save = _fwd_pair(x, acc, bn, D, N)
    assert torch.equal(a1, x)
    assert bool(save[0, 4].isnan()) and bool(bn["rm"][4].isnan())
    fin = [c for c in range(D) if c != 4]
    x64 = x.cpu().double()
    torch.testing.assert_close(save[0].cpu()[fin].double(), x64.mean(0)[fin], rtol=TOL,
                               atol=TOL)
    rv = 0.9 + 0.1 * x64.var(0, unbiased=True)
    torch.testing.assert_close(bn["rv"].cpu()[fin].double(), rv[fin], rtol=TOL, atol=TOL)


def test_bn_acc_layer_with_nonfinite_input_matches_oracle():
    """Train-mode GINE layer (default accumulator path) with +Inf / NaN in x against the CPU
    oracle: equal NaN / Inf pattern of y and of the running statistics, finite running
    means within 1e-5."""
    from oracle import gine_cpu as O
    import copy
    ei, ea, n = knn_batch_graph(300, 8, 2, seed=4)
    for bad in (float("inf"), float("nan"), float("-inf")):
        conv = _conv(64, seed=9)
        ref = O.OracleGINEConv(copy.deepcopy(conv.nn).cpu(), train_eps=True, edge_dim=1)
        ref.load_state_dict({k: v.cpu() for k, v in conv.state_dict().items()})
        ref.train()
        x = torch.randn(n, 64)
        x[123, 7] = bad
        y = conv.forward_residual_relu(x.to(DEV), ei.to(DEV), ea.to(DEV))
        yr = x + torch.relu(ref(x, ei, ea))
        torch.cuda.synchronize()
        assert torch.equal(_cls(y.cpu()), _cls(yr)), bad
        for buf in ("running_mean", "running_var"):
            g, r = getattr(conv.nn[1], buf).cpu(), getattr(ref.nn[1], buf)
            assert torch.equal(_cls(g), _cls(r)), (bad, buf)
            f = torch.isfinite(r)
            torch.testing.assert_close(g[f], r[f], rtol=TOL, atol=TOL)


def test_bn_acc_pairing_break_gives_nan_then_recovers():
    """A producer launch without its consumer (the pairing gine_bnacc.hpp requires) makes
    the next consumer emit NaN statistics instead of mixing two steps; the pair after it is
    exact again."""
    N, D = 512, 32
    p, s = _lib.ptr, _lib.stream_handle(DEV)
    acc = torch.zeros(_words(D), dtype=torch.int64, device=DEV)
    bn = {"g": None, "b": None, "rm": torch.zeros(D, device=DEV),
          "rv": torch.ones(D, device=DEV)}
    x = torch.randn(N, D, device=DEV)
    _, save = _fwd_pair(x, acc, bn, D, N)
    torch.testing.assert_close(save[0].double(), x.double().mean(0), rtol=TOL, atol=TOL)
    eye, zero = torch.eye(D, device=DEV), torch.zeros(D, device=DEV)
    a1 = torch.empty_like(x)
    _lib.call("gine_mlp_fwd1_acc", p(x), p(eye), p(zero), p(a1), None, p(acc), N, D, s)
    _, save = _fwd_pair(x, acc, bn, D, N)      # two producers, one consumer
    assert bool(save[0].isnan().all())
    x3 = torch.randn(N, D, device=DEV) + 2
    _, save = _fwd_pair(x3, acc, bn, D, N)
    torch.testing.assert_close(save[0].double(), x3.double().mean(0), rtol=TOL, atol=TOL)


def test_bn_acc_backward_small_gradients(monkeypatch):
    """Gradients of order 1e-10 (the ADVICE case): the backward accumulator's 2^-64
    resolution keeps them within 1e-5 (max-norm relative) of the fp64-partials path."""
    monkeypatch.setattr(options, "MP_WINDOW", "all")
    ei, ea, n = knn_batch_graph(500, 10, 4, seed=12)
    conv = _conv(128, seed=6)
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    eid, ead = ei.to(DEV), ea.to(DEV)
    x0 = torch.randn(n, 128, device=DEV)
    dy = torch.randn(n, 128, device=DEV) * 1e-10
    grads = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(options, "BN_ACC_BWD", mode == "1")
        conv.load_state_dict(state)
        conv.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        conv.forward_residual_relu(x, eid, ead).backward(dy)
        torch.cuda.synchronize()
        grads[mode] = [x.grad.clone()] + [p.grad.clone() for p in conv.parameters()]
    names = ["x"] + [n for n, _ in conv.named_parameters()]
    w1 = dict(zip(names, grads["0"]))["nn.0.weight"]
    for name, a, b in zip(names, grads["1"], grads["0"]):
        den = float(b.abs().max())
        if name == "nn.0.bias":
            # analytically zero behind train-mode BatchNorm: rounding noise of sum_n d a1,
            # whose scale is that of the weight gradient sum_n d a1 z (z ~ 1)
            den = max(den, float(w1.abs().max()))
        assert float((a - b).abs().max()) <= TOL * den + 1e-30, name
