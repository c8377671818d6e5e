"""CPU: the oracle against the reference's golden vectors and its own independent restatement."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from helpers import knn_batch_graph, random_graph
from oracle import gine_cpu as O

HEADS = os.path.join(GOLDEN, "reference_heads.npz")
CASES = [("normal", "NormalCRPS", "False"), ("normal_mixed", "MixedNormalCRPS", "False"),
         ("mixed", "MixedLoss", "False"), ("mixed_u", "MixedLoss", "True")]


def _params(D, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(D, 1, generator=g), torch.randn(D, generator=g),
            torch.tensor([0.3]))


def test_scatter_add_is_sequential_edge_order():
    """CPU scatter_add_ == per-destination sequential sum in original edge order (the order
    the HIP kernel reproduces), independent of the thread count."""
    ei, ea, n = random_graph(40, 4000, seed=1)  # ~100 in-edges per node: order matters
    x = torch.randn(n, 16) * torch.logspace(-3, 3, 16)
    lw, lb, eps = _params(16, 0)
    from raincast_gnn.functional import edge_linear_flag
    ref = O.gine_aggregate_loops(x, ei, ea, lw, lb, eps,
                                 "fma" if edge_linear_flag() == 0 else "muladd")
    old = torch.get_num_threads()
    try:
        for threads in (1, max(2, old)):
            torch.set_num_threads(threads)
            assert torch.equal(O.gine_aggregate(x, ei, ea, lw, lb, eps), ref)
    finally:
        torch.set_num_threads(old)


def test_index_add_backward_is_sequential_edge_order():
    ei, ea, n = random_graph(40, 3000, seed=2)
    D = 8
    x = (torch.randn(n, D) * 10).requires_grad_(True)
    lw, lb, eps = _params(D, 1)
    z = O.gine_aggregate(x, ei, ea, lw, lb, eps)
    dz = torch.randn_like(z) * torch.logspace(-2, 2, D)
    z.backward(dz)
    # restate: dx_j = sum_{e: src_e=j} dz[dst_e]*1[pre_e>0] (edge order) + (1+eps)*dz_j
    pre = x.detach()[ei[0]] + torch.nn.functional.linear(ea, lw, lb)
    dm = torch.where(pre > 0, dz[ei[1]], torch.zeros(()))
    acc = np.zeros((n, D), dtype=np.float32)
    dmn = dm.numpy()
    for e in range(ei.size(1)):
        s = ei[0, e].item()
        acc[s] = (acc[s] + dmn[e]).astype(np.float32)
    expect = torch.from_numpy(acc) + (1 + eps) * dz
    assert torch.equal(x.grad, expect)


def test_linear_k1_rounding_is_fma_or_muladd():
    """CPU Linear(1, D) rounds a*w+b either once (fma: MKL on Intel) or twice (mul, add: MKL on
    AMD EPYC); the kernel implements both and the host side probes which one applies."""
    from raincast_gnn.functional import edge_linear_flag
    g = torch.Generator().manual_seed(5)
    a = torch.randn(20000, 1, generator=g) * 3
    w = torch.randn(64, 1, generator=g)
    b = torch.randn(64, generator=g)
    got = torch.nn.functional.linear(a, w, b)
    fma = (a.double() * w.double().T + b.double()).float()  # exact product+sum, one rounding
    muladd = a * w.T + b
    assert torch.equal(got, fma) or torch.equal(got, muladd)
    assert edge_linear_flag() == (0 if torch.equal(got, fma) else 2)


def test_oracle_knn_layer_runs_and_is_deterministic():
    ei, ea, n = knn_batch_graph(100, 5, 2)
    torch.manual_seed(0)
    net = O.OracleResGnn(32, 32, 2, 32)
    x = torch.randn(n, 32)
    assert torch.equal(net(x, ei, ea), net(x, ei, ea))


@pytest.mark.parametrize("name,loss,grad_u", CASES)
def test_oracle_heads_match_reference(name, loss, grad_u):
    d = np.load(HEADS)
    raw = torch.from_numpy(d[f"{name}_raw"]).requires_grad_(True)
    y = torch.from_numpy(d[f"{name}_y"])
    pp = O.postprocess(raw, loss, grad_u)
    assert np.allclose(pp.detach().numpy(), d[f"{name}_pp"], rtol=1e-6, atol=1e-7)
    crps, _ = O.make_crps(loss, grad_u, 1.71, 0.5)
    val = crps(pp, y)
    assert str(val.dtype) == str(d[f"{name}_loss_dtype"][0])
    assert abs(val.item() - d[f"{name}_loss"][0]) <= 1e-6 * abs(d[f"{name}_loss"][0])
    val.backward()
    assert np.allclose(raw.grad.numpy(), d[f"{name}_grad"], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("name,loss,grad_u", CASES)
def test_package_heads_match_reference(name, loss, grad_u):
    """raincast_gnn's graph-capturable loss/PostProcess restatement vs the reference."""
    from raincast_gnn.models import make_loss
    from raincast_gnn.postprocess import PostProcess
    d = np.load(HEADS)
    raw = torch.from_numpy(d[f"{name}_raw"]).requires_grad_(True)
    y = torch.from_numpy(d[f"{name}_y"])
    pp = PostProcess(loss, grad_u)(raw)
    assert torch.equal(pp.detach(), torch.from_numpy(d[f"{name}_pp"]))
    fn, out = make_loss(loss, grad_u, 1.71, 0.5)
    assert out == raw.size(1)
    val = fn.crps(pp, y)
    assert str(val.dtype) == str(d[f"{name}_loss_dtype"][0])
    assert abs(val.item() - d[f"{name}_loss"][0]) <= 1e-6 * abs(d[f"{name}_loss"][0])
    val.backward()
    assert np.allclose(raw.grad.numpy(), d[f"{name}_grad"], rtol=1e-5, atol=1e-8)
    assert np.isfinite(raw.grad.numpy()).all()
