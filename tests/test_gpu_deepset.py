"""Fused DeepSet phi kernels (csrc/gine_deepset.hip) against an fp64 restatement of
models/gnn.py:48-68's ``relu(phi[0](ens)).sum(dim=1)`` and its weight gradients.

Tolerances are condition-scaled (fp32 accumulation vs an exact fp64 sum): elementwise
``|gpu - exact| <= 1e-5 * sum|terms|``.  The weight gradients are held against the exact
gradients of the branch the kernel took: its ReLU decisions are read from the bit mask its
forward saved, and each one that differs from the fp64 sign must lie within that decision's
forward rounding bound (tests/helpers.EngineTies' phi[0] bound, 2 gamma_F (|ens||W|^T + |b|)).
"""
import ctypes

import pytest
import torch

from raincast_gnn import _lib, deepset
from raincast_gnn.models import DeepSetEncoder

from helpers import ctypes_int, decode_deepset_mask, gamma_dot

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def _exact(ens, w, b):
    e64, w64, b64 = ens.double(), w.double(), b.double()
    pre = e64 @ w64.T + b64                                      # [N, M, H]
    mag = e64.abs() @ w64.abs().T + b64.abs()                    # condition of each pre
    return pre, mag


def _run(N, M, F, H, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ens = (torch.randn(N, M, F, generator=g) * scale).to(DEV)
    w = (torch.randn(H, F, generator=g) / F ** 0.5).to(DEV).requires_grad_()
    b = (torch.randn(H, generator=g) * 0.1).to(DEV).requires_grad_()
    lin = torch.nn.Linear(F, H).to(DEV)
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.copy_(b)
    return ens, lin


@pytest.mark.parametrize("N,M,F,H", [
    (1, 1, 1, 32), (31, 11, 35, 128), (33, 11, 35, 128), (1000, 11, 35, 128),
    (16000, 11, 35, 128), (257, 1, 16, 64), (100, 33, 64, 256), (77, 5, 20, 32),
    (500, 51, 35, 128), (64, 2, 40, 128), (65, 3, 48, 64), (90, 7, 33, 128), (40, 4, 61, 32),
    # short last groups (whole tiles past N*M rows): N % 32 != 0
    (65, 11, 35, 128), (610, 10, 35, 128), (33, 10, 35, 128), (97, 11, 35, 256)])
def test_phi_sum_forward_and_weight_grads(N, M, F, H):
    ens, lin = _run(N, M, F, H, seed=N + M + F + H)
    r = deepset.phi_sum(ens, lin)
    pre, mag = _exact(ens, lin.weight.detach(), lin.bias.detach())
    r64 = pre.clamp_min(0).sum(1)
    assert ((r.double() - r64).abs() <= TOL * mag.sum(1) + 1e-30).all()

    # the kernel's ReLU decisions (its saved bit mask) against the fp64 signs: a differing
    # decision must lie within its own forward rounding bound
    words = r.grad_fn.saved_tensors[1].detach().cpu().numpy().view("uint16")
    G = ctypes_int(lambda out: _lib.call("gine_deepset_mask_layout", N, H, out))
    on = torch.from_numpy(decode_deepset_mask(words, N, M, H, G)).to(DEV)
    diff = on != (pre > 0)
    beta = 2 * gamma_dot(F) * mag
    assert (pre.abs()[diff] <= beta[diff]).all(), "a ReLU decision outside its rounding bound"

    dr = torch.randn(N, H, device=DEV)
    r.backward(dr)
    live = on.double() * dr.double()[:, None, :]                 # [N, M, H], kernel's branch
    e64 = ens.double()
    dw64 = torch.einsum("nmh,nmf->hf", live, e64)
    db64 = live.sum((0, 1))
    bound_w = TOL * torch.einsum("nmh,nmf->hf", live.abs(), e64.abs()) + 1e-30
    bound_b = TOL * live.abs().sum((0, 1)) + 1e-30
    assert ((lin.weight.grad.double() - dw64).abs() <= bound_w).all()
    assert ((lin.bias.grad.double() - db64).abs() <= bound_b).all()


def test_phi_sum_deterministic():
    ens, lin = _run(16000, 11, 35, 128, seed=3)
    dr = torch.randn(16000, 128, device=DEV)
    outs = []
    for _ in range(2):
        lin.zero_grad(set_to_none=True)
        r = deepset.phi_sum(ens, lin)
        r.backward(dr)
        outs.append((r.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_phi_sum_eval_has_no_mask():
    """Without grad the forward runs alone (no mask buffer) and gives the same r."""
    ens, lin = _run(1000, 11, 35, 128, seed=7)
    r_train = deepset.phi_sum(ens, lin)
    with torch.no_grad():
        r_eval = deepset.phi_sum(ens, lin)
    assert torch.equal(r_train, r_eval)


def test_phi_sum_empty():
    ens, lin = _run(0, 11, 35, 128)
    r = deepset.phi_sum(ens, lin)
    assert r.shape == (0, 128)
    r.sum().backward()
    assert torch.count_nonzero(lin.weight.grad) == 0
    assert torch.count_nonzero(lin.bias.grad) == 0


def test_deepset_encoder_fused_matches_unfused():
    """The encoder dispatches to the fused kernels; it equals the torch formulation."""
    torch.manual_seed(0)
    enc = DeepSetEncoder(35, 128, 128).to(DEV)
    ens = torch.randn(2000, 11, 35, device=DEV)
    assert deepset.fusable(ens, enc.phi[0].weight, enc.phi[0].bias)
    out = enc(ens)
    out.square().sum().backward()
    g_fused = [p.grad.clone() for p in enc.parameters()]
    enc.zero_grad()
    lin1, act, lin2 = enc.phi
    ref = enc.rho(lin2(act(torch.nn.functional.linear(ens, lin1.weight, lin1.bias))).sum(1))
    ref.square().sum().backward()
    assert (out - ref).abs().max() <= 1e-4 * ref.abs().max()
    for gf, p in zip(g_fused, enc.parameters()):
        assert (gf - p.grad).abs().max() <= 1e-4 * p.grad.abs().max()


def test_abi_rejects_unsupported_shapes():
    x = torch.zeros(4, 2, 65, device=DEV)
    w = torch.zeros(128, 65, device=DEV)
    b = torch.zeros(128, device=DEV)
    r = torch.zeros(4, 128, device=DEV)
    s = _lib.stream_handle(DEV)
    lib = _lib.load()
    assert lib.gine_deepset_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(r), None, 4, 2,
                                65, 128, s) == _lib.GINE_ERR_DIM
    assert lib.gine_deepset_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(r), None, 4, 2,
                                35, 96, s) == _lib.GINE_ERR_DIM
    assert not deepset.fusable(x, w, b)
    n = ctypes.c_int32(0)
    assert lib.gine_deepset_bwd_num_partials(16000, 128, ctypes.byref(n)) == 0 and n.value == 500
    # H = 64: groups of 16 nodes up to 16,384 nodes, up to 1,024 partials
    assert lib.gine_deepset_bwd_num_partials(16000, 64, ctypes.byref(n)) == 0 and n.value == 1000
    assert lib.gine_deepset_bwd_num_partials(16000, 96, ctypes.byref(n)) == _lib.GINE_ERR_DIM
