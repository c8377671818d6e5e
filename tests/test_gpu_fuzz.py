"""GPU: seeded random-graph sweeps of the fused launches against their unfused forms.

Each fused entry point has an unfused equivalent built from separately tested kernels, and
the fused form is specified to give the same bits.  These sweeps draw random multigraphs
(unsorted edges, uneven in-degrees up to the fused limit, isolated nodes, sizes that leave
partial 32-row tiles and workgroups with 0, 1 or several tiles) and check that claim:
  * gine_mp_fwd_mlp1           == gine_mp_fwd + gine_mlp_fwd1         (z, a1, BN partials)
  * gine_mp_bwd_win_mlp_wgrad  == gine_mp_bwd_win + gine_mlp_wgrad     (dx, partials, slab)
"""
import ctypes

import numpy as np
import pytest
import torch

from raincast_gnn import options

from raincast_gnn import _lib, functional as Fn
from raincast_gnn.graph import GineGraph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
D = 128


def _graph(seed: int, n: int, max_deg: int, local: int = 0):
    """Random in-degrees in [0, max_deg], sources uniform (or within +-local of the
    destination: block-diagonal-like locality, so window plans exist), edges shuffled."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(0, max_deg + 1, n)
    deg[rng.integers(0, n, max(1, n // 50))] = 0          # some isolated destinations
    dst = np.repeat(np.arange(n), deg)
    if local:
        src = np.clip(dst + rng.integers(-local, local + 1, dst.size), 0, n - 1)
    else:
        src = rng.integers(0, n, dst.size)
    perm = rng.permutation(dst.size)
    ei = torch.tensor(np.stack([src[perm], dst[perm]]), dtype=torch.long)
    ea = torch.from_numpy(rng.uniform(0.2, 5.0, (dst.size, 1)).astype(np.float32))
    return ei, ea


CASES = [(s, n, d) for s, (n, d) in enumerate(
    [(1, 3), (31, 32), (33, 1), (500, 11), (777, 20), (1024, 32), (2049, 7), (4000, 16),
     (9001, 12), (16000, 11), (16384, 5)])]


@pytest.mark.parametrize("seed,n,max_deg", CASES)
@pytest.mark.parametrize("flag", [0, _lib.GINE_MP_LIN_MULADD], ids=["fma", "muladd"])
def test_fused_forward_fuzz(seed, n, max_deg, flag, monkeypatch):
    monkeypatch.setattr(options, "MP_FUSED", "all")
    ei, ea = _graph(1000 + seed, n, max_deg)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    torch.manual_seed(seed)
    x = torch.randn(n, D, device=DEV)
    lw, lb = torch.randn(D, device=DEV) * 0.5, torch.randn(D, device=DEV) * 0.5
    eps = torch.tensor([0.05 * seed], device=DEV)
    w1, b1 = torch.randn(D, D, device=DEV) / 11, torch.randn(D, device=DEV)
    P = Fn._count("gine_mlp_num_partials", n, D)
    s = _lib.stream_handle(DEV)
    p = _lib.ptr
    z1, a11 = torch.full_like(x, 3.0), torch.full_like(x, 3.0)
    part1 = torch.full((P, 2, D), 3.0, dtype=torch.float64, device=DEV)
    _lib.call("gine_mp_fwd_mlp1", p(x), p(g.in_rowptr), p(g.in_src), p(g.in_attr), p(lw),
              p(lb), p(eps), p(w1), p(b1), p(z1), p(a11), p(part1), n, D, g.max_in_degree,
              flag, s)
    z0 = Fn.mp_forward(x, g, lw, lb, eps, lin_flag=flag)
    a10 = torch.empty_like(x)
    part0 = torch.empty(P, 2, D, dtype=torch.float64, device=DEV)
    _lib.call("gine_mlp_fwd1", p(z0), p(w1), p(b1), p(a10), p(part0), n, D, s)
    torch.cuda.synchronize()
    assert torch.equal(z1, z0)
    assert torch.equal(a11, a10)
    assert torch.equal(part1, part0)


@pytest.mark.parametrize("seed,n,max_deg", [c for c in CASES if c[1] >= 33])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_combined_backward_fuzz(seed, n, max_deg, epi, monkeypatch):
    monkeypatch.setattr(options, "MP_WINDOW", "all")
    ei, ea = _graph(2000 + seed, n, max_deg, local=150)
    g = GineGraph(ei.to(DEV), ea.to(DEV), n)
    plan = g.window_plan("out", D)
    if plan is None or plan.slice_channels != 32:
        pytest.skip("no 32-channel window plan for this graph")
    torch.manual_seed(seed)
    r = lambda *sh: torch.randn(*sh, device=DEV)  # noqa: E731
    dz, x, dy, y, a1, dbn, z = r(n, D), r(n, D), r(n, D), r(n, D), r(n, D), r(n, D), r(n, D)
    mask = (r(n, D) > 0).to(torch.uint8)
    bn_save = torch.cat([r(1, D) * 0.1, r(1, D).abs() + 0.5, r(1, D), r(1, D)]).contiguous()
    coef = r(3, D)
    lw, lb = r(D) * 0.5, r(D) * 0.5
    eps = torch.tensor([0.1], device=DEV)
    C = Fn._count("gine_mlp_wgrad_num_chunks", n, D)
    s = _lib.stream_handle(DEV)
    p = _lib.ptr
    flags = _lib.GINE_MP_BWD_SELF | Fn.edge_linear_flag()
    outs = []
    for fused in (True, False):
        dx = torch.full_like(x, 3.0)
        part = torch.full((plan.num_tiles, 3, D), 3.0, dtype=torch.float64, device=DEV)
        slab = torch.full((2 * C * (D * D + D),), 3.0, device=DEV)
        args = (p(dz), p(x), p(g.out_rowptr), p(g.out_dst), p(g.out_attr), p(lw), p(lb),
                p(eps), p(dy), p(dx), p(part), n, D, flags, ctypes.byref(plan))
        if fused:
            _lib.call("gine_mp_bwd_win_mlp_wgrad", *args, p(dy), p(y), p(mask), p(a1),
                      p(bn_save), p(dbn), p(coef), p(z), p(slab), epi, s)
        else:
            _lib.call("gine_mp_bwd_win", *args, s)
            _lib.call("gine_mlp_wgrad", p(dy), p(y), p(mask), p(a1), p(bn_save), p(dbn),
                      p(coef), p(z), p(slab), None, None, None, None, n, D, epi, s)
        outs.append((dx, part, slab))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
