"""Fused dense chain (csrc/gine_chain.hip): phi[2] (member-summed) -> rho -> dim_red of
models/gnn.py:48-68,112-113,132-135, forward and backward, against the same composition
of torch Linears in fp64.  All eight parameter gradients, dr (-> DeepSet backward) and h0
are checked at max-norm relative 1e-5 (fp32 MFMA accumulation over <= 16,000 rows), for
the folded chain (the default: rho[2] folded into dim_red) and the unfolded one."""
import pytest
import torch

from raincast_gnn import chain as fused_chain

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def _lins(D, F, seed):
    torch.manual_seed(seed)
    return (torch.nn.Linear(D, D).to(DEV), torch.nn.Linear(D, D).to(DEV),
            torch.nn.Linear(D, D).to(DEV), torch.nn.Linear(F + D, D).to(DEV))


def _ref(r, x, lins, M):
    p2, r0, r1, dr = [(m.weight.detach().double().requires_grad_(),
                       m.bias.detach().double().requires_grad_()) for m in lins]
    s = r @ p2[0].T + M * p2[1]
    u = torch.relu(s @ r0[0].T + r0[1])
    e = u @ r1[0].T + r1[1]
    h0 = torch.cat([x, e], 1) @ dr[0].T + dr[1]
    return h0, [t for pair in (p2, r0, r1, dr) for t in pair]


@pytest.fixture(params=[True, False], ids=["folded", "unfolded"])
def fold(request, monkeypatch):
    monkeypatch.setattr(fused_chain, "FOLD", request.param)
    return request.param


@pytest.mark.parametrize("N,D,F,M", [(1, 128, 35, 11), (33, 128, 35, 11), (16000, 128, 35, 11),
                                     (1000, 64, 35, 51), (257, 128, 64, 3), (70, 64, 8, 1)])
def test_chain_matches_torch_fp64(N, D, F, M, fold):
    lins = _lins(D, F, N + D + F)
    g = torch.Generator().manual_seed(N)
    r = (torch.randn(N, D, generator=g) * 3).to(DEV).requires_grad_()
    x = torch.randn(N, F, generator=g).to(DEV)
    assert fused_chain.fusable(r, x, lins)
    h0 = fused_chain.chain(r, x, lins, M)
    r64 = r.detach().double().requires_grad_()
    h64, params64 = _ref(r64, x.double(), lins, M)
    assert _rel(h0, h64) <= TOL
    dh = torch.randn(N, D, generator=g).to(DEV)
    h0.backward(dh)
    h64.backward(dh.double())
    assert _rel(r.grad, r64.grad) <= TOL, "dr"
    mine = [t for m in lins for t in (m.weight.grad, m.bias.grad)]
    names = ["dWp2", "dbp2", "dWr0", "dbr0", "dWr1", "dbr1", "dWdr", "dbdr"]
    for name, a, b in zip(names, mine, params64):
        assert _rel(a, b.grad) <= TOL, (name, _rel(a, b.grad))


def test_chain_deterministic(fold):
    lins = _lins(128, 35, 5)
    r = torch.randn(5000, 128, device=DEV, requires_grad=True)
    x = torch.randn(5000, 35, device=DEV)
    out = []
    for _ in range(2):
        for m in lins:
            m.zero_grad(set_to_none=True)
        r.grad = None
        h0 = fused_chain.chain(r, x, lins, 11)
        h0.backward(torch.ones_like(h0))
        out.append(torch.cat([h0.reshape(-1), r.grad.reshape(-1)]
                             + [m.weight.grad.reshape(-1) for m in lins]))
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("N,D,F", [(33, 128, 35), (300, 64, 35)])
def test_chain_bwd_intermediates(N, D, F):
    """de, dt, ds, dr of gine_chain_bwd one by one (C ABI) against fp64 torch."""
    import ctypes

    from raincast_gnn import _lib
    torch.manual_seed(1)
    f = lambda *s: torch.randn(*s, device=DEV)  # noqa: E731
    dh0, x, r, s, e = f(N, D), f(N, F), f(N, D), f(N, D), f(N, D)
    u = torch.relu(f(N, D))
    wp2, wr0, wr1, wdr = f(D, D) / 10, f(D, D) / 10, f(D, D) / 10, f(D, F + D) / 10
    de, dt, ds, dr = (torch.empty(N, D, device=DEV) for _ in range(4))
    fl = ctypes.c_size_t(0)
    _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(fl))
    slab = torch.empty(fl.value, device=DEV)
    g = [torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, F + D), 5.0, device=DEV), torch.empty(D, device=DEV)]
    P = _lib.ptr
    _lib.call("gine_chain_bwd", P(dh0), P(x), P(r), P(s), P(u), P(e), P(wp2), P(wr0), P(wr1),
              P(wdr), P(de), P(dt), P(ds), P(dr), P(slab), P(g[0]), P(g[1]), 1.0, P(g[2]),
              P(g[3]), P(g[4]), P(g[5]), P(g[6]), P(g[7]), N, D, F,
              _lib.stream_handle(DEV))
    torch.cuda.synchronize()
    d = lambda t: t.double()  # noqa: E731
    de64 = d(dh0) @ d(wdr)[:, F:]
    dt64 = (de64 @ d(wr1)) * (u > 0).double()
    ds64 = dt64 @ d(wr0)
    dr64 = ds64 @ d(wp2)
    assert _rel(de, de64) <= TOL, "de"
    assert _rel(dt, dt64) <= TOL, "dt"
    assert _rel(ds, ds64) <= TOL, "ds"
    assert _rel(dr, dr64) <= TOL, "dr"
    xe = torch.cat([d(x), d(e)], 1)
    for name, got, ref in (("dWp2", g[0], ds64.T @ d(r)), ("dbp2", g[1], ds64.sum(0)),
                           ("dWr0", g[2], dt64.T @ d(s)), ("dbr0", g[3], dt64.sum(0)),
                           ("dWr1", g[4], de64.T @ d(u)), ("dbr1", g[5], de64.sum(0)),
                           ("dWdr", g[6], d(dh0).T @ xe), ("dbdr", g[7], d(dh0).sum(0))):
        assert _rel(got, ref) <= TOL, (name, _rel(got, ref))


@pytest.mark.parametrize("N,D,F", [(33, 128, 35), (300, 64, 35), (2000, 128, 64)])
def test_chain_folded_intermediates(N, D, F):
    """The folded chain's pieces (C ABI) against fp64 torch: W' | b' from the forward, dt /
    ds / dr, the engine's G | g and the weight gradients unfolded from it."""
    import ctypes

    from raincast_gnn import _lib
    torch.manual_seed(2)
    f = lambda *s: torch.randn(*s, device=DEV)  # noqa: E731
    r, x = f(N, D), f(N, F)
    wp2, wr0, wr1, wdr = f(D, D) / 10, f(D, D) / 10, f(D, D) / 10, f(D, F + D) / 10
    bp2, br0, br1, bdr = f(D), f(D), f(D), f(D)
    s, u, h0 = (torch.empty(N, D, device=DEV) for _ in range(3))
    wfold = torch.full((2 * D * (F + D) + D,), float("nan"), device=DEV)
    P = _lib.ptr
    st = _lib.stream_handle(DEV)
    _lib.call("gine_chain_fwd_folded", P(r), P(x), P(wp2), P(bp2), 7.0, P(wr0), P(br0), P(wr1),
              P(br1), P(wdr), P(bdr), P(wfold), P(s), P(u), P(h0), N, D, F, st)
    d = lambda t: t.double()  # noqa: E731
    s64 = d(r) @ d(wp2).T + 7.0 * d(bp2)
    u64 = torch.relu(d(s) @ d(wr0).T + d(br0))
    e64 = d(u) @ d(wr1).T + d(br1)
    h64 = torch.cat([d(x), e64], 1) @ d(wdr).T + d(bdr)
    wc64 = d(wdr)[:, F:] @ d(wr1)
    torch.cuda.synchronize()
    W = wfold[:D * (F + D)].view(D, F + D)
    assert torch.equal(W[:, :F], wdr[:, :F])
    assert _rel(W[:, F:], wc64) <= TOL
    assert _rel(wfold[D * (F + D):D * (F + D) + D], d(wdr)[:, F:] @ d(br1) + d(bdr)) <= TOL
    assert torch.equal(wfold[D * (F + D) + D:].view(F + D, D), W.T)
    assert _rel(s, s64) <= TOL and _rel(u, u64) <= TOL and _rel(h0, h64) <= TOL

    dh0 = f(N, D)
    dt, ds, dr = (torch.empty(N, D, device=DEV) for _ in range(3))
    _lib.call("gine_chain_bwd_folded", P(dh0), P(u), P(wp2), P(wr0), P(wfold), P(dt), P(ds),
              P(dr), N, D, F, st)
    fl = ctypes.c_size_t(0)
    _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(fl))
    slab = torch.empty(fl.value, device=DEV)
    gfold = torch.empty(D * (F + D) + D, device=DEV)
    g = [torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, F + D), 5.0, device=DEV), torch.empty(D, device=DEV)]
    _lib.call("gine_chain_wgrad_folded", P(dh0), P(x), P(r), P(s), P(u), P(dt), P(ds), P(slab),
              P(gfold), P(g[2]), P(g[3]), P(g[0]), P(g[1]), 7.0, N, D, F, st)
    _lib.call("gine_chain_unfold_grads", P(gfold), P(wr1), P(br1), P(wdr), P(g[6]), P(g[7]),
              P(g[4]), P(g[5]), D, F, st)
    torch.cuda.synchronize()
    de64 = d(dh0) @ d(wdr)[:, F:]
    dt64 = (de64 @ d(wr1)) * (u > 0).double()
    ds64 = dt64 @ d(wr0)
    dr64 = ds64 @ d(wp2)
    assert _rel(dt, dt64) <= TOL, "dt"
    assert _rel(ds, ds64) <= TOL, "ds"
    assert _rel(dr, dr64) <= TOL, "dr"
    e_in = d(u) @ d(wr1).T + d(br1)  # e of the saved u
    xe = torch.cat([d(x), e_in], 1)
    assert _rel(gfold[:D * (F + D)].view(D, F + D), d(dh0).T @ torch.cat([d(x), d(u)], 1)) <= TOL
    for name, got, ref in (("dWp2", g[0], ds64.T @ d(r)), ("dbp2", g[1], 7.0 * ds64.sum(0)),
                           ("dWr0", g[2], dt64.T @ d(s)), ("dbr0", g[3], dt64.sum(0)),
                           ("dWr1", g[4], de64.T @ d(u)), ("dbr1", g[5], de64.sum(0)),
                           ("dWdr", g[6], d(dh0).T @ xe), ("dbdr", g[7], d(dh0).sum(0))):
        assert _rel(got, ref) <= TOL, (name, _rel(got, ref))


@pytest.mark.parametrize("N,D,F", [(2000, 128, 35), (33, 64, 20), (16000, 128, 64)])
def test_chain_one_launch_forward_matches_two_launch(N, D, F):
    """The folded forward in one launch (W' folded by the DeepSet launch,
    gine_deepset_fwd_fold + gine_chain_fwd_folded3) equals the two-launch form bit for bit,
    forward and backward."""
    from raincast_gnn import deepset
    torch.manual_seed(N + D)
    M, Fe = 11, 36
    ens = torch.randn(N, M, Fe, device=DEV)
    lin1 = torch.nn.Linear(Fe, D).to(DEV)
    lins = _lins(D, F, N)
    x = torch.randn(N, F, device=DEV)
    outs = []
    for one in (False, True):
        for m in lins + (lin1,):
            m.zero_grad(set_to_none=True)
        if one:
            r, wfold = deepset.phi_sum(ens, lin1, fold=(lins[2], lins[3]))
            h0 = fused_chain.chain(r, x, lins, M, wfold=wfold)
        else:
            r = deepset.phi_sum(ens, lin1)
            h0 = fused_chain.chain(r, x, lins, M)
        h0.backward(torch.ones_like(h0))
        outs.append([h0.detach()] + [p.grad.clone() for m in lins + (lin1,)
                                     for p in (m.weight, m.bias)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _ens_lin1(N, D, M=11, Fe=36, seed=0):
    torch.manual_seed(seed)
    return torch.randn(N, M, Fe, device=DEV), torch.nn.Linear(Fe, D).to(DEV)


@pytest.mark.parametrize("N,D,F", [(33, 128, 35), (300, 64, 35), (2000, 128, 64),
                                   (16000, 128, 35), (40000, 128, 35)])
def test_chain_folded2_intermediates(N, D, F):
    """The doubly folded chain's pieces (C ABI) against fp64 torch: [Wf | bf] from the
    DeepSet launch (whose r and [W' | b' | W'^T] equal the single fold's bit for bit), u / h0
    forward, dt / dr backward, G and G2 from the engine and all eight weight gradients
    unfolded from them.  References use the engine's u for the ReLU mask."""
    import ctypes

    from raincast_gnn import _lib, deepset
    M = 11
    ens, lin1 = _ens_lin1(N, D, M, seed=N + D)
    lins = _lins(D, F, N + 1)
    p2, r0, r1, dr_ = lins
    x = torch.randn(N, F, device=DEV)
    with torch.no_grad():
        r, wfold = deepset.phi_sum(ens, lin1, fold=(r1, dr_, r0, p2))
        r_1, wfold_1 = deepset.phi_sum(ens, lin1, fold=(r1, dr_))
    n1 = 2 * D * (F + D) + D
    assert wfold.numel() == n1 + D * D + D
    assert torch.equal(r, r_1) and torch.equal(wfold[:n1], wfold_1)
    d = lambda t: t.detach().double()  # noqa: E731
    wp2, bp2, wr0, br0 = d(p2.weight), d(p2.bias), d(r0.weight), d(r0.bias)
    wr1, br1, wdr, bdr = d(r1.weight), d(r1.bias), d(dr_.weight), d(dr_.bias)
    assert _rel(wfold[n1:n1 + D * D].view(D, D), wr0 @ wp2) <= TOL
    assert _rel(wfold[n1 + D * D:], M * (wr0 @ bp2) + br0) <= TOL

    P = _lib.ptr
    st = _lib.stream_handle(DEV)
    u, h0 = (torch.empty(N, D, device=DEV) for _ in range(2))
    wf1, wf2 = wfold[:n1], wfold[n1:]
    _lib.call("gine_chain_fwd_folded2", P(r), P(x), P(wf1), P(wf2), P(u), P(h0), N, D, F, st)
    s64 = d(r) @ wp2.T + M * bp2
    u64 = torch.relu(s64 @ wr0.T + br0)
    h64 = torch.cat([d(x), d(u) @ wr1.T + br1], 1) @ wdr.T + bdr
    torch.cuda.synchronize()
    assert _rel(u, u64) <= TOL and _rel(h0, h64) <= TOL

    dh0 = torch.randn(N, D, device=DEV)
    dt, dr = (torch.empty(N, D, device=DEV) for _ in range(2))
    _lib.call("gine_chain_bwd_folded2", P(dh0), P(u), P(wf1), P(wf2), P(dt), P(dr), N, D, F, st)
    fl = ctypes.c_size_t(0)
    _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(fl))
    slab = torch.empty(fl.value, device=DEV)
    gfold = torch.empty(D * (F + D) + D, device=DEV)
    g2fold = torch.empty(D * D + D, device=DEV)
    g = [torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, D), 5.0, device=DEV), torch.empty(D, device=DEV),
         torch.full((D, F + D), 5.0, device=DEV), torch.empty(D, device=DEV)]
    _lib.call("gine_chain_wgrad_folded2", P(dh0), P(x), P(r), P(u), P(dt), P(slab), P(gfold),
              P(g2fold), N, D, F, st)
    wr1_, br1_, wdr_ = (t.detach().contiguous() for t in (r1.weight, r1.bias, dr_.weight))
    wp2_, bp2_, wr0_ = (t.detach().contiguous() for t in (p2.weight, p2.bias, r0.weight))
    _lib.call("gine_chain_unfold_grads2", P(gfold), P(wr1_), P(br1_), P(wdr_), P(g[6]),
              P(g[7]), P(g[4]), P(g[5]), P(g2fold), P(wp2_), P(bp2_), P(wr0_), P(g[2]), P(g[3]),
              P(g[0]), P(g[1]), float(M), D, F, st)
    torch.cuda.synchronize()
    de64 = d(dh0) @ wdr[:, F:]
    dt64 = (de64 @ wr1) * (u > 0).double()
    ds64 = dt64 @ wr0
    assert _rel(dt, dt64) <= TOL, "dt"
    assert _rel(dr, ds64 @ wp2) <= TOL, "dr"
    assert _rel(g2fold[:D * D].view(D, D), dt64.T @ d(r)) <= TOL, "G2"
    assert _rel(g2fold[D * D:], dt64.sum(0)) <= TOL, "g2"
    xe = torch.cat([d(x), d(u) @ wr1.T + br1], 1)
    for name, got, ref in (("dWp2", g[0], ds64.T @ d(r)), ("dbp2", g[1], M * ds64.sum(0)),
                           ("dWr0", g[2], dt64.T @ s64), ("dbr0", g[3], dt64.sum(0)),
                           ("dWr1", g[4], de64.T @ d(u)), ("dbr1", g[5], de64.sum(0)),
                           ("dWdr", g[6], d(dh0).T @ xe), ("dbdr", g[7], d(dh0).sum(0))):
        assert _rel(got, ref) <= TOL, (name, _rel(got, ref))


@pytest.mark.parametrize("N,D,F", [(2000, 128, 35), (33, 64, 20), (4000, 128, 64)])
def test_chain_folded2_module_path(N, D, F):
    """chain() on the doubly folded buffer (the models.py path) against the single fold
    within TOL (only the rounding of Wf / bf differs; sizes small enough that no ReLU
    decision of rho[0] sits inside that rounding -- the model parity tests hold the full
    sizes to the branch oracle) and bit-identical when repeated; the deferred-gradient form
    (flat buffer) is covered by the model tests."""
    from raincast_gnn import deepset
    M = 11
    ens, lin1 = _ens_lin1(N, D, M, seed=N)
    lins = _lins(D, F, N)
    x = torch.randn(N, F, device=DEV)
    outs = []
    for fold in ((lins[2], lins[3]), (lins[2], lins[3], lins[1], lins[0]),
                 (lins[2], lins[3], lins[1], lins[0])):
        for m in lins + (lin1,):
            m.zero_grad(set_to_none=True)
        r, wfold = deepset.phi_sum(ens, lin1, fold=fold)
        h0 = fused_chain.chain(r, x, lins, M, wfold=wfold)
        assert type(h0.grad_fn).__name__.startswith(
            "_ChainFolded2Fn" if len(fold) == 4 else "_ChainFoldedFn")
        h0.backward(torch.ones_like(h0))
        outs.append([h0.detach()] + [p.grad.clone() for m in lins + (lin1,)
                                     for p in (m.weight, m.bias)])
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b)
    names = ["h0"] + [f"{m}.{p}" for m in ("p2", "r0", "r1", "dr", "phi0") for p in ("w", "b")]
    for name, a, b in zip(names, outs[0], outs[1]):
        assert _rel(b, a) <= 2 * TOL, (name, _rel(b, a))
