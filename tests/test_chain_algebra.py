"""The algebra the folded dense chain (csrc/gine_chain.hip, gine_chain_*_folded) relies on,
checked in fp64 on the CPU against autograd of the reference composition
(models/gnn.py:60-68, 112-113, 132-135: phi[2] -> rho[0] -> ReLU -> rho[2] -> dim_red):

  h0 = [x | u Wr1^T + br1] Wdr^T + bdr = [x | u] W'^T + b',  W' = [Wdr_x | Wdr_e Wr1],
  b' = Wdr_e br1 + bdr;  with G = dh0^T u, g = sum_n dh0:
  dWdr = [dh0^T x | G Wr1^T + g br1^T], dWr1 = Wdr_e^T G, dbr1 = Wdr_e^T g,
  dt = (dh0 Wdr_e Wr1) * 1[u > 0]."""
import torch


def test_folded_chain_identities():
    g = torch.Generator().manual_seed(0)
    N, D, F = 257, 16, 5
    d = dict(dtype=torch.float64)
    r = torch.randn(N, D, generator=g, **d)
    x = torch.randn(N, F, generator=g, **d)
    Wp2, Wr0, Wr1 = (torch.randn(D, D, generator=g, **d) / 4 for _ in range(3))
    Wdr = torch.randn(D, F + D, generator=g, **d) / 4
    bp2, br0, br1, bdr = (torch.randn(D, generator=g, **d) for _ in range(4))
    params = [t.requires_grad_() for t in (Wp2, bp2, Wr0, br0, Wr1, br1, Wdr, bdr)]
    M = 3.0
    s = r @ Wp2.T + M * bp2
    u = torch.relu(s @ Wr0.T + br0)
    e = u @ Wr1.T + br1
    h0 = torch.cat([x, e], 1) @ Wdr.T + bdr
    dh0 = torch.randn(N, D, generator=g, **d)
    grads = torch.autograd.grad(h0, params + [u], dh0)
    dWr1, dbr1, dWdr, dbdr = grads[4], grads[5], grads[6], grads[7]
    with torch.no_grad():
        Wdr_x, Wdr_e = Wdr[:, :F], Wdr[:, F:]
        Wc = Wdr_e @ Wr1
        Wf = torch.cat([Wdr_x, Wc], 1)
        bf = Wdr_e @ br1 + bdr
        assert torch.allclose(torch.cat([x, u], 1) @ Wf.T + bf, h0, rtol=1e-12, atol=1e-12)
        G = dh0.T @ u
        gs = dh0.sum(0)
        assert torch.allclose(torch.cat([dh0.T @ x, G @ Wr1.T + torch.outer(gs, br1)], 1), dWdr,
                              rtol=1e-12, atol=1e-12)
        assert torch.allclose(gs, dbdr, rtol=1e-12, atol=1e-12)
        assert torch.allclose(Wdr_e.T @ G, dWr1, rtol=1e-12, atol=1e-12)
        assert torch.allclose(Wdr_e.T @ gs, dbr1, rtol=1e-12, atol=1e-12)
        # the input gradient of u (before the ReLU mask) is dh0 Wc
        assert torch.allclose(dh0 @ Wc, grads[8], rtol=1e-12, atol=1e-12)


def test_double_folded_chain_identities():
    """phi[2] folded into rho[0] too (gine_chain_*_folded2):  pre = r Wf^T + bf with
    Wf = Wr0 Wp2, bf = M Wr0 bp2 + br0;  with dt the gradient of pre, G2 = dt^T r and
    g2 = sum_n dt:  dWr0 = G2 Wp2^T + M g2 bp2^T, dbr0 = g2, dWp2 = Wr0^T G2,
    dbp2 = M Wr0^T g2, dr = dt Wf."""
    g = torch.Generator().manual_seed(1)
    N, D, M = 301, 16, 7.0
    d = dict(dtype=torch.float64)
    r = torch.randn(N, D, generator=g, **d).requires_grad_()
    Wp2, Wr0 = (torch.randn(D, D, generator=g, **d) / 4 for _ in range(2))
    bp2, br0 = (torch.randn(D, generator=g, **d) for _ in range(2))
    params = [t.requires_grad_() for t in (Wp2, bp2, Wr0, br0)]
    pre = (r @ Wp2.T + M * bp2) @ Wr0.T + br0
    dt = torch.randn(N, D, generator=g, **d)
    dWp2, dbp2, dWr0, dbr0, dr = torch.autograd.grad(pre, params + [r], dt)
    with torch.no_grad():
        Wf = Wr0 @ Wp2
        bf = M * (Wr0 @ bp2) + br0
        kw = dict(rtol=1e-12, atol=1e-12)
        assert torch.allclose(r @ Wf.T + bf, pre, **kw)
        G2, g2 = dt.T @ r, dt.sum(0)
        assert torch.allclose(G2 @ Wp2.T + M * torch.outer(g2, bp2), dWr0, **kw)
        assert torch.allclose(g2, dbr0, **kw)
        assert torch.allclose(Wr0.T @ G2, dWp2, **kw)
        assert torch.allclose(M * (Wr0.T @ g2), dbp2, **kw)
        assert torch.allclose(dt @ Wf, dr, **kw)
