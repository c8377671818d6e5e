"""Fused dense layers between the DeepSet member sum and the GINE stack.

models/gnn.py:132-135 computes ``dim_red(cat([x, DeepSetEncoder(ensemble)], 1))``; after the
fused member sum ``r = sum_m relu(phi[0](ens_m))`` (:mod:`.deepset`) what remains is four
dense Linears and a ReLU on [N, D] rows::

    s = phi[2](r) (bias x M)  ->  u = relu(rho[0](s))  ->  e = rho[2](u)  ->  h0 = dim_red([x | e])

By default the chain runs FOLDED (``gine_chain_fwd_folded``): rho[2] and dim_red have no
nonlinearity between them, so ``h0 = [x | u] W'^T + b'`` with ``W' = [Wdr_x | Wdr_e Wr1]``
folded from the current weights inside the first kernel; the backward needs one
input-gradient GEMM and one weight-gradient product fewer, and dWr1 / dWdr_e are unfolded
from ``G = dh0^T u`` after the slab reduction (profiles/r02_s38_chain_fold_ab_*: cfg2
0.575 -> 0.560 ms per step, cfg3 3.26 -> 2.97).  ``FOLD = False`` runs the unfolded
chain: ``gine_chain_fwd`` as two 2-stage row-chain kernels and ``gine_chain_bwd`` (two chain
kernels, one weight-gradient launch for all four Linears, one reduction) -- csrc/
gine_chain.hip.  Modules, parameters and state_dict keys are the reference's; this is only
the execution of ``GNN.forward``'s first half.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, gradbuf
from .gradbuf import grad_out

HIDDEN = (64, 128)
MAX_FEATURES = 64


def fusable(r: torch.Tensor, x: torch.Tensor, lins) -> bool:
    return r.is_cuda and r.dtype == torch.float32 and fusable_dims(r.size(1), x, lins)


def fusable_dims(D: int, x: torch.Tensor, lins) -> bool:
    """The chain's conditions on everything but r (r [N, D] fp32 on the device)."""
    p2, r0, r1, dr = lins
    F = x.size(1)
    shapes = ((p2, D, D), (r0, D, D), (r1, D, D), (dr, F + D, D))
    return (x.is_cuda and x.dtype == torch.float32
            and D in HIDDEN and 0 < F <= MAX_FEATURES and not x.requires_grad
            and all(isinstance(m, torch.nn.Linear) and m.bias is not None
                    and m.weight.dtype == torch.float32 and m.in_features == i
                    and m.out_features == o for m, i, o in shapes))


class _ChainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r, x, wp2, bp2, wr0, br0, wr1, br1, wdr, bdr, members):
        r = r.contiguous()
        x = x.contiguous()
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        ws = [t.detach().contiguous() for t in (wp2, bp2, wr0, br0, wr1, br1, wdr, bdr)]
        s, u, e, h0 = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(4))
        P = _lib.ptr
        _lib.call("gine_chain_fwd", P(r), P(x), P(ws[0]), P(ws[1]), float(members), P(ws[2]),
                  P(ws[3]), P(ws[4]), P(ws[5]), P(ws[6]), P(ws[7]), P(s), P(u), P(e), P(h0),
                  N, D, F, _lib.stream_handle(dev))
        ctx.save_for_backward(r, x, s, u, e, ws[0], ws[2], ws[4], ws[6])
        ctx.params = (wp2, bp2, wr0, br0, wr1, br1, wdr, bdr)
        ctx.members = float(members)
        return h0

    @staticmethod
    def backward(ctx, dh0):
        r, x, s, u, e, wp2, wr0, wr1, wdr = ctx.saved_tensors
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        dh0 = dh0.contiguous()
        de, dt, ds, dr = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(4))
        floats = ctypes.c_size_t(0)
        _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(floats))
        slab = torch.empty(floats.value, dtype=torch.float32, device=dev)
        p = ctx.params
        g = [grad_out(p[0], (D, D), dev), grad_out(p[1], (D,), dev),
             grad_out(p[2], (D, D), dev), grad_out(p[3], (D,), dev),
             grad_out(p[4], (D, D), dev), grad_out(p[5], (D,), dev),
             grad_out(p[6], (D, F + D), dev), grad_out(p[7], (D,), dev)]
        P = _lib.ptr
        # input gradients (de, dt, ds -> dr) on the current stream: the DeepSet backward
        # needs dr next ...
        _lib.call("gine_chain_bwd", P(dh0), P(x), P(r), P(s), P(u), P(e), P(wp2), P(wr0),
                  P(wr1), P(wdr), P(de), P(dt), P(ds), P(dr), None, None, None, ctx.members,
                  None, None, None, None, None, None, N, D, F, _lib.stream_handle(dev))
        members = ctx.members
        if gradbuf.deferrable(*g):
            # the engine leaves its slab; the end-of-backward batch reduces it
            _lib.call("gine_chain_wgrad", P(dh0), P(x), P(r), P(s), P(u), P(e), P(de),
                      P(dt), P(ds), P(slab), None, None, members, None, None, None, None,
                      None, None, N, D, F, _lib.stream_handle(dev))
            job = _lib.GradJob()
            _lib.call("gine_chain_wgrad_grad_job", N, D, F, P(slab), members, P(g[0]),
                      P(g[1]), P(g[2]), P(g[3]), P(g[4]), P(g[5]), P(g[6]), P(g[7]),
                      ctypes.byref(job))
            gradbuf.defer(job, dev, (slab,))
            return (dr, None, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], None)
        # ... else the four weight gradients reduced in the same call
        _lib.call("gine_chain_wgrad", P(dh0), P(x), P(r), P(s), P(u), P(e), P(de), P(dt),
                  P(ds), P(slab), P(g[0]), P(g[1]), members, P(g[2]), P(g[3]), P(g[4]),
                  P(g[5]), P(g[6]), P(g[7]), N, D, F, _lib.stream_handle(dev))
        return (dr, None, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], None)


class _ChainFoldedFn(torch.autograd.Function):
    """The folded chain (gine_chain_fwd_folded, include/gine_hip.h): rho[2] and dim_red have
    no nonlinearity between them, so ``h0 = [x | u] W'^T + b'`` with ``W' = [Wdr_x | Wdr_e
    Wr1]`` -- the embedding ``e`` and its gradient are never formed, and dWr1 / dWdr_e come
    from the one product ``G = dh0^T u``.  Same parameters and gradients as :class:`_ChainFn`
    (the rounding of sums differs, within the fp32 tolerance of the oracle tests)."""

    @staticmethod
    def forward(ctx, r, x, wp2, bp2, wr0, br0, wr1, br1, wdr, bdr, members, wfold=None):
        r = r.contiguous()
        x = x.contiguous()
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        ws = [t.detach().contiguous() for t in (wp2, bp2, wr0, br0, wr1, br1, wdr, bdr)]
        s, u, h0 = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(3))
        P = _lib.ptr
        if wfold is not None:  # folded by the DeepSet launch: the whole forward in one launch
            _lib.call("gine_chain_fwd_folded3", P(r), P(x), P(ws[0]), P(ws[1]), float(members),
                      P(ws[2]), P(ws[3]), P(wfold), P(s), P(u), P(h0), N, D, F,
                      _lib.stream_handle(dev))
        else:
            wfold = torch.empty(2 * D * (F + D) + D, dtype=torch.float32, device=dev)
            _lib.call("gine_chain_fwd_folded", P(r), P(x), P(ws[0]), P(ws[1]), float(members),
                      P(ws[2]), P(ws[3]), P(ws[4]), P(ws[5]), P(ws[6]), P(ws[7]), P(wfold),
                      P(s), P(u), P(h0), N, D, F, _lib.stream_handle(dev))
        ctx.save_for_backward(r, x, s, u, wfold, ws[0], ws[2], ws[4], ws[5], ws[6])
        ctx.params = (wp2, bp2, wr0, br0, wr1, br1, wdr, bdr)
        ctx.members = float(members)
        return h0

    @staticmethod
    def backward(ctx, dh0):
        r, x, s, u, wfold, wp2, wr0, wr1, br1, wdr = ctx.saved_tensors
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        dh0 = dh0.contiguous()
        dt, ds, dr = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(3))
        floats = ctypes.c_size_t(0)
        _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(floats))
        slab = torch.empty(floats.value, dtype=torch.float32, device=dev)
        gfold = torch.empty(D * (F + D) + D, dtype=torch.float32, device=dev)
        p = ctx.params
        g = [grad_out(p[0], (D, D), dev), grad_out(p[1], (D,), dev),
             grad_out(p[2], (D, D), dev), grad_out(p[3], (D,), dev),
             grad_out(p[4], (D, D), dev), grad_out(p[5], (D,), dev),
             grad_out(p[6], (D, F + D), dev), grad_out(p[7], (D,), dev)]
        P = _lib.ptr
        stream = _lib.stream_handle(dev)
        _lib.call("gine_chain_bwd_folded", P(dh0), P(u), P(wp2), P(wr0), P(wfold), P(dt), P(ds),
                  P(dr), N, D, F, stream)
        members = ctx.members

        # raw pointers only: a reference to a gradient tensor held past this function would
        # stop autograd adopting it as param.grad (it copies a shared tensor)
        ptrs = (P(gfold), P(wr1), P(br1), P(wdr), P(g[6]), P(g[7]), P(g[4]), P(g[5]))

        def unfold(st):
            _lib.call("gine_chain_unfold_grads", *ptrs, D, F, st)

        if gradbuf.deferrable(*g):
            # the engine leaves its slab; the end-of-backward batch reduces it into
            # G | dWr0 | dWp2, then unfolds G into dWdr / dWr1
            _lib.call("gine_chain_wgrad_folded", P(dh0), P(x), P(r), P(s), P(u), P(dt), P(ds),
                      P(slab), None, None, None, None, None, members, N, D, F, stream)
            job = _lib.GradJob()
            _lib.call("gine_chain_wgrad_folded_grad_job", N, D, F, P(slab), members, P(gfold),
                      P(g[2]), P(g[3]), P(g[0]), P(g[1]), ctypes.byref(job))
            gradbuf.defer(job, dev, (slab, gfold, wr1, br1, wdr), post=unfold)
        else:
            _lib.call("gine_chain_wgrad_folded", P(dh0), P(x), P(r), P(s), P(u), P(dt), P(ds),
                      P(slab), P(gfold), P(g[2]), P(g[3]), P(g[0]), P(g[1]), members, N, D, F,
                      stream)
            unfold(stream)
        return (dr, None, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], None, None)


class _ChainFolded2Fn(torch.autograd.Function):
    """The doubly folded chain (gine_chain_fwd_folded2, include/gine_hip.h): phi[2] meets
    rho[0] with only the member sum between them, so ``rho[0](s) = r Wf^T + bf`` with
    ``Wf = Wr0 Wp2``, ``bf = M Wr0 bp2 + br0`` (folded by the DeepSet launch into the tail
    of ``wfold``).  Neither s nor its gradient is formed: one 2-stage launch forward
    (u, h0), one backward (dt, dr), two weight-gradient products (G = dh0^T [x | u],
    G2 = dt^T r) unfolded into all six chain gradients by one launch."""

    @staticmethod
    def forward(ctx, r, x, wp2, bp2, wr0, br0, wr1, br1, wdr, bdr, members, wfold):
        r = r.contiguous()
        x = x.contiguous()
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        n1 = 2 * D * (F + D) + D
        wf1, wf2 = wfold[:n1], wfold[n1:]
        u, h0 = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(2))
        P = _lib.ptr
        _lib.call("gine_chain_fwd_folded2", P(r), P(x), P(wf1), P(wf2), P(u), P(h0), N, D, F,
                  _lib.stream_handle(dev))
        ws = [t.detach().contiguous() for t in (wp2, bp2, wr0, wr1, br1, wdr)]
        ctx.save_for_backward(r, x, u, wfold, *ws)
        ctx.params = (wp2, bp2, wr0, br0, wr1, br1, wdr, bdr)
        ctx.members = float(members)
        return h0

    @staticmethod
    def backward(ctx, dh0):
        r, x, u, wfold, wp2, bp2, wr0, wr1, br1, wdr = ctx.saved_tensors
        N, D = r.shape
        F = x.size(1)
        dev = r.device
        n1 = 2 * D * (F + D) + D
        wf1, wf2 = wfold[:n1], wfold[n1:]
        dh0 = dh0.contiguous()
        dt, dr = (torch.empty(N, D, dtype=torch.float32, device=dev) for _ in range(2))
        floats = ctypes.c_size_t(0)
        _lib.call("gine_chain_bwd_slab_floats", N, D, F, ctypes.byref(floats))
        slab = torch.empty(floats.value, dtype=torch.float32, device=dev)
        gf = torch.empty(D * (F + D) + D + D * D + D, dtype=torch.float32, device=dev)
        gfold, g2fold = gf[:D * (F + D) + D], gf[D * (F + D) + D:]
        p = ctx.params
        g = [grad_out(p[0], (D, D), dev), grad_out(p[1], (D,), dev),
             grad_out(p[2], (D, D), dev), grad_out(p[3], (D,), dev),
             grad_out(p[4], (D, D), dev), grad_out(p[5], (D,), dev),
             grad_out(p[6], (D, F + D), dev), grad_out(p[7], (D,), dev)]
        P = _lib.ptr
        stream = _lib.stream_handle(dev)
        _lib.call("gine_chain_bwd_folded2", P(dh0), P(u), P(wf1), P(wf2), P(dt), P(dr), N, D, F,
                  stream)
        # raw pointers only (see _ChainFoldedFn.backward)
        ptrs = (P(gfold), P(wr1), P(br1), P(wdr), P(g[6]), P(g[7]), P(g[4]), P(g[5]),
                P(g2fold), P(wp2), P(bp2), P(wr0), P(g[2]), P(g[3]), P(g[0]), P(g[1]),
                ctx.members)

        def unfold(st):
            _lib.call("gine_chain_unfold_grads2", *ptrs, D, F, st)

        if gradbuf.deferrable(*g):
            _lib.call("gine_chain_wgrad_folded2", P(dh0), P(x), P(r), P(u), P(dt), P(slab), None,
                      None, N, D, F, stream)
            job = _lib.GradJob()
            _lib.call("gine_chain_wgrad_folded2_grad_job", N, D, F, P(slab), P(gfold),
                      P(g2fold), ctypes.byref(job))
            gradbuf.defer(job, dev, (slab, gf, wp2, bp2, wr0, wr1, br1, wdr), post=unfold)
        else:
            _lib.call("gine_chain_wgrad_folded2", P(dh0), P(x), P(r), P(u), P(dt), P(slab),
                      P(gfold), P(g2fold), N, D, F, stream)
            unfold(stream)
        return (dr, None, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], None, None)


# False: the unfolded chain (four GEMM stages forward, e materialised); measured slower
# (cfg2 0.5749 vs 0.5595 ms per step, r02_s38), kept for the tests that compare the two
FOLD = True


# False: the folded forward as two launches (W' folded by the first).  The one-launch form (three stages, one workgroup per CU) wins while a CU walks a few tiles
# (cfg2, 16,000 nodes: 0.5442 -> 0.5405 ms per step) and loses at many (cfg3, 128,000:
# 2.922 -> 2.937, profiles/r02_s67_*), so it is used up to F3_MAX_NODES rows.
F3 = True
F3_MAX_NODES = 32768

# True: on the one-launch path (F3) phi[2] is folded into rho[0] as well (_ChainFolded2Fn),
# at every size: its forward has two stages, not three, and wins at cfg3 (128,000 nodes:
# 2.749 -> 2.665 ms per step) and cfg5 (80,000: 1.715 -> 1.622) too, where the singly folded
# one-launch form lost (F3_MAX_NODES; profiles/r04_s18_chain_fold2_large.txt)
FOLD2 = True


def chain(r: torch.Tensor, x: torch.Tensor, lins, members: int, wfold=None) -> torch.Tensor:
    """``dim_red(cat([x, rho(phi[2](r) summed over members)]))`` on the fused kernels;
    ``wfold`` = the folded dim_red weight from gine_deepset_fwd_fold (folded chain only; with
    [Wf | bf] appended by gine_deepset_fwd_fold2, the doubly folded chain)."""
    p2, r0, r1, dr = lins
    D = r.size(1)
    if FOLD and wfold is not None and wfold.numel() > 2 * D * (x.size(1) + D) + D:
        return _ChainFolded2Fn.apply(r, x, p2.weight, p2.bias, r0.weight, r0.bias, r1.weight,
                                     r1.bias, dr.weight, dr.bias, members, wfold)
    if FOLD:
        return _ChainFoldedFn.apply(r, x, p2.weight, p2.bias, r0.weight, r0.bias, r1.weight,
                                    r1.bias, dr.weight, dr.bias, members, wfold)
    return _ChainFn.apply(r, x, p2.weight, p2.bias, r0.weight, r0.bias, r1.weight, r1.bias,
                          dr.weight, dr.bias, members)
