"""Fused DeepSet phi head: ``sum_m relu(phi[0](ens[:, m]))`` on one HIP kernel pair.

models/gnn.py:48-68 evaluates ``phi = Sequential(Linear(F, H), ReLU(), Linear(H, H))`` on
every (station, member) row and sums over members.  :class:`~raincast_gnn.models.
DeepSetEncoder` moves the member sum before ``phi[2]`` (a Linear commutes with a sum); what
remains, ``r = sum_m relu(ens W1^T + b1)``, is the ``[N, M, H]`` activation the reference
materialises three times per training step (90 MB each at the 24h_mixed benchmark shape).
``gine_deepset_fwd`` keeps it in MFMA accumulators and writes only ``r [N, H]``;
the forward also records its ReLU pattern as bits (2.8 MB instead of 90 MB), from which
``gine_deepset_bwd`` produces dW1/db1 directly (csrc/gine_deepset.hip).  The ensemble tensor is data (never requires grad in the
reference); a caller that needs d/d(ens) gets the unfused torch path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import gradbuf
from .gradbuf import grad_out

HIDDEN = (32, 64, 128, 256)
MAX_FEATURES = 64


def fusable(ens: torch.Tensor, weight: torch.Tensor, bias) -> bool:
    return (ens.is_cuda and ens.dim() == 3 and ens.dtype == torch.float32
            and weight.dtype == torch.float32 and bias is not None
            and weight.size(0) in HIDDEN and 0 < weight.size(1) <= MAX_FEATURES
            and ens.size(2) == weight.size(1) and ens.size(1) > 0
            and not ens.requires_grad)


class _PhiSumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ens, weight, bias, fold=None):
        """``fold`` = (rho[2] weight, rho[2] bias, dim_red weight, dim_red bias): the same
        launch also folds the dense chain's dim_red weight (gine_deepset_fwd_fold) and the
        function returns (r, wfold), wfold not differentiable."""
        ens = ens.contiguous()
        weight, bias = weight.contiguous(), bias.contiguous()
        N, M, Fdim = ens.shape
        H = weight.size(0)
        r = torch.empty(N, H, dtype=torch.float32, device=ens.device)
        mask = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            nbytes = ctypes.c_size_t(0)
            _lib.call("gine_deepset_mask_bytes", N, M, H, ctypes.byref(nbytes))
            mask = torch.empty(nbytes.value, dtype=torch.uint8, device=ens.device)
        ctx.save_for_backward(ens, mask)
        ctx.params = (weight, bias)
        ctx.hidden = H
        stream = _lib.stream_handle(ens.device)
        if fold is None:
            _lib.call("gine_deepset_fwd", _lib.ptr(ens), _lib.ptr(weight), _lib.ptr(bias),
                      _lib.ptr(r), _lib.ptr(mask), N, M, Fdim, H, stream)
            return r
        wr1, br1, wdr, bdr, *more = (t.detach().contiguous() for t in fold)
        F = wdr.size(1) - H
        n1 = 2 * H * (F + H) + H
        P = _lib.ptr
        if not more:
            wfold = torch.empty(n1, dtype=torch.float32, device=ens.device)
            _lib.call("gine_deepset_fwd_fold", P(ens), P(weight), P(bias), P(r), P(mask), N, M,
                      Fdim, H, P(wr1), P(br1), P(wdr), P(bdr), P(wfold), F, stream)
        else:  # the double fold: [W' | b' | W'^T] then [Wf | bf] in one buffer
            wr0, br0, wp2, bp2 = more
            wfold = torch.empty(n1 + H * H + H, dtype=torch.float32, device=ens.device)
            _lib.call("gine_deepset_fwd_fold2", P(ens), P(weight), P(bias), P(r), P(mask), N, M,
                      Fdim, H, P(wr1), P(br1), P(wdr), P(bdr), P(wfold), F, P(wr0), P(br0),
                      P(wp2), P(bp2), P(wfold[n1:]), stream)
        ctx.mark_non_differentiable(wfold)
        # no zero-filled gradient for wfold in the backward (a fill launch per step)
        ctx.set_materialize_grads(False)
        return r, wfold

    @staticmethod
    def backward(ctx, dr, *unused):
        ens, mask = ctx.saved_tensors
        if dr is None:  # (grads are not materialised in the folding form)
            return None, None, None, None
        N, M, Fdim = ens.shape
        H = ctx.hidden
        dr = dr.contiguous()
        parts = ctypes.c_int32(0)
        _lib.call("gine_deepset_bwd_num_partials", N, H, ctypes.byref(parts))
        slab = torch.empty(parts.value * (H * Fdim + H), dtype=torch.float32, device=dr.device)
        dw = grad_out(ctx.params[0], (H, Fdim), dr.device)
        db = grad_out(ctx.params[1], (H,), dr.device)
        defer = gradbuf.deferrable(dw, db)  # slab reduced in the end-of-backward batch
        _lib.call("gine_deepset_bwd", _lib.ptr(ens), _lib.ptr(mask), _lib.ptr(dr),
                  _lib.ptr(slab), None if defer else _lib.ptr(dw),
                  None if defer else _lib.ptr(db), N, M, Fdim, H,
                  _lib.stream_handle(dr.device))
        if defer:
            job = _lib.GradJob()
            _lib.call("gine_deepset_bwd_grad_job", N, Fdim, H, _lib.ptr(slab), _lib.ptr(dw),
                      _lib.ptr(db), ctypes.byref(job))
            gradbuf.defer(job, dr.device, (slab,))
        return None, dw, db, None


def phi_sum(ens: torch.Tensor, lin1: torch.nn.Linear, fold=None):
    """``relu(lin1(ens)).sum(dim=1)`` for ens [N, M, F] on the fused kernels; with
    ``fold`` = (rho[2], dim_red) Linears, (r, wfold) for the one-launch folded chain; with
    ``fold`` = (rho[2], dim_red, rho[0], phi[2]), (r, wfold) for the doubly folded chain
    (wfold then also holds [Wf | bf], gine_deepset_fwd_fold2)."""
    if fold is None:
        return _PhiSumFn.apply(ens, lin1.weight, lin1.bias)
    return _PhiSumFn.apply(ens, lin1.weight, lin1.bias,
                           tuple(t for m in fold for t in (m.weight, m.bias)))
