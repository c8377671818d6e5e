"""Fused output head: ``PostProcess(aggr(h))`` on one HIP kernel each way.

models/gnn.py:140-141 evaluates ``self.postprocess(self.aggr(h))`` -- a Linear(D, K) and
the per-column transforms of models/model_utils.py:70-113 (softplus + 1e-6 on the scales,
sigmoid on the point mass, 2.12 * sigmoid on a learned threshold).  ``gine_head_fwd`` /
``gine_head_bwd`` (csrc/gine_head.hip) run both, forward and backward, in one row-streaming
kernel each; the module structure and parameters (``GNN.aggr``, ``GNN.postprocess``) are
unchanged.
"""
from __future__ import annotations

import ctypes

import torch

from torch.utils.weak import WeakIdKeyDictionary

from . import _lib
from . import gradbuf
from .gradbuf import grad_out

MAX_CHANNELS = 256


class HeadRecord:
    """What the CRPS pass needs to run this head's backward ahead of time (loss.py,
    gine_crps_head_fwd_grad): the head's input, weight and pre-PostProcess output.  ``pre``
    = (grad_unit, dh, slab) once it has: the backward then uses dh / slab if its incoming
    gradient is that very grad_unit tensor (a unit-seeded loss.backward()).  ``y`` /
    ``count_parts``: the batch targets the forward was given and their non-NaN partial
    counts (gine_head_fwd_count), which the loss uses when it is called with that ``y``."""

    __slots__ = ("h", "w", "raw", "kind", "params", "pre", "y", "y_version", "count_parts")

    def __init__(self, h, w, raw, kind, params):
        self.h, self.w, self.raw, self.kind, self.params = h, w, raw, kind, params
        self.pre = None
        self.y = self.y_version = self.count_parts = None

    def counts_for(self, y: torch.Tensor):
        """The partial counts of ``y`` if this forward counted exactly that tensor, as it
        is now (same object, no in-place change since), else None."""
        if self.y is y and y._version == self.y_version:
            return self.count_parts
        return None


_records = WeakIdKeyDictionary()  # pred tensor -> HeadRecord


def record_of(pred: torch.Tensor) -> HeadRecord | None:
    """The HeadRecord of a prediction returned by :func:`head` (None for any other tensor)."""
    return _records.get(pred)


def loss_kind(loss: str, grad_u) -> int | None:
    """GINE_LOSS_* of PostProcess(loss, grad_u) (its ``== "True"`` string test, gnn.py:98)."""
    if loss == "NormalCRPS":
        return _lib.LOSS_NORMAL
    if loss == "MixedNormalCRPS":
        return _lib.LOSS_MIXED_NORMAL
    if loss == "MixedLoss":
        return _lib.LOSS_MIXED_U if grad_u == "True" else _lib.LOSS_MIXED
    return None


K_OF = {_lib.LOSS_NORMAL: 2, _lib.LOSS_MIXED_NORMAL: 3, _lib.LOSS_MIXED: 4, _lib.LOSS_MIXED_U: 5}


def fusable(h: torch.Tensor, lin: torch.nn.Linear, kind) -> bool:
    return (kind is not None and h.is_cuda and h.dim() == 2 and h.dtype == torch.float32
            and lin.weight.dtype == torch.float32 and lin.bias is not None
            and lin.out_features == K_OF[kind] and lin.in_features == h.size(1)
            and h.size(1) % 4 == 0 and h.size(1) <= MAX_CHANNELS)


def _counts_y(y, N: int, dev) -> bool:
    """The targets can be counted beside the head (gine_head_fwd_count / gine_layer_head)."""
    return (y is not None and y.is_cuda and y.device == dev and y.dtype == torch.float32
            and y.is_contiguous() and y.numel() == N)


class HeadPlan:
    """The head forward folded into the last GINE layer's launch (gine_layer_head,
    csrc/gine_mpmlp.hip): the outputs are allocated here, handed to that launch
    (functional.GineLayer) and taken by :func:`head` when its input is exactly the tensor
    that launch wrote (``done`` = its data pointer); otherwise the head runs its own launch."""

    __slots__ = ("params", "versions", "w", "b", "kind", "y", "raw", "pred", "parts", "done")

    def __init__(self, N: int, D: int, lin: torch.nn.Linear, kind: int, y, dev):
        self.params = (lin.weight, lin.bias)
        self.versions = (lin.weight._version, lin.bias._version)
        self.w, self.b = lin.weight.detach().contiguous(), lin.bias.detach().contiguous()
        self.kind = kind
        K = self.w.size(0)
        self.raw = torch.empty(N, K, dtype=torch.float32, device=dev)
        self.pred = torch.empty(N, K, dtype=torch.float32, device=dev)
        self.y = y if _counts_y(y, N, dev) else None
        self.parts = (torch.empty(_lib.COUNT_PARTS, dtype=torch.int32, device=dev)
                      if self.y is not None else None)
        self.done = None

    def args(self, N: int, D: int, dev):
        """The gine_layer_head of a launch writing [N, D] rows on ``dev``, or None."""
        if self.raw.size(0) != N or self.w.size(1) != D or self.raw.device != dev:
            return None
        return _lib.LayerHead(_lib.ptr(self.w), _lib.ptr(self.b), _lib.ptr(self.raw),
                              _lib.ptr(self.pred), _lib.ptr(self.y), _lib.ptr(self.parts),
                              self.kind)

    def take(self, h: torch.Tensor, weight, bias, kind: int, y):
        """(raw, pred, parts | None) when the launch that wrote ``h`` also ran this head (the
        same parameters, unchanged since, and kind), else None; one use."""
        done, self.done = self.done, None
        if (done is None or done != (h.data_ptr(), tuple(h.shape)) or kind != self.kind
                or self.params[0] is not weight or self.params[1] is not bias
                or self.versions != (weight._version, bias._version)):
            return None
        return self.raw, self.pred, (self.parts if y is self.y else None)


def plan(h: torch.Tensor, lin: torch.nn.Linear, kind: int, y=None) -> HeadPlan:
    """A HeadPlan for the head that follows the GINE stack whose input is ``h``."""
    return HeadPlan(h.size(0), h.size(1), lin, kind, y, h.device)


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias, kind, y=None, hplan=None):
        h = h.contiguous()
        w, b = weight.detach().contiguous(), bias.detach().contiguous()
        N, D = h.shape
        K = w.size(0)
        done = hplan.take(h, weight, bias, kind, y) if hplan is not None else None
        if done is not None:  # computed by the last layer's launch
            raw, pred, parts = done
        else:
            raw = torch.empty(N, K, dtype=torch.float32, device=h.device)
            pred = torch.empty(N, K, dtype=torch.float32, device=h.device)
        rec = HeadRecord(h, w, raw, kind, (weight, bias))
        if done is not None:
            if parts is not None:
                rec.y, rec.y_version, rec.count_parts = y, y._version, parts
        elif _counts_y(y, N, h.device):
            # the loss's valid-target count, computed beside the head (no launch of its own)
            parts = torch.empty(_lib.COUNT_PARTS, dtype=torch.int32, device=h.device)
            _lib.call("gine_head_fwd_count", _lib.ptr(h), _lib.ptr(w), _lib.ptr(b),
                      _lib.ptr(raw), _lib.ptr(pred), N, D, kind, _lib.ptr(y), _lib.ptr(parts),
                      _lib.stream_handle(h.device))
            rec.y, rec.y_version, rec.count_parts = y, y._version, parts
        else:
            _lib.call("gine_head_fwd", _lib.ptr(h), _lib.ptr(w), _lib.ptr(b), _lib.ptr(raw),
                      _lib.ptr(pred), N, D, kind, _lib.stream_handle(h.device))
        ctx.save_for_backward(h, w, raw)
        ctx.kind = kind
        ctx.params = (weight, bias)
        ctx.rec = rec
        _records[pred] = ctx.rec
        return pred

    @staticmethod
    def backward(ctx, gpred):
        h, w, raw = ctx.saved_tensors
        N, D = h.shape
        K = w.size(0)
        dev = h.device
        pre, ctx.rec.pre = ctx.rec.pre, None
        if pre is not None and gpred is pre[0]:  # run by the CRPS pass (unit seed)
            _, dh, slab = pre
            dw = grad_out(ctx.params[0], (K, D), dev)
            db = grad_out(ctx.params[1], (K,), dev)
            job = _lib.GradJob()
            _lib.call("gine_crps_head_grad_job", N, D, ctx.kind, _lib.ptr(slab), _lib.ptr(dw),
                      _lib.ptr(db), ctypes.byref(job))
            if gradbuf.deferrable(dw, db):
                gradbuf.defer(job, dev, (slab,))
            else:
                arr = (_lib.GradJob * 1)(job)
                _lib.call("gine_grad_finalize_batch", arr, 1, _lib.stream_handle(dev))
            return dh, dw, db, None, None, None
        gpred = gpred.float().contiguous()
        floats = ctypes.c_size_t(0)
        _lib.call("gine_head_bwd_slab_floats", N, D, ctx.kind, ctypes.byref(floats))
        slab = torch.empty(floats.value, dtype=torch.float32, device=dev)
        dh = torch.empty_like(h)
        dw = grad_out(ctx.params[0], (K, D), dev)
        db = grad_out(ctx.params[1], (K,), dev)
        defer = gradbuf.deferrable(dw, db)  # slab reduced in the end-of-backward batch
        _lib.call("gine_head_bwd", _lib.ptr(gpred), _lib.ptr(raw), _lib.ptr(h), _lib.ptr(w),
                  _lib.ptr(dh), _lib.ptr(slab), None if defer else _lib.ptr(dw),
                  None if defer else _lib.ptr(db), N, D, ctx.kind, _lib.stream_handle(dev))
        if defer:
            job = _lib.GradJob()
            _lib.call("gine_head_bwd_grad_job", N, D, ctx.kind, _lib.ptr(slab), _lib.ptr(dw),
                      _lib.ptr(db), ctypes.byref(job))
            gradbuf.defer(job, dev, (slab,))
        return dh, dw, db, None, None, None


def head(h: torch.Tensor, lin: torch.nn.Linear, kind: int, y: torch.Tensor | None = None,
         hplan: HeadPlan | None = None) -> torch.Tensor:
    """``PostProcess(lin(h))`` for the loss ``kind`` on the fused kernels.  ``y``: the
    batch targets, whose non-NaN count the launch also takes for the loss that follows.
    ``hplan``: the plan handed to the GINE stack (:func:`plan`); when its last layer's launch
    ran the head on exactly ``h``, its outputs are used and no launch is made here."""
    return _HeadFn.apply(h, lin.weight, lin.bias, kind, y, hplan)
