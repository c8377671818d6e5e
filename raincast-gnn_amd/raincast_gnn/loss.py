"""CRPS losses of the reference (models/loss.py), restated for device execution.

On a HIP device the reduced loss runs as ONE fused kernel pass (``gine_crps_fwd`` /
``gine_crps_bwd``, csrc/gine_loss.hip: closed form + exact per-node gradient by fp64
forward-mode duals, NaN-masked mean).  The torch formulation below is kept for CPU tensors
and ``reduce=False``; both are pinned to the reference's own outputs (tests/golden/).

Same closed forms, same dtype promotions (the censoring point ``c = log(0.01)`` is a float64
tensor, so every term that touches it -- and the loss -- is float64, loss.py:33-34,
230-231), same NaN semantics: rows whose target is NaN do not contribute.  The reference
drops them with boolean indexing (``mu[mask]``, loss.py:39-42, 234-239), which needs a
device->host sync for the result shape; here NaN targets are replaced by 0 before the
closed form and the mean is taken over the valid rows with a masked sum, so a training
step contains no host sync and can be captured in a HIP graph.  The masked rows get exactly
zero gradient, as in the reference.  ``torch.distributions.Normal`` (which validates its
arguments with a host sync) is replaced by its own cdf/log_prob formulas for loc 0, scale 1.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib, gradbuf
from . import head as _head

_LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
# NormalCRPS keeps 1/sqrt(pi) as an fp32 tensor (loss.py:343): same value as a Python float
_INV_SQRT_PI_F32 = float(1 / torch.sqrt(torch.tensor(np.pi)))


def _cdf(v: torch.Tensor) -> torch.Tensor:
    # Normal(0, 1).cdf: 0.5 * (1 + erf((v - loc) * scale.reciprocal() / sqrt(2)))
    return 0.5 * (1 + torch.erf(v / math.sqrt(2)))


def _pdf(v: torch.Tensor) -> torch.Tensor:
    # Normal(0, 1).log_prob(v).exp(): -(v - loc)**2 / (2 var) - log(scale) - log(sqrt(2 pi))
    return torch.exp(-(v ** 2) / 2 - _LOG_SQRT_2PI)


class _Consts:
    """Per-device 1-element constant tensors, created once (a host->device copy inside a
    captured step would be illegal), with the reference's dtypes: ``torch.tensor([c])`` of
    a Python/NumPy float gives float64 for np.float64 and float32 for a plain float."""

    def __init__(self):
        self._cache = {}

    def get(self, value, device) -> torch.Tensor:
        key = (repr(value), type(value).__name__, str(device))
        t = self._cache.get(key)
        if t is None:
            t = torch.tensor([value], device=device)
            self._cache[key] = t
        return t


_consts = _Consts()

_tickets: dict = {}


def _ticket(device) -> torch.Tensor:
    """Per-device uint32 work counter of gine_crps_fwd's last-workgroup finish (zeroed once;
    every launch leaves it at 0 again)."""
    key = str(device)
    t = _tickets.get(key)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=device)
        _tickets[key] = t
    return t


def _finish(crps: torch.Tensor, mask: torch.Tensor, reduce: bool) -> torch.Tensor:
    if not reduce:  # reference shape: only the rows with a target, [M, 1]
        return crps[mask]
    return _masked_mean(crps, mask)


def _masked_mean(values: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    m = mask.reshape(values.shape)
    total = torch.where(m, values, torch.zeros_like(values)).sum()
    return total / m.sum().to(values.dtype)


def _valid_count(y: torch.Tensor, rec=None, y_orig=None) -> torch.Tensor:
    """Number of non-NaN targets of ``y`` as GINE_COUNT_PARTS device partial counts: the
    ones the fused head forward took beside its launch when it was given this very ``y``
    (models.GNN.forward passes ``data.y``), else one gine_count_valid launch.  Counted on
    every step -- inside a captured step too, so a replay whose ``y`` was refilled in place
    (``static_y.copy_(new)``) divides by the count of the new targets.  ``y_orig``: the
    tensor the caller passed (``y`` may be its fp32 contiguous copy)."""
    parts = rec.counts_for(y if y_orig is None else y_orig) if rec is not None else None
    if parts is not None:
        return parts
    parts = torch.empty(_lib.COUNT_PARTS, dtype=torch.int32, device=y.device)
    _lib.call("gine_count_valid", _lib.ptr(y), y.numel(), _lib.ptr(parts),
              _lib.stream_handle(y.device))
    return parts


# The head backward of a unit-seeded loss runs inside the CRPS pass (gine_crps_head_fwd_grad;
# otherwise gine_head_bwd, its own launch).  The CRPS pass that runs it takes 64 nodes per workgroup: one round of workgroups up to
# HEAD_BWD_MAX_NODES nodes (cfg2, 16,000: one launch fewer), several rounds of the fp64 loss
# chain above (cfg3 / cfg5 lose), so it is used up to that size.
HEAD_BWD = True
HEAD_BWD_MAX_NODES = 32768


class _FusedCRPS(torch.autograd.Function):
    """Reduced CRPS of ``pred [N, K]`` vs ``y [N]`` in one HIP pass (fp64 result).  When the
    prediction needs a gradient, the pass also writes d loss / d pred for a unit seed
    (gine_crps_fwd_grad): ``loss.backward()`` seeded with the cached 1 of
    gradbuf.loss_backward then costs no launch (any other seed: gine_crps_bwd).  ``rec``: the
    HeadRecord of the fused head that produced ``pred``; the pass then also runs that head's
    backward for the unit seed (gine_crps_head_fwd_grad), which the head's backward picks up
    when it receives exactly this grad_unit tensor."""

    @staticmethod
    def forward(ctx, pred, y, kind, u, xi, c, t, rec=None, count_rec=None):
        needs = ctx.needs_input_grad[0]
        pred = pred.detach().float().contiguous()
        y_in = y
        y = y.detach().float().contiguous()
        N, K = pred.shape
        dev = pred.device
        n_part = ctypes.c_int32(0)
        _lib.call("gine_crps_num_partials", N, ctypes.byref(n_part))
        dpred = torch.empty(N, K, dtype=torch.float64, device=dev)
        partials = torch.empty(n_part.value, 2, dtype=torch.float64, device=dev)
        loss = torch.empty((), dtype=torch.float64, device=dev)
        count = torch.empty(1, dtype=torch.float64, device=dev)
        ctx.grad_unit = None
        if needs and N > 0:
            count_in = _valid_count(y, count_rec, y_in)
            ctx.grad_unit = torch.empty(N, K, dtype=torch.float32, device=dev)
            if rec is not None:
                D = rec.h.size(1)
                floats = ctypes.c_size_t(0)
                _lib.call("gine_crps_head_slab_floats", N, D, kind, ctypes.byref(floats))
                slab = torch.empty(floats.value, dtype=torch.float32, device=dev)
                dh = torch.empty_like(rec.h)
                _lib.call("gine_crps_head_fwd_grad", _lib.ptr(pred), _lib.ptr(y), N, kind, u, xi,
                          c, t, _lib.ptr(dpred), _lib.ptr(partials), _lib.ptr(loss),
                          _lib.ptr(count), _lib.ptr(_ticket(dev)), _lib.ptr(count_in),
                          _lib.ptr(ctx.grad_unit), _lib.ptr(rec.raw), _lib.ptr(rec.h),
                          _lib.ptr(rec.w), D, _lib.ptr(dh), _lib.ptr(slab),
                          _lib.stream_handle(dev))
                rec.pre = (ctx.grad_unit, dh, slab)
            else:
                _lib.call("gine_crps_fwd_grad", _lib.ptr(pred), _lib.ptr(y), N, kind, u, xi, c,
                          t, _lib.ptr(dpred), _lib.ptr(partials), _lib.ptr(loss),
                          _lib.ptr(count), _lib.ptr(_ticket(dev)), _lib.ptr(count_in),
                          _lib.ptr(ctx.grad_unit), _lib.stream_handle(dev))
        else:
            _lib.call("gine_crps_fwd", _lib.ptr(pred), _lib.ptr(y), N, kind, u, xi, c, t,
                      _lib.ptr(dpred), _lib.ptr(partials), _lib.ptr(loss), _lib.ptr(count),
                      _lib.ptr(_ticket(dev)), _lib.stream_handle(dev))
        ctx.save_for_backward(dpred, count)
        ctx.kind = kind
        return loss

    @staticmethod
    def backward(ctx, gloss):
        if ctx.grad_unit is not None and gradbuf.is_unit_seed(gloss):
            return ctx.grad_unit, None, None, None, None, None, None, None, None
        dpred, count = ctx.saved_tensors
        N = dpred.size(0)
        g = gloss.detach().to(torch.float64).reshape(1).contiguous()
        grad = torch.empty(dpred.shape, dtype=torch.float32, device=dpred.device)
        _lib.call("gine_crps_bwd", _lib.ptr(dpred), _lib.ptr(count), _lib.ptr(g), N, ctx.kind,
                  _lib.ptr(grad), _lib.stream_handle(dpred.device))
        return grad, None, None, None, None, None, None, None, None


def _fused(prediction, y, kind, u=0.0, xi=0.5, c=float(np.log(0.01)), t=5.0):
    if prediction.dim() != 2:
        raise ValueError("prediction must be [N, K]")
    count_rec = _head.record_of(prediction)
    rec = count_rec if HEAD_BWD else None
    if rec is not None and (rec.kind != kind or rec.raw.shape != prediction.shape
                            or not prediction.requires_grad
                            or prediction.size(0) > HEAD_BWD_MAX_NODES):
        rec = None
    return _FusedCRPS.apply(prediction, y, kind, float(u), float(xi), float(c), float(t), rec,
                            count_rec)


def _use_fused(prediction: torch.Tensor, reduce: bool = True, fused: bool = True) -> bool:
    return fused and reduce and prediction.is_cuda


def _prepare(prediction: torch.Tensor, y: torch.Tensor, width: int):
    mask = ~torch.isnan(y)
    cols = torch.split(prediction, 1, dim=1)
    if len(cols) != width:
        raise ValueError(f"prediction must have {width} columns, got {prediction.size(1)}")
    y_safe = torch.where(mask, y, torch.zeros_like(y)).unsqueeze(1)
    return mask, cols, y_safe


class NormalCRPS(torch.nn.Module):
    """models/loss.py:335-369.  ``fused`` (every loss class): False keeps the torch
    formulation on a HIP device too (the drop-in model, raincast_gnn/dropin.py)."""

    fused = True

    def crps(self, prediction: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        # the reference's NormalCRPS stays fp32 (loss.py:358-369)
        if _use_fused(prediction, True, self.fused):
            return _fused(prediction, y, _lib.LOSS_NORMAL).to(torch.float32)
        mask, (mu, sigma), y1 = _prepare(prediction, y, 2)
        z = (y1 - mu) / sigma
        crps = sigma * (z * (2.0 * _cdf(z) - 1.0) + 2.0 * _pdf(z) - _INV_SQRT_PI_F32)
        return _finish(crps, mask, True)


class MixedNormalCRPS(torch.nn.Module):
    """Censored normal with a point mass p at c, models/loss.py:6-68."""

    fused = True

    def __init__(self, reduce: bool = True, c: float = np.log(0.01)):
        super().__init__()
        self.reduce = reduce
        self.c = c

    def crps(self, prediction: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if _use_fused(prediction, self.reduce, self.fused):
            return _fused(prediction, y, _lib.LOSS_MIXED_NORMAL, c=float(self.c))
        mask, (mu, sigma, p), y1 = _prepare(prediction, y, 3)
        c = _consts.get(self.c, y.device)  # float64: np.float64 is a float
        y_t = (y1 - mu) / sigma
        c_t = (c - mu) / sigma
        P_c = p + (1 - p) * _cdf(c_t)
        t1 = y_t * (2 * (p + (1 - p) * _cdf(y_t)) - 1)
        t2 = -c_t * torch.pow(P_c, 2)
        t3 = 2 * (1 - p) * (-_pdf(c_t)) * P_c
        t4 = -2 * (1 - p) * (-_pdf(y_t))
        t5 = (2 * torch.pow(1 - p, 2) * (-1 / (2 * math.sqrt(math.pi)))
              * (1 - _cdf(math.sqrt(2) * c_t)))
        crps = sigma * (t1 + t2 + t3 + t4 + t5)
        return _finish(crps, mask, self.reduce)


class MixedLoss(torch.nn.Module):
    """Censored normal body + generalised Pareto tail above u, models/loss.py:71-272."""

    fused = True

    def __init__(self, grad_u: bool, xi: float, u=None, reduce: bool = True, t: float = 5,
                 c=np.log(0.01)):
        super().__init__()
        self.reduce, self.c, self.grad_u, self.u, self.xi, self.t = reduce, c, grad_u, u, xi, t

    @staticmethod
    def _gpd(x_re, xi):
        return torch.where(x_re <= 0, 0, 1 - (1 + xi * x_re).pow(-1 / xi))

    @staticmethod
    def _delta_u(u_t, p):
        return p + (1 - p) * _cdf(u_t)

    def _pareto_crps(self, y, u, m, sigma, xi):
        y_t = (y - u) / sigma
        cdf = self._gpd(y_t, xi)
        return sigma * (torch.abs(y_t) - 2 * (1 - m) / (1 - xi) * (1 - torch.pow(1 - cdf, 1 - xi))
                        + torch.pow(1 - m, 2) / (2 - xi))

    @staticmethod
    def _body(p, c_t, u_t):
        P_c = p + (1 - p) * _cdf(c_t)
        P_u = (1 - p) * (1 - _cdf(u_t))
        t2 = -c_t * torch.pow(P_c, 2) + u_t * torch.pow(P_u, 2)
        t3 = 2 * (1 - p) * (-_pdf(c_t)) * P_c + 2 * (1 - p) * (-_pdf(u_t)) * P_u
        t5 = (2 * torch.pow(1 - p, 2) * (-1 / (2 * math.sqrt(math.pi)))
              * (_cdf(math.sqrt(2) * u_t) - _cdf(math.sqrt(2) * c_t)))
        return P_u, t2, t3, t5

    def _mixed_normal_crps(self, y_t, p, c_t, u_t, sigma):
        _, t2, t3, t5 = self._body(p, c_t, u_t)
        t1 = y_t * (2 * (p + (1 - p) * _cdf(y_t)) - 1)
        t4 = -2 * (1 - p) * (-_pdf(y_t))
        return sigma * (t1 + t2 + t3 + t4 + t5)

    def _mixed_normal_crps_upper(self, p, c_t, u_t, sigma):
        P_u, t2, t3, t5 = self._body(p, c_t, u_t)
        t4 = -2 * ((1 - p) * (-_pdf(u_t)) + u_t * P_u)
        return sigma * (u_t + t2 + t3 + t4 + t5)

    def crps(self, prediction: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if _use_fused(prediction, self.reduce, self.fused):
            # u / xi are fp32 tensors in the reference (torch.tensor([python float]))
            kind = _lib.LOSS_MIXED_U if self.grad_u else _lib.LOSS_MIXED
            u = 0.0 if self.grad_u else float(np.float32(self.u))
            return _fused(prediction, y, kind, u=u, xi=float(np.float32(self.xi)),
                          c=float(self.c), t=float(self.t))
        if self.grad_u == True:  # noqa: E712  (reference compares with == True, loss.py:227)
            mask, (mu, sigma, p, sigma_u, u), y1 = _prepare(prediction, y, 5)
        else:
            mask, (mu, sigma, p, sigma_u), y1 = _prepare(prediction, y, 4)
            u = _consts.get(self.u, y.device)
        c = _consts.get(self.c, y.device)
        xi = _consts.get(self.xi, y.device)
        c_t = (c - mu) / sigma
        u_t = (u - mu) / sigma
        y_t = (y1 - mu) / sigma
        m_u = self._delta_u(u_t, p)
        loss_1 = (self._mixed_normal_crps(y_t, p, c_t, u_t, sigma)
                  + self._pareto_crps(u, u, m_u, sigma_u, xi))
        loss_2 = (self._pareto_crps(y1, u, m_u, sigma_u, xi)
                  + self._mixed_normal_crps_upper(p, c_t, u_t, sigma))
        if self.grad_u:
            crps = torch.sigmoid((u - y1) * self.t) * (loss_1 - loss_2) + loss_2
        else:
            crps = torch.where(y1 < u, loss_1, loss_2)
        return _finish(crps, mask, self.reduce)
