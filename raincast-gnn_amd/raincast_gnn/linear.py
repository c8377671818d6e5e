"""``Linear`` whose weight gradient runs on the split-row HIP kernel.

Same module, parameters and state_dict keys as ``torch.nn.Linear`` (models/gnn.py uses
nn.Linear for the DeepSet phi/rho, dim_red and aggr layers).  Forward and the input
gradient stay on the library GEMM (well shaped: many rows, small weight); the weight and
bias gradients -- contractions over 16,000-176,000 rows into a tiny [O x I] output, which
library GEMMs tile into a handful of workgroups -- use ``gine_linear_wgrad``
(csrc/gine_linear.hip).  CPU tensors take the stock torch path.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _lib
from .gradbuf import grad_out


class _RowLinearFn(torch.autograd.Function):
    """y = x W^T + bias_scale * b."""

    @staticmethod
    def forward(ctx, x, weight, bias, bias_scale=1.0):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.params = (weight, bias)
        ctx.bias_scale = float(bias_scale)
        if bias is None or bias_scale == 1.0:
            return F.linear(x, weight, bias)
        x2 = x.reshape(-1, x.size(-1))
        y = torch.addmm(bias, x2, weight.t(), beta=bias_scale)
        return y.reshape(*x.shape[:-1], weight.size(0))

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        O, I = weight.shape
        dx = dy @ weight if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dy2 = dy.reshape(-1, O).contiguous()
            x2 = x.reshape(-1, I).contiguous()
            R = dy2.size(0)
            chunks = ctypes.c_int32(0)
            _lib.call("gine_linear_wgrad_num_chunks", R, O, I, ctypes.byref(chunks))
            slab = torch.empty(chunks.value * (O * I + O), dtype=torch.float32, device=dy.device)
            dw = grad_out(ctx.params[0], (O, I), dy.device)
            db = grad_out(ctx.params[1], (O,), dy.device) if ctx.has_bias else None
            _lib.call("gine_linear_wgrad", _lib.ptr(dy2), _lib.ptr(x2), R, O, I, _lib.ptr(slab),
                      _lib.ptr(dw), _lib.ptr(db), ctx.bias_scale, _lib.stream_handle(dy.device))
        return dx, dw, db, None


class Linear(torch.nn.Linear):
    def forward(self, x: torch.Tensor, bias_scale: float = 1.0) -> torch.Tensor:
        """``x W^T + bias_scale * b`` (bias_scale=1: torch.nn.Linear)."""
        if (x.is_cuda and x.dtype == torch.float32 and self.weight.dtype == torch.float32
                and torch.is_grad_enabled()):
            return _RowLinearFn.apply(x, self.weight, self.bias, bias_scale)
        if bias_scale == 1.0 or self.bias is None:
            return F.linear(x, self.weight, self.bias)
        return F.linear(x, self.weight) + bias_scale * self.bias
