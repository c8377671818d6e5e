"""Flat-buffer AdamW for the benchmarked training step (train.py:67-69).

The reference steps ``torch.optim.AdamW(model.parameters(), lr=params["lr"])`` (train.py:185)
over ~40 small parameter tensors (209,800 fp32 values for 24h_mixed): on a GPU that is a
few hundred tiny launches per step.  :class:`FlatAdamW` re-points every parameter at a view
of ONE contiguous buffer (and every ``.grad`` at a view of one contiguous gradient buffer --
the same buffer the data-parallel all-reduce uses), then updates all of them with one HIP
kernel (``gine_adamw_step``, include/gine_hip.h) that reproduces torch's AdamW arithmetic.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, gradbuf


class FlatAdamW:
    ALIGN = 64  # floats: parameter offsets in the flat buffers

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        _lib.require_device(self.params[0], "FlatAdamW")
        if any(p.dtype != torch.float32 or p.device != dev for p in self.params):
            raise TypeError("FlatAdamW needs fp32 parameters on one device")
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), betas, float(eps), \
            float(weight_decay)
        # every parameter starts on a 256-byte boundary (the kernels' weight fragment loads
        # use 16-byte vectors when a weight is aligned); the gaps stay zero in all four flat
        # buffers, which AdamW leaves at zero
        self._offsets = []
        off = 0
        for p in self.params:
            self._offsets.append(off)
            off = -(-(off + p.numel()) // self.ALIGN) * self.ALIGN
        n = off
        self.flat_param = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(n, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, off in zip(self.params, self._offsets):
                k = p.numel()
                view = self.flat_param[off:off + k].view_as(p)
                view.copy_(p)
                p.data = view
                gradbuf.register(p, self.flat_grad, off)
        self.exp_avg = torch.zeros_like(self.flat_param)
        self.exp_avg_sq = torch.zeros_like(self.flat_param)
        # [count, ticket, -, 8 sub-tickets at 32 + 32 g]: gine_adamw_step bumps the count in
        # its last workgroup (two-level ticket, include/gine_hip.h)
        floats = ctypes.c_int64(0)
        _lib.call("gine_adamw_state_floats", ctypes.byref(floats))
        self._step_state = torch.zeros(int(floats.value), dtype=torch.float32, device=dev)
        self.step_count = self._step_state[:1]

    @property
    def numel(self) -> int:
        return self.flat_param.numel()

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Release the gradients.  The HIP backward kernels then write each parameter's
        gradient straight into its slice of ``flat_grad`` (raincast_gnn/gradbuf.py);
        ``set_to_none=False`` instead keeps ``.grad`` as slice views and zeroes them
        (gradients are then accumulated by autograd, one add per parameter)."""
        if set_to_none:
            for p in self.params:
                p.grad = None
            gradbuf.new_step(self.params)
        else:
            for p, off in zip(self.params, self._offsets):
                if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:].data_ptr():
                    p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            self.flat_grad.zero_()

    @torch.no_grad()
    def gather_grads(self) -> None:
        """Make ``flat_grad`` hold every gradient: parameters whose ``.grad`` is not their
        slice (a CPU-side or generic-torch backward produced it) are copied in, unused ones
        zeroed.  Host-side pointer checks only when everything already landed in place."""
        base = self.flat_grad.data_ptr()
        for p, off in zip(self.params, self._offsets):
            g = p.grad
            if g is not None and g.data_ptr() == base + 4 * off:
                continue
            sl = self.flat_grad[off:off + p.numel()]
            if g is None:
                sl.zero_()
            else:
                sl.copy_(g.reshape(-1))
            p.grad = sl.view_as(p)

    @torch.no_grad()
    def step(self) -> None:
        self.gather_grads()
        b1, b2 = self.betas
        _lib.call("gine_adamw_step", _lib.ptr(self.flat_param), _lib.ptr(self.flat_grad),
                  _lib.ptr(self.exp_avg), _lib.ptr(self.exp_avg_sq), _lib.ptr(self._step_state),
                  self.numel, self.lr, float(b1), float(b2), self.eps, self.weight_decay,
                  _lib.stream_handle(self.flat_param.device))

    def views_intact(self) -> bool:
        """True while every parameter and gradient still aliases the flat buffers."""
        pb, gb = self.flat_param.data_ptr(), self.flat_grad.data_ptr()
        end_p, end_g = pb + 4 * self.numel, gb + 4 * self.numel
        return all(pb <= p.data_ptr() < end_p and p.grad is not None
                   and gb <= p.grad.data_ptr() < end_g for p in self.params)
