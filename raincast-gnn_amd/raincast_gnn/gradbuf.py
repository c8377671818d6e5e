"""Parameter-gradient outputs that land directly in a flat gradient buffer.

When an optimizer keeps every gradient in one flat buffer (:class:`~raincast_gnn.optim.
FlatAdamW`, whose buffer is also the data-parallel all-reduce payload), the HIP backward
kernels can write each parameter gradient straight into that parameter's slice: the
backward returns a FRESH view of the slice, and autograd's AccumulateGrad, seeing
``param.grad is None`` and no other reference to the tensor, adopts it as ``param.grad``
without a copy.  That removes one gradient-copy launch per parameter per step.

A slice is handed out at most once per step (a second contribution to the same parameter
gets an ordinary tensor and is summed by autograd as usual); the optimizer verifies before
using the buffer that every ``param.grad`` really is its slice and copies it in otherwise.
"""
from __future__ import annotations

import torch
from torch.utils.weak import WeakIdKeyDictionary  # identity keys (Tensor.__eq__ is elementwise)

_slots = WeakIdKeyDictionary()   # param -> (flat buffer, offset)
_issued = WeakIdKeyDictionary()  # params whose slice was handed out this step


def register(param: torch.Tensor, flat: torch.Tensor, offset: int) -> None:
    _slots[param] = (flat, offset)


def slice_of(param: torch.Tensor):
    slot = _slots.get(param)
    if slot is None:
        return None
    flat, off = slot
    return flat[off:off + param.numel()].view(param.shape)


def new_step(params) -> None:
    for p in params:
        _issued.pop(p, None)


def grad_out(param: torch.Tensor | None, shape=None, device=None) -> torch.Tensor:
    """Output tensor for d(loss)/d(param): its flat-buffer slice when that is safe to
    hand to autograd, a new tensor otherwise."""
    if param is not None and param.grad is None and param not in _issued:
        view = slice_of(param)
        if view is not None:
            _issued[param] = True
            return view if shape is None else view.view(shape)
    shp = param.shape if shape is None else shape
    dev = param.device if device is None else device
    return torch.empty(shp, dtype=torch.float32, device=dev)
