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

import threading
import weakref

import torch
from torch.utils.weak import WeakIdKeyDictionary  # identity keys (Tensor.__eq__ is elementwise)

from . import _lib

_slots = WeakIdKeyDictionary()   # param -> (flat buffer, offset)
_issued = WeakIdKeyDictionary()  # params whose slice was handed out this step
_flats: list = []                # weak references to the registered flat buffers


def register(param: torch.Tensor, flat: torch.Tensor, offset: int) -> None:
    _slots[param] = (flat, offset)
    if not any(r() is flat for r in _flats):
        _flats.append(weakref.ref(flat))


def in_flat_buffer(t: torch.Tensor | None) -> bool:
    """True when ``t`` lies inside a registered flat gradient buffer."""
    if t is None:
        return False
    p = t.data_ptr()
    for r in _flats:
        f = r()
        if f is not None and f.data_ptr() <= p < f.data_ptr() + 4 * f.numel():
            return True
    return False


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


# ---------------------------------------------------------------------------------------
# Deferred gradient reductions (gine_grad_finalize_batch, include/gine_hip.h)
# ---------------------------------------------------------------------------------------
# Reductions whose outputs only the optimizer reads -- dW_e/db_e/eps of every GINE layer,
# the head / dense-chain / DeepSet weight-gradient slabs -- are collected during a backward
# pass and run as ONE launch when the pass ends (an autograd final callback, so
# ``param.grad`` is complete when ``backward()`` returns and before any accumulation).  Only
# outputs that are flat-buffer slices adopted as ``param.grad`` qualify: autograd then
# never reads them during the pass.  (BATCH_ENABLED = False: one finish launch per
# reduction, the form the tests compare the batch with.)

BATCH_ENABLED = True
_pending: list = []
_pending_lock = threading.Lock()


def deferrable(*outs) -> bool:
    """True when every gradient output is a flat-buffer slice and a backward pass is
    running (its end-of-pass callback will run the batch)."""
    if not BATCH_ENABLED or not outs:
        return False
    if not all(in_flat_buffer(t) for t in outs if t is not None):
        return False
    return torch._C._current_graph_task_id() != -1


def defer(job: "_lib.GradJob", device: torch.device, keep_alive=(), post=None) -> None:
    """Queue ``job`` (its buffers kept alive) for the end-of-backward batch launch.
    ``post(stream)``, if given, is called after the batch launches of that stream (work that
    reads the job's reduced outputs, e.g. gine_chain_unfold_grads)."""
    stream = _lib.stream_handle(device)
    with _pending_lock:
        first = not _pending
        _pending.append((job, stream, tuple(keep_alive), post))
    if first:
        torch.autograd.Variable._execution_engine.queue_callback(flush)


def flush() -> None:
    """Run every queued reduction (one launch per stream and per GRAD_MAX_JOBS jobs), then
    the queued post steps."""
    with _pending_lock:
        items = list(_pending)
        _pending.clear()
    by_stream: dict = {}
    for job, stream, keep, post in items:
        by_stream.setdefault(stream, ([], []))
        by_stream[stream][0].append(job)
        if post is not None:
            by_stream[stream][1].append(post)
    for stream, (jobs, posts) in by_stream.items():
        for i in range(0, len(jobs), _lib.GRAD_MAX_JOBS):
            part = jobs[i:i + _lib.GRAD_MAX_JOBS]
            arr = (_lib.GradJob * len(part))(*part)
            _lib.call("gine_grad_finalize_batch", arr, len(part), stream)
        for post in posts:
            post(stream)
    # the buffers in ``items`` are released here, after their consumers are enqueued


def mp_job(partials: torch.Tensor, rows: int, channels: int, eps_cols: int, dlw, dlb, deps):
    j = _lib.GradJob()
    j.kind = _lib.GRAD_JOB_MP
    j.src = partials.data_ptr()
    j.rows, j.channels, j.eps_cols = int(rows), int(channels), int(eps_cols)
    j.w[0], j.w[1], j.w[2] = dlw.data_ptr(), dlb.data_ptr(), deps.data_ptr()
    return j


_seeds: dict = {}  # (device, dtype) -> the constant 1 that seeds a scalar loss's backward


def loss_backward(loss: torch.Tensor) -> None:
    """``loss.backward()`` without its seed-fill launch: autograd uses a gradient tensor it
    is given as is, so d loss / d loss = 1 comes from a cached device scalar instead of a
    ``ones_like`` kernel per step (one launch fewer in the captured training step).  The
    scalar is created outside graph capture (the eager warm-up steps); inside a capture
    without one, the plain call runs."""
    key = (loss.device, loss.dtype)
    one = _seeds.get(key)
    if one is None:
        if loss.is_cuda and torch.cuda.is_current_stream_capturing():
            loss.backward()
            return
        one = _seeds[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
    loss.backward(one)


def is_unit_seed(g: torch.Tensor) -> bool:
    """True when ``g`` is the cached constant 1 that :func:`loss_backward` seeds with (the
    object autograd hands to the loss node unchanged)."""
    one = _seeds.get((g.device, g.dtype))
    return one is not None and g is one
