"""Independent backward work on a side HIP stream.

A few launches of the backward produce only parameter gradients that nothing reads until
the optimizer (the dense chain's weight gradients, the message-passing dW_e/db_e/eps
finish, the head's weight reduction).  :func:`launch` runs such work on a per-device side
stream that first waits for everything already queued on the current stream, so it
executes beside the main chain of the backward (under HIP-graph capture it becomes a
parallel branch of the graph), and joins it back into the current stream when the
backward pass ends (``queue_callback``; immediately when called outside a backward).
The tensors the side work touches are kept alive until that join, so the caching
allocator cannot hand their memory to later main-stream work early.

Gradient OUTPUTS written on the side stream must not be read by autograd on the main
stream: that holds when autograd adopts them as ``param.grad`` (the parameter had no
gradient yet -- no kernel runs), so callers pass ``params`` and the work runs inline when
any of them already holds a gradient (autograd would then add into it on the main
stream).  The outputs themselves are not kept alive here: a second reference would make
autograd copy instead of adopt.  A parameter that receives a SECOND gradient contribution
later in the same backward (shared weights) would be summed by autograd on the main
stream while the side work may still write the first one; no model of this package shares
parameters between these layers.

Off by default (``RAINCAST_SIDE_STREAMS=1`` enables it): measured on MI355X, a fork/join
pair in a replayed HIP graph costs more than the overlap wins at the 24h_mixed shape
(chain weight gradients beside the DeepSet backward: 0.700 ms/step vs 0.673 inline).
"""
from __future__ import annotations

import os
import threading

import torch

ENABLED = os.environ.get("RAINCAST_SIDE_STREAMS", "0") == "1"

_lock = threading.Lock()
_streams: dict[int, torch.cuda.Stream] = {}


def side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _lock:
        s = _streams.get(idx)
        if s is None:
            s = torch.cuda.Stream(device=torch.device("cuda", idx))
            _streams[idx] = s
        return s


_unjoined: list = []  # (main, side) stream pairs with side work not yet joined


def wait_all() -> None:
    """Make every main stream wait for the side work queued from it (the end-of-backward
    gradient batch calls this before it reads slabs written on a side stream)."""
    with _lock:
        pairs = list(_unjoined)
        _unjoined.clear()
    for main, side in pairs:
        main.wait_stream(side)


def launch(device: torch.device, fn, keep_alive=(), params=()) -> None:
    """``fn(stream_handle)`` on the side stream of ``device``, ordered after the current
    stream's queued work and joined back into it at the end of the backward pass (inline
    on the current stream when a parameter in ``params`` already has a gradient)."""
    main = torch.cuda.current_stream(device)
    if not ENABLED or any(p is not None and p.grad is not None for p in params):
        fn(main.cuda_stream)
        return
    side = side_stream(device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        fn(side.cuda_stream)
    held = tuple(keep_alive)
    with _lock:
        _unjoined.append((main, side))

    def join():
        main.wait_stream(side)
        del held_ref[:]

    held_ref = [held]
    try:
        torch.autograd.Variable._execution_engine.queue_callback(join)
    except RuntimeError:  # not inside a backward pass
        join()
