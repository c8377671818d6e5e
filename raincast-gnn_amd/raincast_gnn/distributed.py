"""Data parallelism over the GPUs of one node (absent in the reference: train.py:163 uses a
single device; the north star shards graph mini-batches over 8 MI355X).

Graphs of a batch are disjoint components (block-diagonal collation), so sharding whole
graphs across ranks needs no halo exchange; the only exchange is the gradient.  The model
holds ~0.2 M fp32 parameters (209,800 for 24h_mixed = 839 KB), far below what a ring needs to
become bandwidth-bound on xGMI, so the gradient lives in ONE flat buffer and is reduced with
ONE RCCL all-reduce per step (no bucketing, no per-parameter collectives).  BatchNorm keeps
per-rank batch statistics, like the reference's single-process BN over its own batch; the
running buffers are broadcast from rank 0 before they are read (validation, checkpoints:
raincast_gnn/train.py), which gives DistributedDataParallel's buffer semantics there.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


_SHARED_DEVICE = False


def device_shared() -> bool:
    """True when another rank of the process group uses this process's GPU as well (set by
    note_device_sharing).  Their kernels can then hold CUs whenever ours launch, so launches
    that need their whole grid resident at once (the one-launch layer forward's grid
    barrier: raincast_gnn.functional.layer_forward_ok) are not used."""
    return _SHARED_DEVICE


def note_device_sharing(group=None) -> bool:
    """Find out (collectively: every rank of ``group`` calls this) whether ranks share a
    device -- the same host and device index -- and remember it for device_shared()."""
    global _SHARED_DEVICE
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        _SHARED_DEVICE = False
        return False
    import socket
    me = (socket.gethostname(),
          torch.cuda.current_device() if torch.cuda.is_available() else -1)
    every = [None] * dist.get_world_size(group)
    dist.all_gather_object(every, me, group=group)
    _SHARED_DEVICE = me[1] >= 0 and every.count(me) > 1
    return _SHARED_DEVICE


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


class FlatGradReducer:
    """Makes every ``param.grad`` a view into one contiguous fp32 buffer.

    Autograd accumulates into existing ``.grad`` tensors in place, so after ``backward`` the
    whole gradient sits in ``self.flat``; :meth:`all_reduce_` averages it across ranks with a
    single collective.  Optimisers see ordinary ``.grad`` tensors.
    """

    def __init__(self, params, group=None, flat: torch.Tensor | None = None,
                 force: bool = False):
        self.force = force  # all-reduce even in a 1-rank group (rehearsing the collective)
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.group = group
        if flat is not None:  # gradients already live in this buffer (e.g. FlatAdamW's,
            # whose parameter slices are aligned: it may hold zero gaps between them)
            if flat.numel() < total:
                raise ValueError("flat gradient buffer does not match the parameters")
            self.flat = flat
            return
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatGradReducer expects fp32 parameters")
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n

    @property
    def numel(self) -> int:
        return self.flat.numel()

    def zero_(self) -> None:
        self.flat.zero_()

    def all_reduce_(self) -> None:
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = dist.get_world_size(self.group)
        if world == 1 and not self.force:
            return
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.div_(world)

    def check_views(self) -> bool:
        """True while every .grad still aliases the flat buffer (nobody replaced it)."""
        base = self.flat.data_ptr()
        end = base + self.flat.numel() * 4
        return all(p.grad is not None and base <= p.grad.data_ptr() < end for p in self.params)


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Start every rank from rank ``src``'s parameters and buffers."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t, src=src, group=group)


def shard_range(num_graphs: int, rank: int, world: int) -> tuple[int, int]:
    """Graphs [lo, hi) of a global batch owned by ``rank`` (contiguous, balanced)."""
    base, rem = divmod(num_graphs, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)
