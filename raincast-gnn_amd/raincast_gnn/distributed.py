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
    note_device_sharing), or when the launcher started more local ranks than this host has
    visible GPUs (LOCAL_WORLD_SIZE > device count: some ranks must share one -- detected
    without the caller's help, e.g. for drop-in GINEConv users that never call
    note_device_sharing).  Their kernels can then hold CUs whenever ours launch, so launches
    that need their whole grid resident at once (the one-launch layer forward's and
    backward's grid barriers: raincast_gnn.functional.layer_forward_ok / layer_backward_ok)
    are not used."""
    if _SHARED_DEVICE:
        return True
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    return local > 1 and torch.cuda.is_available() and local > torch.cuda.device_count()


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
                 force: bool = False, offsets=None):
        self.force = force  # all-reduce even in a 1-rank group (rehearsing the collective)
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.group = group
        self._tail_lo = None       # overlap_after: where the early-reduced tail starts
        self._tail_started = False
        self._armed = False        # this step's hook is registered (tail-then-front order)
        self._tail_work = None
        self._side = None
        if flat is not None:  # gradients already live in this buffer (e.g. FlatAdamW's,
            # whose parameter slices are aligned: it may hold zero gaps between them;
            # ``offsets``: each parameter's slice offset, FlatAdamW._offsets)
            if flat.numel() < total:
                raise ValueError("flat gradient buffer does not match the parameters")
            self.flat = flat
            self.offsets = list(offsets) if offsets is not None else None
            return
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        self.offsets = []
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("FlatGradReducer expects fp32 parameters")
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            self.offsets.append(off)
            off += n

    @property
    def numel(self) -> int:
        return self.flat.numel()

    def zero_(self) -> None:
        self.flat.zero_()

    def _collective(self) -> bool:
        if not (dist.is_available() and dist.is_initialized()):
            return False
        return dist.get_world_size(self.group) > 1 or self.force

    def _mean(self, t: torch.Tensor, world: int) -> None:
        """t <- the mean of t over the ranks.  RCCL: one ReduceOp.AVG collective (its
        scaling by 1/world is exact for the power-of-two worlds the benchmark runs, so the
        bits are those of the sum divided by world, without the division's extra kernel);
        gloo (no AVG): the sum, then the division."""
        if dist.get_backend(self.group) == "nccl":
            dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.div_(world)

    def all_reduce_(self) -> None:
        if not self._collective():
            return
        world = dist.get_world_size(self.group)
        armed, self._armed = self._armed, False
        if not self._tail_started:
            if armed:
                # the hook bailed on this rank (a tail gradient outside the flat buffer) while
                # other ranks may have started their tail: keep the collective sequence every
                # rank issues -- tail, then front -- independent of the rank
                tail, head = self.flat[self._tail_lo:], self.flat[:self._tail_lo]
                self._mean(tail, world)
                self._mean(head, world)
                return
            self._mean(self.flat, world)
            return
        # the tail's collective is in flight (overlap_after): the rest of the buffer now,
        # then join the tail's stream (or wait for its work object on CPU tensors)
        self._tail_started = False
        head = self.flat[:self._tail_lo]
        self._mean(head, world)
        if self._tail_work is not None:
            self._tail_work.wait()
            self._tail_work = None
            self.flat[self._tail_lo:].div_(world)
        else:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)

    # -- overlap of the tail's all-reduce with the rest of the backward --------------------
    def overlap_after(self, module: torch.nn.Module, tail_params) -> None:
        """Start the all-reduce of ``tail_params``' gradients -- which must fill the END of
        the flat buffer, e.g. the GINE stack and the head behind it (models/gnn.py:136-139)
        -- as soon as autograd has differentiated ``module``'s input (``module`` = the GINE
        stack: by then the backward has produced every gradient behind it), on a side stream,
        so that it overlaps the rest of the backward (dense chain, DeepSet).  all_reduce_()
        then reduces the front of the buffer and joins.  Deferred HIP reductions queued so
        far are launched first (raincast_gnn.gradbuf.flush), so the tail is final.  Works
        eagerly and inside HIP-graph capture (RCCL: the tail's collective and the join are
        captured as a fork of the step graph); on CPU tensors (gloo) the tail's collective
        is an async work object."""
        tail = [p for p in tail_params if p.requires_grad]
        if self.offsets is None:
            raise ValueError("overlap_after needs the parameters' offsets in the flat buffer")
        pos = {id(p): off for p, off in zip(self.params, self.offsets)}
        if any(id(p) not in pos for p in tail):
            raise ValueError("overlap_after: a tail parameter is not reduced by this reducer")
        lo = min(pos[id(p)] for p in tail)
        tail_ids = {id(p) for p in tail}
        if any(off >= lo and id(p) not in tail_ids for p, off in zip(self.params, self.offsets)):
            raise ValueError("overlap_after: the tail parameters must fill the end of the "
                             "flat buffer")
        self._tail_lo = lo
        self._tail_params = tail
        if self.flat.is_cuda and self._side is None:
            self._side = torch.cuda.Stream(self.flat.device)
        module.register_forward_pre_hook(self._arm)

    def _arm(self, module, inputs):
        x = inputs[0] if inputs else None
        if (isinstance(x, torch.Tensor) and x.requires_grad and torch.is_grad_enabled()
                and self._collective()):
            x.register_hook(self._start_tail)
            self._armed = True

    def _start_tail(self, grad):
        # every tail gradient must already sit in its slice (adopted flat views); otherwise
        # the end-of-backward gather copies it in and the whole buffer is reduced then
        base, flat = self.flat.data_ptr(), self.flat
        for p in self._tail_params:
            g = p.grad
            if g is None or not (base <= g.data_ptr() < base + 4 * flat.numel()):
                return None
        from . import gradbuf
        gradbuf.flush()  # the deferred reductions of the tail (their kernels precede ours)
        tail = flat[self._tail_lo:]
        world = dist.get_world_size(self.group)
        if flat.is_cuda:
            cur = torch.cuda.current_stream(flat.device)
            self._side.wait_stream(cur)
            with torch.cuda.stream(self._side):
                self._mean(tail, world)
            # (the backward keeps writing the front of the buffer on ``cur`` meanwhile; the
            # flat buffer outlives the step, so no allocator bookkeeping is needed)
        else:
            self._tail_work = dist.all_reduce(tail, op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True)
        self._tail_started = True
        return None

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
