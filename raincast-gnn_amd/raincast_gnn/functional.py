"""Autograd bindings of the gfx950 GINE kernels.

Two functions sit behind ``GINEConv``:

* :class:`GineMessagePassing` -- ``z = scatter_add(relu(x[src] + lin(a))) + (1 + eps) * x``,
  i.e. PyG ``GINEConv.forward`` up to ``self.nn`` (upstream gine_conv.py; call sites
  models/gnn.py:41,44).  Used with any ``nn``.
* :class:`GineLayer` -- the same plus the node MLP ``Linear -> BatchNorm1d -> ReLU -> Linear``
  (models/gnn.py:21-26) and optionally ResGnn's outer ReLU / residual (models/gnn.py:38-44),
  all in HIP.  Used when ``nn`` has exactly that structure.

Every kernel launch goes to the current HIP stream of the tensors' device; backward runs on
PyTorch's autograd device thread and touches no thread-local state.  Nothing here falls
back to CPU: a tensor on another device raises.
"""
from __future__ import annotations

import ctypes
import os
import weakref
import warnings

import torch

from . import _lib, options
from ._lib import call, ptr
from . import gradbuf
from .gradbuf import grad_out

EPI_NONE, EPI_RELU, EPI_RESIDUAL_RELU = _lib.EPI_NONE, _lib.EPI_RELU, _lib.EPI_RESIDUAL_RELU


_LIN_FLAG = None


def edge_linear_flag() -> int:
    """Rounding of the K=1 edge Linear, matched to what PyG's CPU path does on THIS host.

    CPU ``Linear(1, D)`` is an MKL sgemm with K=1; MKL rounds ``a*w + b`` once (fma) on Intel
    CPUs and twice (mul, then add) on AMD EPYC CPUs, so the reference's own result is
    host-dependent.  ``GINE_EDGE_LINEAR_ROUNDING`` = ``fma`` | ``muladd`` | ``auto`` (default:
    probe torch's CPU Linear once and match it, so the HIP result is bit-identical to the
    reference run on the same machine).
    """
    global _LIN_FLAG
    if _LIN_FLAG is not None:
        return _LIN_FLAG
    mode = os.environ.get("GINE_EDGE_LINEAR_ROUNDING", "auto").lower()
    if mode == "fma":
        _LIN_FLAG = 0
    elif mode == "muladd":
        _LIN_FLAG = _lib.GINE_MP_LIN_MULADD
    elif mode == "auto":
        g = torch.Generator().manual_seed(7)
        a = torch.randn(4096, 1, generator=g) * 3
        w = torch.randn(32, 1, generator=g)
        b = torch.randn(32, generator=g)
        lin = torch.nn.functional.linear(a, w, b)
        fma = (a.double() * w.double().T + b.double()).float()
        muladd = a * w.T + b
        miss_fma = int((lin != fma).sum())
        miss_muladd = int((lin != muladd).sum())
        _LIN_FLAG = 0 if miss_fma <= miss_muladd else _lib.GINE_MP_LIN_MULADD
        if min(miss_fma, miss_muladd) > 2:
            warnings.warn("host CPU Linear(1,D) rounding is neither fma nor mul+add; "
                          "using the closer one", RuntimeWarning)
    else:
        raise ValueError(f"GINE_EDGE_LINEAR_ROUNDING={mode!r}: expected fma, muladd or auto")
    return _LIN_FLAG


_COUNTS: dict = {}  # size queries of the library (functions of their arguments and the device)


def _count(fn: str, n: int, d: int) -> int:
    # some counts follow the device's CU count (grid sizes), so the device is part of the key
    key = (fn, n, d, torch.cuda.current_device() if torch.cuda.is_available() else -1)
    v = _COUNTS.get(key)
    if v is None:
        out = ctypes.c_int32(0)
        call(fn, n, d, ctypes.byref(out))
        v = _COUNTS[key] = int(out.value)
    return v


def _count64(fn: str, d: int) -> int:
    key = (fn, d)
    v = _COUNTS.get(key)
    if v is None:
        out = ctypes.c_int64(0)
        call(fn, d, ctypes.byref(out))
        v = _COUNTS[key] = int(out.value)
    return v


def _as_vec(p: torch.Tensor) -> torch.Tensor:
    """Linear(1, D).weight [D, 1] / bias [D] -> contiguous fp32 [D] view."""
    return p.detach().reshape(-1).contiguous()


def mp_forward(x, graph, lin_w, lin_b, eps, lin_flag=None):
    N, D = x.shape
    z = torch.empty_like(x)
    if N == 0:
        return z
    flag = edge_linear_flag() if lin_flag is None else lin_flag
    plan = graph.window_plan("in", D)
    if plan is not None:
        call("gine_mp_fwd_win", ptr(x), ptr(graph.in_rowptr), ptr(graph.in_src),
             ptr(graph.in_attr), ptr(lin_w), ptr(lin_b), ptr(eps), ptr(z), N, D, flag,
             ctypes.byref(plan), _lib.stream_handle(x.device))
        return z
    call("gine_mp_fwd", ptr(x), ptr(graph.in_rowptr), ptr(graph.in_src), ptr(graph.in_attr),
         ptr(lin_w), ptr(lin_b), ptr(eps), ptr(z), N, D, flag, _lib.stream_handle(x.device))
    return z


def mp_backward(dz, x, graph, lin_w, lin_b, eps, dres=None, self_term=True, lin_flag=None,
                params=(None, None, None), side=None, engine=None, jobs=None):
    """Returns (dx, dlin_w, dlin_b, deps); ``params`` = the (lin.weight, lin.bias, eps)
    Parameters, whose gradients then go straight to their flat-buffer slices if any.
    ``side`` = (slab, chunks, D, dw1, db1, dw2, db2): a node-MLP weight-gradient slab left
    by gine_mlp_bwd1_wgrad, reduced by extra workgroups of the same launch.
    ``engine`` = (dy, y, mask, a1, bn_save, dbn, coef, z, slab, epilogue): the node-MLP
    weight-gradient engine run by extra workgroups of the window launch (the caller checked
    engine_in_mp_ok).  ``jobs``: a list the window form's finish job is appended to (the
    caller launches it with its own in one gine_grad_finalize_batch) instead of its own
    finish launch, when the reduction is not deferred to the end of the backward."""
    N, D = x.shape
    dev = x.device
    dx = torch.empty_like(x)
    p_w, p_b, p_e = params
    dlw = grad_out(p_w, (D,), dev) if p_w is not None else torch.empty(D, device=dev)
    dlb = grad_out(p_b, (D,), dev) if p_b is not None else torch.empty(D, device=dev)
    deps = grad_out(p_e, (1,), dev) if p_e is not None else torch.empty(1, device=dev)
    if N == 0:
        return dx, dlw.zero_(), dlb.zero_(), deps.zero_()
    stream = _lib.stream_handle(dev)
    flags = (_lib.GINE_MP_BWD_SELF if self_term else 0) | (
        edge_linear_flag() if lin_flag is None else lin_flag)
    args = (ptr(dz), ptr(x), ptr(graph.out_rowptr), ptr(graph.out_dst), ptr(graph.out_attr),
            ptr(lin_w), ptr(lin_b), ptr(eps), ptr(dres), ptr(dx))
    plan = graph.window_plan("out", D)
    if plan is not None:
        P = plan.num_tiles
        partials = torch.empty(P, 3, D, dtype=torch.float64, device=dev)
        if engine is not None:
            e_dy, e_y, e_mask, e_a1, e_bn, e_dbn, e_coef, e_z, e_slab, e_epi = engine
            call("gine_mp_bwd_win_mlp_wgrad", *args, ptr(partials), N, D, flags,
                 ctypes.byref(plan), ptr(e_dy), ptr(e_y), ptr(e_mask), ptr(e_a1), ptr(e_bn),
                 ptr(e_dbn), ptr(e_coef), ptr(e_z), ptr(e_slab), e_epi, stream)
        elif side is None:
            call("gine_mp_bwd_win", *args, ptr(partials), N, D, flags, ctypes.byref(plan),
                 stream)
        else:
            slab, chunks, Dm, dw1, db1, dw2, db2 = side
            call("gine_mp_bwd_win_side", *args, ptr(partials), N, D, flags, ctypes.byref(plan),
                 ptr(slab), chunks, Dm, ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), stream)
        if gradbuf.deferrable(dlw, dlb, deps):  # in the end-of-backward batch
            gradbuf.defer(gradbuf.mp_job(partials, P, D, D // plan.slice_channels, dlw, dlb,
                                         deps), dev, (partials,))
        elif jobs is not None:  # in the caller's batch (it keeps ``partials`` alive)
            jobs.append((gradbuf.mp_job(partials, P, D, D // plan.slice_channels, dlw, dlb,
                                        deps), partials))
        else:
            call("gine_mp_bwd_win_finalize", ptr(partials), P, D, plan.slice_channels,
                 ptr(dlw), ptr(dlb), ptr(deps), stream)
        return dx, dlw, dlb, deps
    P = _count("gine_mp_bwd_num_partials", N, D)
    partials = torch.empty(P, 3, D, dtype=torch.float64, device=dev)
    if side is None:
        call("gine_mp_bwd", *args, ptr(partials), N, D, flags, stream)
    else:
        slab, chunks, Dm, dw1, db1, dw2, db2 = side
        call("gine_mp_bwd_side", *args, ptr(partials), N, D, flags, ptr(slab), chunks, Dm,
             ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), stream)
    if gradbuf.deferrable(dlw, dlb, deps):
        gradbuf.defer(gradbuf.mp_job(partials, P, D, 1, dlw, dlb, deps), dev, (partials,))
    else:
        call("gine_mp_bwd_finalize", ptr(partials), P, D, ptr(dlw), ptr(dlb), ptr(deps),
             stream)
    return dx, dlw, dlb, deps


class GineMessagePassing(torch.autograd.Function):
    """z = sum_{e: dst_e = i} relu(x[src_e] + a_e * W_e + b_e) + (1 + eps) * x_i."""

    @staticmethod
    def forward(ctx, x, lin_w, lin_b, eps, graph):
        x = x.contiguous()
        lw, lb, ep = _as_vec(lin_w), _as_vec(lin_b), eps.detach().contiguous()
        z = mp_forward(x, graph, lw, lb, ep)
        ctx.save_for_backward(x, lw, lb, ep)
        ctx.graph = graph
        ctx.lin_w_shape = lin_w.shape
        ctx.params = (lin_w, lin_b, eps)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, lw, lb, ep = ctx.saved_tensors
        dx, dlw, dlb, deps = mp_backward(dz.contiguous(), x, ctx.graph, lw, lb, ep,
                                         params=ctx.params)
        return dx, dlw.view(ctx.lin_w_shape), dlb, deps.view_as(ep), None


class BnConfig:
    """What GineLayer needs from a BatchNorm1d module (torch semantics)."""

    __slots__ = ("running_mean", "running_var", "num_batches_tracked", "momentum", "eps",
                 "use_batch_stats", "update_running", "module")

    def __init__(self, bn: torch.nn.BatchNorm1d):
        self.module = bn
        self.running_mean = bn.running_mean
        self.running_var = bn.running_var
        self.num_batches_tracked = bn.num_batches_tracked
        self.momentum = -1.0 if bn.momentum is None else float(bn.momentum)
        self.eps = float(bn.eps)
        # torch: batch statistics in training mode, or when no running stats are tracked
        self.use_batch_stats = bn.training or (bn.running_mean is None and bn.running_var is None)
        self.update_running = bn.training and bn.track_running_stats


# gine_mp_fwd_mlp1 wins while each workgroup has at most 2 row tiles (256 workgroups of
# 32-row tiles): 15.1 vs 16.9 us at cfg2, but 121 vs 96 us at cfg3 (csrc/gine_mpmlp.hip).
FUSED_MAX_NODES = 2 * 256 * 32


def fused_forward_ok(graph, N: int, D: int) -> bool:
    """gine_mp_fwd_mlp1 applies: D = 128, edge attributes, every in-degree within
    GINE_MP_FUSED_MAX_DEGREE, N <= FUSED_MAX_NODES, no forward window plan
    (options.MP_FUSED: "0" turns it off, "all" lifts the size limit)."""
    mode = options.MP_FUSED
    if mode == "0" or (N > FUSED_MAX_NODES and mode != "all"):
        return False
    deg = graph.max_in_degree
    return (D == 128 and N > 0 and graph.in_attr is not None and deg is not None
            and deg <= _lib.MP_FUSED_MAX_DEGREE and graph.window_plan("in", D) is None)


def engine_in_mp_ok(graph, D: int) -> bool:
    """gine_mp_bwd_win_mlp_wgrad applies: D = 64 or 128 and a 32-channel window plan for
    the backward (options.ENGINE_IN_MP = False keeps the engine in the dz launch)."""
    if not options.ENGINE_IN_MP or D not in (64, 128):
        return False
    plan = graph.window_plan("out", D)
    return plan is not None and plan.slice_channels == 32


_LAYER_OK = {}


def layer_policy_key():
    """What besides the sizes decides layer_forward_ok: whether other processes share this
    device (then part of the chip may be held by their kernels whenever ours launch)."""
    from . import distributed
    return distributed.device_shared()


def layer_window_args(graph) -> tuple:
    """(tile_windows, window_rows) for gine_mp_fwd_layer: the graph's layer window plan when
    it has one and options.LAYER_WIN, else (None, 0) -- the L2 gather."""
    lw = getattr(graph, "layer_windows", None)
    if lw is None or not options.LAYER_WIN:
        return None, 0
    return ptr(lw[0]), lw[1]


def layer_forward_ok(N: int, D: int, max_in_degree) -> bool:
    """gine_mp_fwd_layer applies (include/gine_hip.h: D = 128, in-degree <= 32, at most two row
    tiles per workgroup and the whole grid resident at once on this device).  Its grid
    barrier needs every workgroup resident at once, which the occupancy query promises only
    for an otherwise idle device: when other ranks share this GPU (distributed.device_shared)
    the pair of launches runs instead.  A barrier that still cannot complete (another
    process's kernels) fails loudly: check_grid_barriers."""
    if max_in_degree is None or not options.LAYER_FWD or layer_policy_key():
        return False
    dev = torch.cuda.current_device()
    key = (dev, N, D, int(max_in_degree))
    ok = _LAYER_OK.get(key)
    if ok is None:
        out = ctypes.c_int32(0)
        call("gine_mp_fwd_layer_ok", N, D, int(max_in_degree), ctypes.byref(out))
        ok = _LAYER_OK[key] = bool(out.value)
    return ok


_LAYER_BWD_OK = {}


def layer_backward_ok(N: int, D: int) -> bool:
    """gine_mlp_bwd_layer applies (include/gine_hip.h: D = 128, at most two row tiles per
    workgroup, the whole grid resident at once); off when other ranks share this GPU, for
    the reason layer_forward_ok gives."""
    if not options.LAYER_BWD or layer_policy_key():
        return False
    dev = torch.cuda.current_device()
    key = (dev, N, D)
    ok = _LAYER_BWD_OK.get(key)
    if ok is None:
        out = ctypes.c_int32(0)
        call("gine_mlp_bwd_layer_ok", N, D, ctypes.byref(out))
        ok = _LAYER_BWD_OK[key] = bool(out.value)
    return ok


_BN_ACC = weakref.WeakKeyDictionary()


def bn_accumulator(bn: "BnConfig", D: int, dev, kind: str = "fwd") -> "torch.Tensor | None":
    """The int64 fixed-point accumulator of gine_mlp_fwd2_bn for this BatchNorm (one per
    module and device, zeroed at allocation, then owned by the kernels), or None when the
    finish launch is needed: eval mode, momentum=None, or options.BN_ACC = False."""
    if (not bn.use_batch_stats or bn.momentum < 0 or bn.module is None
            or not options.BN_ACC):
        return None
    per_dev = _BN_ACC.setdefault(bn.module, {})
    acc = per_dev.get((dev, kind))
    words = _count64("gine_bn_acc_words", D)
    if acc is None or acc.numel() != words:
        acc = torch.zeros(words, dtype=torch.int64, device=dev)
        per_dev[(dev, kind)] = acc
    return acc


_FAIL_INDEX: dict = {}


def check_grid_barriers(group=None) -> None:
    """Raise GineError if a one-launch layer forward's or backward's grid barrier timed out
    since the last check (gine_bn_acc_barrier_failures_index: the grid was not resident at
    once, so that launch's outputs are NaN in the failed workgroups' rows; the failure is
    sticky on the device: every later statistic of that accumulator is NaN until this reset).
    The affected accumulators are re-zeroed, so the next step starts a fresh pairing.  Reads
    device memory: call it where the caller synchronises anyway (end of an epoch, after a
    benchmark's timed steps; drop-in GINEConv users: at their own synchronisation points).
    Collective under torch.distributed (every rank of ``group`` must call it): the failure
    counts are all-reduced (MAX) first, so every rank raises together instead of the others
    blocking in their next collective."""
    failed = []
    for mod, per_dev in list(_BN_ACC.items()):
        for (dev, kind), acc in list(per_dev.items()):
            D = mod.num_features
            idx = _FAIL_INDEX.get(D)
            if idx is None:
                out = ctypes.c_int64(0)
                call("gine_bn_acc_barrier_failures_index", D, ctypes.byref(out))
                idx = _FAIL_INDEX[D] = int(out.value)
            n = int(acc[idx].item())
            if n:
                failed.append((type(mod).__name__, kind, str(dev), n))
                acc.zero_()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        on_gpu = dist.get_backend(group) == "nccl"
        t = torch.tensor([len(failed)], dtype=torch.int64,
                         device=torch.device("cuda", torch.cuda.current_device()) if on_gpu
                         else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        if int(t.item()) and not failed:
            raise _lib.GineError(
                "gine_mp_fwd_layer / gine_mlp_bwd_layer: another rank's grid barrier timed out "
                "(its launch's outputs are NaN); raised on every rank together")
    if failed:
        raise _lib.GineError(
            "gine_mp_fwd_layer / gine_mlp_bwd_layer: the grid barrier timed out (the launch's "
            f"workgroups were not all resident at once: other work held CUs) -- {failed} "
            "(module, fwd|bwd, device, workgroups); those launches' outputs are NaN in the "
            "failed workgroups' rows and the running statistics were not updated; the "
            "accumulators were reset")


class _paired:
    """Producer/consumer launches on one BatchNorm accumulator (csrc/gine_bnacc.hpp): if
    anything raises between the two, the accumulator is re-zeroed so the next step starts a
    fresh pairing instead of differencing against a stale snapshot."""

    __slots__ = ("acc",)

    def __init__(self, acc):
        self.acc = acc

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is not None and self.acc is not None:
            self.acc.zero_()
        return False


class GineLayer(torch.autograd.Function):
    """y = epilogue( Linear2( ReLU( BN( Linear1( z ) ) ) ) ),  z = GINE message passing.

    epilogue: EPI_NONE -> o, EPI_RELU -> relu(o), EPI_RESIDUAL_RELU -> x + relu(o).
    head: a head.HeadPlan for the output head that reads y (the stack's last layer), run by
    the one-launch form's epilogue (gine_layer_head); other forms leave it to the head.
    """

    @staticmethod
    def forward(ctx, x, lin_w, lin_b, eps, w1, b1, gamma, beta, w2, b2, graph, bn, epilogue,
                head=None):
        x = x.contiguous()
        N, D = x.shape
        dev = x.device
        stream = _lib.stream_handle(dev)
        lw, lb, ep = _as_vec(lin_w), _as_vec(lin_b), eps.detach().contiguous()
        w1c, b1c, w2c, b2c = (t.detach().contiguous() for t in (w1, b1, w2, b2))
        g = gamma.detach().contiguous() if gamma is not None else None
        bt = beta.detach().contiguous() if beta is not None else None
        if bn.use_batch_stats and N <= 1:
            raise ValueError(
                f"Expected more than 1 value per channel when training, got input size "
                f"{torch.Size([N, D])}")

        a1 = torch.empty_like(x)
        acc = bn_accumulator(bn, D, dev)
        # everything the consumer needs exists before the producer launches (gine_bnacc.hpp:
        # a producer without its consumer breaks the pairing)
        bn_save = torch.empty(4, D, dtype=torch.float32, device=dev)
        nbt = ptr(bn.num_batches_tracked) if bn.update_running else None
        update_running = int(bn.update_running and bn.running_mean is not None)
        y = torch.empty_like(x)
        mask = (torch.empty(N, D, dtype=torch.uint8, device=dev)
                if epilogue == EPI_RESIDUAL_RELU else None)
        fused = fused_forward_ok(graph, N, D)
        # fused: the gather runs inside the Linear1 launch; else the gather first, unpaired
        z = torch.empty_like(x) if fused else mp_forward(x, graph, lw, lb, ep)
        if acc is None:
            P = _count("gine_mlp_num_partials", N, D)
            partials = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
        else:  # statistics summed by integer atomics, finished inside the second GEMM
            partials = None
        layer = fused and acc is not None and layer_forward_ok(N, D, graph.max_in_degree)
        hargs = head.args(N, D, dev) if layer and head is not None else None
        with _paired(acc):
            if layer:
                # the whole layer forward in one launch (grid barrier between its halves)
                call("gine_mp_fwd_layer", ptr(x), ptr(graph.in_rowptr), ptr(graph.in_src),
                     ptr(graph.in_attr), ptr(lw), ptr(lb), ptr(ep), ptr(w1c), ptr(b1c), ptr(z),
                     ptr(a1), ptr(acc), ptr(g), ptr(bt), ptr(bn.running_mean),
                     ptr(bn.running_var), nbt, ptr(bn_save), bn.momentum, bn.eps,
                     update_running, ptr(w2c), ptr(b2c), ptr(y), ptr(mask), N, D,
                     graph.max_in_degree, edge_linear_flag(), epilogue,
                     *layer_window_args(graph),
                     ctypes.byref(hargs) if hargs is not None else None, stream)
                if hargs is not None:
                    head.done = (y.data_ptr(), tuple(y.shape))
            elif fused:
                # gather of the next tile beside the matrix chain of this one: one launch
                args = (ptr(x), ptr(graph.in_rowptr), ptr(graph.in_src), ptr(graph.in_attr),
                        ptr(lw), ptr(lb), ptr(ep), ptr(w1c), ptr(b1c), ptr(z), ptr(a1),
                        ptr(partials))
                tail = (N, D, graph.max_in_degree, edge_linear_flag(), stream)
                if acc is None:
                    call("gine_mp_fwd_mlp1", *args, *tail)
                else:
                    call("gine_mp_fwd_mlp1_acc", *args, ptr(acc), *tail)
            elif acc is None:
                call("gine_mlp_fwd1", ptr(z), ptr(w1c), ptr(b1c), ptr(a1), ptr(partials), N,
                     D, stream)
            else:
                call("gine_mlp_fwd1_acc", ptr(z), ptr(w1c), ptr(b1c), ptr(a1), None,
                     ptr(acc), N, D, stream)
            if layer:
                pass
            elif acc is None:
                call("gine_bn_fwd_finalize", ptr(partials), P, ptr(g), ptr(bt),
                     ptr(bn.running_mean), ptr(bn.running_var), nbt, ptr(bn_save), N, D,
                     bn.momentum, bn.eps, int(bn.use_batch_stats), update_running, stream)
                call("gine_mlp_fwd2", ptr(a1), ptr(bn_save), ptr(w2c), ptr(b2c), ptr(x),
                     ptr(y), ptr(mask), N, D, epilogue, stream)
            else:
                call("gine_mlp_fwd2_bn", ptr(a1), ptr(acc), ptr(g), ptr(bt),
                     ptr(bn.running_mean), ptr(bn.running_var), nbt, ptr(bn_save),
                     bn.momentum, bn.eps, update_running, ptr(w2c), ptr(b2c), ptr(x), ptr(y),
                     ptr(mask), N, D, epilogue, stream)

        ctx.save_for_backward(x, z, a1, y if epilogue == EPI_RELU else None, mask, bn_save,
                              lw, lb, ep, w1c, w2c, g)
        ctx.graph, ctx.epilogue = graph, epilogue
        ctx.use_batch_stats = bn.use_batch_stats
        # backward form (options.BN_ACC_BWD); allocated here, outside backward
        ctx.bn_acc_bwd = bn_accumulator(bn, D, dev, "bwd") if options.BN_ACC_BWD else None
        ctx.params = (lin_w, lin_b, eps, w1, b1, gamma, beta, w2, b2)
        ctx.shapes = (lin_w.shape, gamma is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, z, a1, y, mask, bn_save, lw, lb, ep, w1c, w2c, g = ctx.saved_tensors
        dy = dy.contiguous()
        N, D = x.shape
        dev = x.device
        stream = _lib.stream_handle(dev)
        epi = ctx.epilogue

        p_lw, p_lb, p_eps, p_w1, p_b1, p_g, p_bt, p_w2, p_b2 = ctx.params
        dgamma = grad_out(p_g, (D,), dev) if p_g is not None else None
        dbeta = grad_out(p_bt, (D,), dev) if p_bt is not None else None
        dw1, db1 = grad_out(p_w1, (D, D), dev), grad_out(p_b1, (D,), dev)
        dw2, db2 = grad_out(p_w2, (D, D), dev), grad_out(p_b2, (D,), dev)
        deferrable = gradbuf.deferrable(dw1, db1, dw2, db2)
        # the node-MLP weight-gradient engine inside the window backward launch wherever a
        # 32-channel plan exists: its slab joins the end-of-backward batch (deferred), or
        # this layer's own batch launch with the message passing's finish (drop-in path)
        use_engine = engine_in_mp_ok(ctx.graph, D)
        # BatchNorm backward sums as fixed-point atomics, finished in the dz GEMM
        acc = ctx.bn_acc_bwd if use_engine else None

        dbn = torch.empty_like(x)
        coef = torch.empty(3, D, dtype=torch.float32, device=dev)
        dz = torch.empty_like(x)
        C = _count("gine_mlp_wgrad_num_chunks", N, D)
        slab = torch.empty(2 * C * (D * D + D), dtype=torch.float32, device=dev)
        if acc is None:
            P = _count("gine_mlp_num_partials", N, D)
            partials = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
            call("gine_mlp_bwd2", ptr(dy), ptr(y), ptr(mask), ptr(a1), ptr(bn_save), ptr(w2c),
                 ptr(dbn), ptr(partials), N, D, epi, stream)
            call("gine_bn_bwd_finalize", ptr(partials), P, ptr(g), ptr(bn_save), ptr(dgamma),
                 ptr(dbeta), ptr(coef), N, D, int(ctx.use_batch_stats), stream)
        engine = None
        if use_engine:
            # dz = da1 W1 alone; the dW1, dW2 slab from extra workgroups of the
            # message-passing backward launch below
            if acc is None:
                call("gine_mlp_bwd1", ptr(dbn), ptr(a1), ptr(bn_save), ptr(coef), ptr(w1c),
                     ptr(dz), N, D, stream)
            else:
                with _paired(acc):  # producer + consumer back to back
                    if layer_backward_ok(N, D):  # the pair in one launch (grid barrier)
                        call("gine_mlp_bwd_layer", ptr(dy), ptr(y), ptr(mask), ptr(a1),
                             ptr(bn_save), ptr(w2c), ptr(dbn), ptr(acc), ptr(g), ptr(dgamma),
                             ptr(dbeta), ptr(coef), ptr(w1c), ptr(dz), N, D, epi, stream)
                    else:
                        call("gine_mlp_bwd2_acc", ptr(dy), ptr(y), ptr(mask), ptr(a1),
                             ptr(bn_save), ptr(w2c), ptr(dbn), None, ptr(acc), N, D, epi,
                             stream)
                        call("gine_mlp_bwd1_bn", ptr(dbn), ptr(a1), ptr(bn_save), ptr(acc),
                             ptr(g), ptr(dgamma), ptr(dbeta), ptr(coef), ptr(w1c), ptr(dz),
                             N, D, stream)
            engine = (dy, y, mask, a1, bn_save, dbn, coef, z, slab, epi)
        else:
            # dz = da1 W1 and the dW1, dW2 partial slabs side by side in one launch
            call("gine_mlp_bwd1_wgrad", ptr(dy), ptr(y), ptr(mask), ptr(a1), ptr(bn_save),
                 ptr(dbn), ptr(coef), ptr(z), ptr(w1c), ptr(dz), ptr(slab), None, None, None,
                 None, N, D, epi, stream)
        dres = dy if epi == EPI_RESIDUAL_RELU else None
        jobs = None
        if deferrable or use_engine:
            # only the optimizer reads dW1/db1/dW2/db2: the slab is reduced by a batch launch
            # (the end-of-backward one when deferrable), off the message passing's path
            per = D * D + D
            job = _lib.GradJob()
            job.kind, job.src, job.rows, job.nz = _lib.GRAD_JOB_SLAB, slab.data_ptr(), C, 2
            job.cstride, job.zstride = per, per * C
            for zi, (wg, bg) in enumerate(((dw2, db2), (dw1, db1))):  # MlpWgradOut order
                job.per[zi], job.wsize[zi], job.bscale[zi] = per, D * D, 1.0
                job.w[zi], job.b[zi] = wg.data_ptr(), bg.data_ptr()
            if deferrable:
                gradbuf.defer(job, dev, (slab,))
            else:
                jobs = [(job, slab)]
            side = None
        else:  # reduced by extra workgroups of the message-passing backward launch
            side = (slab, C, D, dw1, db1, dw2, db2)
        dx, dlw, dlb, deps = mp_backward(dz, x, ctx.graph, lw, lb, ep, dres=dres,
                                         params=(p_lw, p_lb, p_eps), side=side, engine=engine,
                                         jobs=jobs)
        if jobs:  # this layer's slab and message-passing finish in one launch
            arr = (_lib.GradJob * len(jobs))(*[j for j, _ in jobs])
            call("gine_grad_finalize_batch", arr, len(jobs), stream)
        lin_w_shape, affine = ctx.shapes
        return (dx, dlw.view(lin_w_shape), dlb, deps.view_as(ep), dw1, db1, dgamma, dbeta,
                dw2, db2, None, None, None, None)
