"""The C++ autograd binding of the GINE layer (csrc/torch/gine_torch.cpp) for the drop-in path.

``raincast_gnn.nn.GINEConv`` called from the reference's own module tree and training loop
(models/gnn.py:41,44; train.py:61-71: eager autograd, no HIP graph) spends its time on the
host: the Python autograd Function issues one ctypes call per launch and marshals ~30
arguments each time (profiles/r04_s02_dropin_prof.txt).  The extension issues the same
launches from one C++ torch::autograd::Function -- one Python call per layer forward, none in
backward.  It is built in-tree next to libgine_hip.so (``build()``, called by
``__graft_entry__.build``) and loaded from there; a missing extension leaves the Python
Function in charge (same kernels, same bits), it is never a CPU fallback.
"""
from __future__ import annotations

import importlib.util
import os
import threading

import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
EXT_DIR = os.path.join(_HERE, "_native", "torch_ext")
EXT_PATH = os.path.join(EXT_DIR, "gine_torch.so")
SOURCE = os.path.join(os.path.dirname(_HERE), "csrc", "torch", "gine_torch.cpp")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")

_lock = threading.Lock()
_ext = None
_tried = False


def build(verbose: bool = False) -> str:
    """Compile the extension in-tree (g++ against torch's headers, linked to libgine_hip.so
    with an $ORIGIN rpath).  Returns the path of the built module."""
    from torch.utils.cpp_extension import load
    os.makedirs(EXT_DIR, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    load(name="gine_torch", sources=[SOURCE], build_directory=EXT_DIR, verbose=verbose,
         extra_include_paths=[INCLUDE],
         extra_cflags=["-O2", "-D__HIP_PLATFORM_AMD__", f"-I{rocm}/include"],
         extra_ldflags=[f"-L{os.path.dirname(_lib.LIB_PATH)}", "-lgine_hip",
                        "-Wl,-rpath,\\$$ORIGIN/..", "-lc10_hip", "-ltorch_hip"])
    return EXT_PATH


def get():
    """The loaded extension module, or None when it was not built (or was built against
    another ABI version of the library)."""
    global _ext, _tried
    if _tried:
        return _ext
    with _lock:
        if not _tried:
            _tried = True
            if os.path.exists(EXT_PATH) and os.environ.get("GINE_HIP_LIB") is None:
                _lib.load()   # the same libgine_hip.so the extension links (rpath $ORIGIN/..)
                spec = importlib.util.spec_from_file_location("gine_torch", EXT_PATH)
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                if mod.ABI_VERSION == _lib.ABI_VERSION:
                    _ext = mod
    return _ext


# io option order of gine_torch.cpp (IntOpt): then 5 scalars per window plan (in, out)
(IO_EPI, IO_LIN, IO_BATCH, IO_UPDATE, IO_FUSED, IO_LAYER, IO_DEG, IO_ENGINE, IO_LAYER_BWD,
 IO_PLAN_IN) = range(10)
IO_PLAN_OUT = IO_PLAN_IN + 5


def _plan_args(graph, side: str, D: int):
    """(5 scalars, 5 device arrays) of a window plan for gine_torch.cpp: num_tiles (0: no
    plan), slice_channels, max_rows, max_edges, max_nodes; tile_begin, win_lo, win_rows, slot,
    edge_begin (None where absent).  The arrays travel as tensors, so the C++ autograd node
    holds them between forward and backward whatever the graph cache does meanwhile."""
    entry = graph.window_plan_entry(side, D)
    if entry is None:
        return [0, 0, 0, 0, 0], [None] * 5
    plan, arrays = entry
    tb, lo, rows, edge_begin = arrays[:4]
    slot = arrays[4] if len(arrays) > 4 else None
    return ([plan.num_tiles, plan.slice_channels, plan.max_rows, plan.max_edges,
             plan.max_nodes], [tb, lo, rows, slot, edge_begin])


def _graph_opts(graph, N: int, D: int, has_acc: bool) -> tuple:
    """(io options, graph tensor list) that depend only on the graph, the sizes and the path
    switches, cached on the graph object (one dict lookup per layer call instead of the plan
    and occupancy queries)."""
    from . import functional as Fn
    from . import options
    key = (N, D, has_acc, options.MP_FUSED, options.LAYER_FWD, options.LAYER_BWD,
           options.LAYER_WIN, options.ENGINE_IN_MP, Fn.layer_policy_key())
    cache = graph._ext_opts
    got = cache.get(key)
    if got is None:
        fused = Fn.fused_forward_ok(graph, N, D)
        lay = fused and has_acc and Fn.layer_forward_ok(N, D, graph.max_in_degree)
        pin, ain = _plan_args(graph, "in", D)
        pout, aout = _plan_args(graph, "out", D)
        lw = graph.layer_windows if options.LAYER_WIN else None
        io = [int(fused), int(lay),
              int(graph.max_in_degree if graph.max_in_degree is not None else -1),
              int(Fn.engine_in_mp_ok(graph, D)), int(Fn.layer_backward_ok(N, D))] + pin + pout
        io += [lw[1] if lw is not None else 0]
        tensors = [graph.in_rowptr, graph.in_src, graph.in_attr, graph.out_rowptr,
                   graph.out_dst, graph.out_attr] + ain + aout
        tensors.append(lw[0] if lw is not None else None)
        got = cache[key] = (io, tensors)
    return got


def layer(ext, x, conv, graph, epilogue: int) -> torch.Tensor:
    """GINEConv.forward's fused layer through the extension (the caller checked that the
    layer's parameters are not flat-buffer slices, i.e. its backward is the non-deferred
    form)."""
    from . import functional as Fn
    from . import options
    l1, bn_mod, _, l2 = conv.nn
    N, D = x.shape
    bn = Fn.BnConfig(bn_mod)
    acc = Fn.bn_accumulator(bn, D, x.device)
    bacc = Fn.bn_accumulator(bn, D, x.device, "bwd") if options.BN_ACC_BWD else None
    gio, tensors = _graph_opts(graph, N, D, acc is not None)
    io = [epilogue, Fn.edge_linear_flag(), int(bn.use_batch_stats),
          int(bn.update_running)] + gio
    fo = [bn.momentum, bn.eps]
    return ext.gine_layer(x, conv.lin.weight, conv.lin.bias, conv.eps, l1.weight, l1.bias,
                          bn_mod.weight, bn_mod.bias, l2.weight, l2.bias, tensors,
                          [bn.running_mean, bn.running_var,
                           bn.num_batches_tracked if bn.update_running else None, acc, bacc],
                          io, fo)
