"""ctypes binding of ``libgine_hip.so`` (the C ABI declared in ``include/gine_hip.h``).

The library is loaded lazily on first use and never replaced by a fallback: when it is
missing or a device is absent every op raises.  ``torch`` is imported first on purpose --
its bundled ``libamdhip64.so`` (SONAME ``libamdhip64.so.7``) must be the runtime our library
binds to, so both share one HIP runtime, one set of streams and one caching allocator.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (load order: torch's HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GINE_HIP_LIB", os.path.join(_HERE, "_native", "libgine_hip.so"))

GINE_OK = 0
GINE_ERR_INVALID, GINE_ERR_DIM = 1, 2
GINE_ERR_HIP_BASE = 1000
GINE_MP_BWD_SELF = 1
GINE_MP_LIN_MULADD = 2
EPI_NONE, EPI_RELU, EPI_RESIDUAL_RELU = 0, 1, 2
LOSS_NORMAL, LOSS_MIXED_NORMAL, LOSS_MIXED, LOSS_MIXED_U = 0, 1, 2, 3
ABI_VERSION = 8
COUNT_PARTS = 64  # GINE_COUNT_PARTS

_c_void_p = ctypes.c_void_p
_i32, _i64, _f32, _size = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t
_f64 = ctypes.c_double



class WindowPlan(ctypes.Structure):
    """``gine_window_plan`` (include/gine_hip.h): device tile arrays + LDS sizing."""
    _fields_ = [("tile_begin", _c_void_p), ("win_lo", _c_void_p), ("win_rows", _c_void_p),
                ("num_tiles", _i32), ("slice_channels", _i32), ("max_rows", _i32),
                ("max_edges", _i32), ("max_nodes", _i32), ("slot", _c_void_p),
                ("edge_begin", _c_void_p)]


_plan_p = ctypes.POINTER(WindowPlan)


class GradJob(ctypes.Structure):
    """``gine_grad_job`` (include/gine_hip.h): one reduction of gine_grad_finalize_batch."""
    _fields_ = [("kind", _i32), ("rows", _i32), ("channels", _i32), ("eps_cols", _i32),
                ("nz", _i32), ("pad_", _i32), ("src", _c_void_p), ("cstride", _i64),
                ("zstride", _i64), ("per", _i64 * 4), ("wsize", _i64 * 4),
                ("bscale", _f32 * 4), ("w", _c_void_p * 4), ("b", _c_void_p * 4)]


class LayerHead(ctypes.Structure):
    """``gine_layer_head`` (include/gine_hip.h): the output head folded into the last layer's
    gine_mp_fwd_layer launch."""
    _fields_ = [("weight", _c_void_p), ("bias", _c_void_p), ("raw", _c_void_p),
                ("pred", _c_void_p), ("y_target", _c_void_p), ("count_parts", _c_void_p),
                ("kind", _i32)]


GRAD_JOB_MP, GRAD_JOB_SLAB, GRAD_MAX_JOBS = 1, 2, 12
MP_FUSED_MAX_DEGREE = 32  # GINE_MP_FUSED_MAX_DEGREE
_job_p = ctypes.POINTER(GradJob)
WINDOW_LDS_BYTES = 80 * 1024

# name -> argtypes (every entry point returns int status)
_SIGNATURES = {
    "gine_graph_workspace_bytes": [_i64, _i64, ctypes.POINTER(_size)],
    "gine_graph_build": [_c_void_p, _c_void_p, _i64, _i64, _c_void_p, _c_void_p, _c_void_p,
                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size, _c_void_p],
    "gine_graph_same_edges": [_c_void_p] * 4 + [_i64, _c_void_p, _c_void_p],
    "gine_host_device_ptr": [_c_void_p, ctypes.POINTER(_c_void_p)],
    "gine_mp_fwd": [_c_void_p] * 8 + [_i64, _i32, _i32, _c_void_p],
    "gine_mp_bwd_num_partials": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_mp_bwd": [_c_void_p] * 11 + [_i64, _i32, _i32, _c_void_p],
    "gine_mp_bwd_side": [_c_void_p] * 11 + [_i64, _i32, _i32, _c_void_p, _i32, _i32]
                        + [_c_void_p] * 5,
    "gine_mp_bwd_finalize": [_c_void_p, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "gine_graph_order_locality": [_c_void_p, _c_void_p, _i64, _c_void_p],
    "gine_graph_plan_windows": [_c_void_p, _c_void_p, _i64, _i32, _i32, _i32, _c_void_p,
                                _c_void_p, _c_void_p, ctypes.POINTER(_i32), _c_void_p],
    "gine_mp_fwd_win": [_c_void_p] * 8 + [_i64, _i32, _i32, _plan_p, _c_void_p],
    "gine_mp_bwd_win": [_c_void_p] * 11 + [_i64, _i32, _i32, _plan_p, _c_void_p],
    "gine_mp_bwd_win_mlp_wgrad": [_c_void_p] * 11 + [_i64, _i32, _i32, _plan_p]
                                 + [_c_void_p] * 9 + [_i32, _c_void_p],
    "gine_mp_bwd_win_side": [_c_void_p] * 11 + [_i64, _i32, _i32, _plan_p, _c_void_p, _i32,
                                                 _i32] + [_c_void_p] * 5,
    "gine_mp_bwd_win_finalize": [_c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p,
                                 _c_void_p],
    "gine_grad_finalize_batch": [_job_p, _i32, _c_void_p],
    "gine_head_bwd_grad_job": [_i64, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _job_p],
    "gine_chain_wgrad_grad_job": [_i64, _i32, _i32, _c_void_p, _f32] + [_c_void_p] * 8
                                 + [_job_p],
    "gine_deepset_bwd_grad_job": [_i64, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _job_p],
    "gine_mlp_num_partials": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_mlp_fwd1": [_c_void_p] * 5 + [_i64, _i32, _c_void_p],
    "gine_mp_fwd_mlp1": [_c_void_p] * 12 + [_i64, _i32, _i32, _i32, _c_void_p],
    "gine_mp_fwd_mlp1_acc": [_c_void_p] * 13 + [_i64, _i32, _i32, _i32, _c_void_p],
    "gine_mp_fwd_layer_ok": [_i64, _i32, _i32, ctypes.POINTER(_i32)],
    "gine_mp_fwd_layer": [_c_void_p] * 18 + [_f32, _f32, _i32] + [_c_void_p] * 4
                         + [_i64, _i32, _i32, _i32, _i32, _c_void_p, _i32,
                            ctypes.POINTER(LayerHead), _c_void_p],
    "gine_graph_plan_layer_windows": [_c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p,
                                      _c_void_p],
    "gine_mp_fwd_layer_windows_fit": [_i32, _i32, ctypes.POINTER(_i32)],
    "gine_mlp_fwd1_acc": [_c_void_p] * 6 + [_i64, _i32, _c_void_p],
    "gine_mlp_fwd2_bn": [_c_void_p] * 8 + [_f32, _f32, _i32] + [_c_void_p] * 5
                        + [_i64, _i32, _i32, _c_void_p],
    "gine_bn_acc_words": [_i32, _c_void_p],
    "gine_bn_acc_barrier_failures_index": [_i32, _c_void_p],
    "gine_testing_layer_extra_workgroups": [_i32],
    "gine_testing_sum_32": [_c_void_p, _c_void_p, _i32, _i32, _c_void_p],
    "gine_mlp_bwd2_acc": [_c_void_p] * 9 + [_i64, _i32, _i32, _c_void_p],
    "gine_mlp_bwd1_bn": [_c_void_p] * 10 + [_i64, _i32, _c_void_p],
    "gine_mlp_bwd_layer_ok": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_mlp_bwd_layer": [_c_void_p] * 14 + [_i64, _i32, _i32, _c_void_p],
    "gine_testing_bwd_layer_extra_workgroups": [_i32],
    "gine_bn_fwd_finalize": [_c_void_p, _i32] + [_c_void_p] * 6 + [_i64, _i32, _f32, _f32, _i32,
                                                                   _i32, _c_void_p],
    "gine_mlp_fwd2": [_c_void_p] * 7 + [_i64, _i32, _i32, _c_void_p],
    "gine_mlp_bwd2": [_c_void_p] * 8 + [_i64, _i32, _i32, _c_void_p],
    "gine_bn_bwd_finalize": [_c_void_p, _i32] + [_c_void_p] * 5 + [_i64, _i32, _i32, _c_void_p],
    "gine_mlp_bwd1": [_c_void_p] * 6 + [_i64, _i32, _c_void_p],
    "gine_mlp_wgrad_num_chunks": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_mlp_wgrad": [_c_void_p] * 13 + [_i64, _i32, _i32, _c_void_p],
    "gine_mlp_bwd1_wgrad": [_c_void_p] * 15 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_wgrad": [_c_void_p] * 12 + [_f32] + [_c_void_p] * 6 + [_i64, _i32, _i32,
                                                                        _c_void_p],
    "gine_head_bwd_reduce": [_c_void_p] * 3 + [_i64, _i32, _i32, _c_void_p],
    "gine_adamw_step": [_c_void_p] * 5 + [_i64, _f32, _f32, _f32, _f32, _f32, _c_void_p],
    "gine_crps_num_partials": [_i64, ctypes.POINTER(_i32)],
    "gine_crps_fwd": [_c_void_p, _c_void_p, _i64, _i32, _f64, _f64, _f64, _f64, _c_void_p,
                      _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "gine_crps_bwd": [_c_void_p, _c_void_p, _c_void_p, _i64, _i32, _c_void_p, _c_void_p],
    "gine_count_valid": [_c_void_p, _i64, _c_void_p, _c_void_p],
    "gine_adamw_state_floats": [ctypes.POINTER(_i64)],
    "gine_crps_fwd_grad": [_c_void_p, _c_void_p, _i64, _i32, _f64, _f64, _f64, _f64]
                          + [_c_void_p] * 8,
    "gine_crps_head_slab_floats": [_i64, _i32, _i32, ctypes.POINTER(ctypes.c_size_t)],
    "gine_crps_head_fwd_grad": [_c_void_p, _c_void_p, _i64, _i32, _f64, _f64, _f64, _f64]
                               + [_c_void_p] * 10 + [_i32] + [_c_void_p] * 3,
    "gine_crps_head_grad_job": [_i64, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _job_p],
    "gine_linear_wgrad_num_chunks": [_i64, _i32, _i32, ctypes.POINTER(_i32)],
    "gine_linear_wgrad": [_c_void_p, _c_void_p, _i64, _i32, _i32, _c_void_p, _c_void_p,
                          _c_void_p, _f32, _c_void_p],
    "gine_deepset_mask_bytes": [_i64, _i32, _i32, ctypes.POINTER(_size)],
    "gine_deepset_mask_layout": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_copy_f4": [_c_void_p, _c_void_p, _i64, _c_void_p],
    "gine_probe_chain": [_i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p],
    "gine_deepset_fwd":[_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _i32,
                         _i32, _i32, _c_void_p],
    "gine_deepset_bwd_num_partials": [_i64, _i32, ctypes.POINTER(_i32)],
    "gine_deepset_bwd": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                         _i64, _i32, _i32, _i32, _c_void_p],
    "gine_head_fwd": [_c_void_p] * 5 + [_i64, _i32, _i32, _c_void_p],
    "gine_head_fwd_count": [_c_void_p] * 5 + [_i64, _i32, _i32] + [_c_void_p] * 3,
    "gine_head_bwd_slab_floats": [_i64, _i32, _i32, ctypes.POINTER(_size)],
    "gine_head_bwd": [_c_void_p] * 8 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_fwd": [_c_void_p] * 4 + [_f32] + [_c_void_p] * 10 + [_i64, _i32, _i32,
                                                                       _c_void_p],
    "gine_chain_bwd_slab_floats": [_i64, _i32, _i32, ctypes.POINTER(_size)],
    "gine_chain_bwd": [_c_void_p] * 17 + [_f32] + [_c_void_p] * 6 + [_i64, _i32, _i32,
                                                                       _c_void_p],
    "gine_graph_plan_window_slots": [_c_void_p, _c_void_p, _i32, _c_void_p],
    "gine_chain_fwd_folded": [_c_void_p] * 4 + [_f32] + [_c_void_p] * 10 + [_i64, _i32, _i32,
                                                                              _c_void_p],
    "gine_chain_bwd_folded": [_c_void_p] * 8 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_fwd_folded3": [_c_void_p] * 4 + [_f32] + [_c_void_p] * 6 + [_i64, _i32, _i32,
                                                                             _c_void_p],
    "gine_deepset_fwd_fold": [_c_void_p] * 5 + [_i64, _i32, _i32, _i32] + [_c_void_p] * 5
                             + [_i32, _c_void_p],
    "gine_chain_wgrad_folded": [_c_void_p] * 13 + [_f32, _i64, _i32, _i32, _c_void_p],
    "gine_chain_wgrad_folded_grad_job": [_i64, _i32, _i32, _c_void_p, _f32] + [_c_void_p] * 5
                                        + [_job_p],
    "gine_chain_unfold_grads": [_c_void_p] * 8 + [_i32, _i32, _c_void_p],
    "gine_deepset_fwd_fold2": [_c_void_p] * 5 + [_i64, _i32, _i32, _i32] + [_c_void_p] * 5
                              + [_i32] + [_c_void_p] * 6,
    "gine_chain_fwd_folded2": [_c_void_p] * 6 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_bwd_folded2": [_c_void_p] * 6 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_wgrad_folded2": [_c_void_p] * 8 + [_i64, _i32, _i32, _c_void_p],
    "gine_chain_wgrad_folded2_grad_job": [_i64, _i32, _i32] + [_c_void_p] * 3 + [_job_p],
    "gine_chain_unfold_grads2": [_c_void_p] * 16 + [_f32, _i32, _i32, _c_void_p],
}

EXPORTED_SYMBOLS = ("gine_abi_version", "gine_status_string") + tuple(_SIGNATURES)

_lock = threading.Lock()
_lib = None


class GineError(RuntimeError):
    """A native entry point returned a non-zero status."""


def load(path: str | None = None) -> ctypes.CDLL:
    """Load and type the shared library (idempotent).  Raises when it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise GineError(
                f"native GINE library not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        lib = ctypes.CDLL(p)
        lib.gine_abi_version.restype = ctypes.c_int
        lib.gine_abi_version.argtypes = []
        lib.gine_status_string.restype = ctypes.c_char_p
        lib.gine_status_string.argtypes = [ctypes.c_int]
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = argtypes
        if lib.gine_abi_version() != ABI_VERSION:
            raise GineError(f"ABI mismatch: library {lib.gine_abi_version()} != {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def check(status: int, what: str) -> None:
    if status != GINE_OK:
        msg = load().gine_status_string(status).decode()
        raise GineError(f"{what} failed with status {status}: {msg}")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def ptr(t) -> int | None:
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise GineError(
            f"{what}: the MI355X GINE engine runs on HIP devices only (got a {t.device} tensor); "
            "there is no CPU fallback")
