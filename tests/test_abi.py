"""CPU: the C-ABI library loads and exports every symbol include/gine_hip.h declares.

No compute calls (no GPU here); only the host-side argument validation, which returns
before any HIP call.
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from raincast_gnn import _lib

HEADER = os.path.join(ROOT, "include", "gine_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(gine_\w+)\s*\(", text, re.M)))


def test_header_and_binding_agree():
    decl = declared_symbols()
    assert len(decl) >= 17
    assert sorted(_lib.EXPORTED_SYMBOLS) == decl


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.gine_abi_version() == _lib.ABI_VERSION
    out = os.popen(f"nm -D --defined-only {_lib.LIB_PATH}").read()
    exported = set(re.findall(r"\bT (gine_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_status_strings():
    lib = _lib.load()
    assert lib.gine_status_string(0) == b"ok"
    assert b"channel" in lib.gine_status_string(2)
    assert lib.gine_status_string(12345) != b""


def test_host_validation_without_device():
    lib = _lib.load()
    # unsupported channel counts are rejected before any HIP call
    assert lib.gine_mp_fwd(None, None, None, None, None, None, None, None, 10, 6, 0, None) == 2
    assert lib.gine_mp_fwd(None, None, None, None, None, None, None, None, 10, 2048, 0, None) == 2
    assert lib.gine_mp_fwd(None, None, None, None, None, None, None, None, -1, 8, 0, None) == 1
    assert lib.gine_mp_fwd(None, None, None, None, None, None, None, None, 0, 8, 0, None) == 0
    assert lib.gine_mp_fwd(None, None, None, None, None, None, None, None, 5, 8, 4, None) == 1
    n = ctypes.c_int32(0)
    assert lib.gine_mlp_num_partials(1000, 48, ctypes.byref(n)) == 2
    assert lib.gine_mlp_num_partials(1000, 128, ctypes.byref(n)) == 0 and n.value > 0
    assert lib.gine_mp_bwd_num_partials(16000, 128, ctypes.byref(n)) == 0 and n.value > 0
    assert lib.gine_mlp_wgrad_num_chunks(16000, 128, ctypes.byref(n)) == 0 and n.value > 0
    with pytest.raises(_lib.GineError, match="channel"):
        _lib.check(2, "probe")


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.GineError, match="not found"):
        _lib.load(str(tmp_path / "nope.so"))


def test_grad_batch_validation_without_device():
    lib = _lib.load()
    jobs = (_lib.GradJob * 1)()
    assert lib.gine_grad_finalize_batch(jobs, 0, None) == 0          # nothing to do
    assert lib.gine_grad_finalize_batch(jobs, _lib.GRAD_MAX_JOBS + 1, None) == 1
    jobs[0].kind = 99
    assert lib.gine_grad_finalize_batch(jobs, 1, None) == 1          # unknown kind
    jobs[0].kind = _lib.GRAD_JOB_MP
    assert lib.gine_grad_finalize_batch(jobs, 1, None) == 1          # no source
    job = _lib.GradJob()
    buf = ctypes.create_string_buffer(64)
    p = ctypes.addressof(buf)
    assert lib.gine_head_bwd_grad_job(100, 128, 2, p, p, p, ctypes.byref(job)) == 0
    assert job.kind == _lib.GRAD_JOB_SLAB and job.nz == 1 and job.per[0] == 4 * 128 + 4
    assert lib.gine_chain_wgrad_grad_job(16000, 128, 35, p, 11.0, *([p] * 8),
                                         ctypes.byref(job)) == 0
    assert job.nz == 4 and job.wsize[0] == 128 * 163 and job.bscale[3] == 11.0
    assert lib.gine_deepset_bwd_grad_job(16000, 35, 128, p, p, p, ctypes.byref(job)) == 0
    assert job.wsize[0] == 128 * 35 and job.per[0] == 128 * 36


def test_fused_entry_points_validate_without_device():
    """gine_mp_fwd_mlp1 and gine_mp_bwd_win_mlp_wgrad reject bad arguments before any HIP
    call (channels, degree limit, flags, NULL operands, missing plan)."""
    lib = _lib.load()
    buf = ctypes.create_string_buffer(64)
    p = ctypes.addressof(buf)
    f = lib.gine_mp_fwd_mlp1
    assert f(*([p] * 12), 100, 64, 5, 0, None) == 2                       # D != 128
    assert f(*([p] * 12), 100, 128, _lib.MP_FUSED_MAX_DEGREE + 1, 0, None) == 1
    assert f(*([p] * 12), 100, 128, 5, 8, None) == 1                       # bad flag
    assert f(*([p] * 3), None, *([p] * 8), 100, 128, 5, 0, None) == 1      # no edge attrs
    assert f(*([p] * 12), 0, 128, 5, 0, None) == 1                         # no nodes
    g = lib.gine_mp_bwd_win_mlp_wgrad
    plan = _lib.WindowPlan()
    args = [p] * 11 + [100, 128, 1, ctypes.byref(plan)] + [p] * 9
    assert g(*args, 2, None) == 1                                          # empty plan
    assert g(*([p] * 11 + [100, 128, 1, ctypes.byref(plan)] + [None] + [p] * 8), 2, None) == 1
    assert g(*args, 7, None) == 1                                          # bad epilogue
    assert g(*([p] * 11 + [100, 32, 1, ctypes.byref(plan)] + [p] * 9), 2, None) == 2  # D 32
    assert g(*([p] * 11 + [100, 64, 1, ctypes.byref(plan)] + [p] * 9), 2, None) == 1  # D 64


@pytest.mark.parametrize("N,M,H", [(1, 11, 128), (500, 11, 128), (8192, 11, 128),
                                   (8193, 11, 128), (16000, 11, 128), (16000, 11, 64),
                                   (16385, 11, 64), (128000, 17, 128), (97, 5, 256),
                                   (40, 4, 32)])
def test_deepset_group_layout_sizes(N, M, H):
    """Host-side sizing of the DeepSet kernels (csrc/gine_deepset.hip): groups of 2G nodes,
    G = 8 while G = 16 would leave at most one wave per SIMD (H/32 waves per group), 4 below
    half a wave per SIMD, each
    walked as ceil(G*M/16) tiles; one uint16 ReLU mask word per tile and thread (2H
    threads); backward partials: one per group, capped at 512 (H >= 128) or 1,024."""
    lib = _lib.load()
    g16 = -(-N // 32)
    waves16 = g16 * (H // 32)
    G = 4 if waves16 <= 512 else (8 if waves16 <= 1024 else 16)
    groups = -(-N // (2 * G))
    tpg = -(-(G * M) // 16)
    nb = ctypes.c_size_t(0)
    assert lib.gine_deepset_mask_bytes(N, M, H, ctypes.byref(nb)) == 0
    assert nb.value == groups * tpg * 2 * H * 2
    n = ctypes.c_int32(0)
    assert lib.gine_deepset_bwd_num_partials(N, H, ctypes.byref(n)) == 0
    assert n.value == min(groups, 512 if H >= 128 else 1024)


def test_layer_window_fit_query():
    """gine_mp_fwd_layer_windows_fit (host only): (rows + 1) x 512 B of window rows, a 32 x
    round_up(in-degree, 4) slot table of 8-byte entries and 33 rowptr words within the
    launch's 73,712-byte region; at most 144 rows (9 staging loads per gather thread) and
    in-degree <= 32."""
    lib = _lib.load()
    ok = ctypes.c_int32(7)
    for rows, deg, want in [(129, 11, 1), (136, 11, 1), (137, 11, 0), (120, 32, 1),
                            (127, 32, 0), (126, 32, 1), (1, 33, 0), (0, 0, 0), (1, 0, 1),
                            (144, 0, 0), (-1, 0, 0), (10, -1, 0)]:
        assert lib.gine_mp_fwd_layer_windows_fit(rows, deg, ctypes.byref(ok)) == 0
        assert ok.value == want, (rows, deg)
