"""CPU: ISA audit of the shipped gfx950 code objects (tools/isa_audit.py).

* No packed-FP32 VALU instruction (v_pk_fma/mul/add_f32) anywhere in libgine_hip.so: their
  low halves came out wrong beside v_mfma_f32_32x32x16_bf16 waves on MI355X (DESIGN.md 4,
  profiles/r05_s03_determinism_probes.txt), and the only guard is the Makefile's NOPK feature
  switch -- a toolchain update or a new build rule could drop it silently.
* The detector is live: the same per-edge arithmetic compiled without NOPK does contain them.
* Scratch (spill) instructions per kernel stay within the committed ceiling
  (tests/golden/isa_scratch_ceiling.json; kernels not listed: none).
"""
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT
from raincast_gnn import _lib

import sys
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_audit  # noqa: E402

CSRC = os.path.join(ROOT, "raincast-gnn_amd", "csrc")
CEILING = os.path.join(GOLDEN, "isa_scratch_ceiling.json")
NOPK = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


@pytest.fixture(scope="module")
def table():
    assert os.path.exists(_lib.LIB_PATH), "build the library first (__graft_entry__.build)"
    return isa_audit.audit(_lib.LIB_PATH)


def test_shipped_library_has_no_packed_fp32(table):
    assert len(table) > 100  # every code object was unbundled and disassembled
    bad = {k: v["packed_f32"] for k, v in table.items() if v.get("packed_f32")}
    assert not bad, f"packed-FP32 VALU in {len(bad)} kernels: {sorted(bad)[:5]}"
    # the hot kernels are in the table and run their MFMA chains (the window backward: its
    # engine-carrying instantiations)
    for frag, every in (("k_mp_fwd_layer", True), ("k_mlp_bwd_layer", True),
                        ("k_mp_bwd_win", False)):
        hits = [v.get("mfma", 0) > 0 for k, v in table.items() if frag in k]
        assert hits and (all(hits) if every else any(hits)), frag


def test_scratch_within_committed_ceiling(table):
    ceiling = json.load(open(CEILING))
    over = {}
    for k, v in table.items():
        s = v.get("scratch", 0)
        if s > ceiling.get(k, 0):
            over[k] = (s, ceiling.get(k, 0))
    assert not over, f"scratch ops above the ceiling (found, allowed): {over}"


def _compile_probe(tmp_path, flags):
    out = tmp_path / ("probe_%d.o" % len(flags))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", *flags, "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                    "-c", os.path.join(ROOT, "tests", "native", "pk_probe.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    table = {}
    for obj in isa_audit.code_objects(str(out)):
        table.update(isa_audit.count_ops(isa_audit.disassemble(obj)))
    return sum(v.get("packed_f32", 0) for v in table.values())


def test_detector_sees_packed_fp32_without_nopk(tmp_path):
    assert _compile_probe(tmp_path, []) > 0  # the default build would ship them
    assert _compile_probe(tmp_path, NOPK) == 0
