"""ISA audit of the shipped gfx950 code objects (test infrastructure, CPU only).

Unbundles every gfx950 code object of a HIP shared library's `.hip_fatbin` section (the
clang offload-bundle format: magic, entry count, then offset / size / triple per entry),
disassembles it with llvm-objdump and counts, per kernel symbol:
  * packed-FP32 VALU instructions (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): the library
    must contain none (csrc/Makefile NOPK; gine_common.hpp);
  * scratch (spill) memory instructions (scratch_load_* / scratch_store_*);
  * MFMA instructions (for the record).
    python tools/isa_audit.py [lib.so]      # table of every kernel with packed / scratch ops
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile
from collections import defaultdict

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PACKED_F32 = ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32")
_SYM = re.compile(r"^[0-9a-f]+ <([^>]+)>:$")


def section_bytes(lib: str, section: str = ".hip_fatbin") -> bytes:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sec.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", f"--only-section={section}", lib,
                        out], check=True)
        return open(out, "rb").read()


def code_objects(lib: str, arch: str = "gfx950") -> list[bytes]:
    """Every `arch` device code object in the library's offload bundles."""
    data = section_bytes(lib)
    objs, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return objs
        (n,) = struct.unpack_from("<Q", data, i + len(MAGIC))
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if triple.endswith(arch) and size > 0:
                objs.append(data[i + off:i + off + size])
        pos = i + len(MAGIC)


def disassemble(obj: bytes, arch: str = "gfx950") -> str:
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "co.o")
        open(f, "wb").write(obj)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--mcpu={arch}", f], check=True,
                              capture_output=True, text=True).stdout


def count_ops(asm: str) -> dict[str, dict[str, int]]:
    """{kernel symbol: {"packed_f32", "scratch", "mfma", "insts"}} for one disassembly."""
    out: dict[str, dict[str, int]] = defaultdict(lambda: defaultdict(int))
    sym = None
    for line in asm.splitlines():
        m = _SYM.match(line.strip())
        if m:
            sym = m.group(1)
            continue
        if sym is None or not line.startswith("\t"):
            continue
        op = line.split(None, 1)[0] if line.strip() else ""
        if not op:
            continue
        c = out[sym]
        c["insts"] += 1
        if op.startswith(PACKED_F32):
            c["packed_f32"] += 1
        elif op.startswith(("scratch_load", "scratch_store")):
            c["scratch"] += 1
        elif op.startswith("v_mfma"):
            c["mfma"] += 1
    return out


def audit(lib: str) -> dict[str, dict[str, int]]:
    table: dict[str, dict[str, int]] = {}
    for obj in code_objects(lib):
        for sym, c in count_ops(disassemble(obj)).items():
            table[sym] = dict(c)
    return table


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                           text=True)
    except OSError:
        return list(names)
    return r.stdout.splitlines() if r.returncode == 0 else list(names)


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        here, "raincast-gnn_amd", "raincast_gnn", "_native", "libgine_hip.so")
    t = audit(lib)
    rows = sorted((k for k, v in t.items() if v.get("packed_f32") or v.get("scratch")))
    print(f"{len(t)} kernels; packed-FP32 total {sum(v.get('packed_f32', 0) for v in t.values())}")
    for k, name in zip(rows, demangle(rows)):
        v = t[k]
        print(f"  pk {v.get('packed_f32', 0):4d}  scratch {v.get('scratch', 0):4d}  "
              f"mfma {v.get('mfma', 0):4d}  {name}")
