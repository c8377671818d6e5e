"""Phase profile of the row-tile GEMM (workgroup 0's timeline, s_memtime cycles).
    GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/../csrc/build/dbg/libgine_hip_rgprof.so \\
        python tools/rg_prof.py [--nodes 16000]
Phases: 0 start -> 1 weights issued / tile top -> 2 tile staged -> 3 MFMA chain done ->
4 epilogue done (-> 1 next tile) -> 5 partials written."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "raincast-gnn_amd"))
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402
from raincast_gnn import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, D = a.nodes, 128
    lib = _lib.load()
    z = torch.randn(N, D, device=dev)
    x = torch.randn(N, D, device=dev)
    dy = torch.randn(N, D, device=dev)
    w1 = torch.randn(D, D, device=dev) / 11
    w2 = torch.randn(D, D, device=dev) / 11
    b1 = torch.randn(D, device=dev)
    b2 = torch.randn(D, device=dev)
    P = Fn._count("gine_mlp_num_partials", N, D)
    part = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
    a1, y, dbn, dz = (torch.empty_like(z) for _ in range(4))
    mask = torch.empty(N, D, dtype=torch.uint8, device=dev)
    bn_save = torch.ones(4, D, device=dev)
    coef = torch.ones(3, D, device=dev)
    s = _lib.stream_handle(dev)
    c, p = _lib.call, _lib.ptr
    kernels = {
        "fwd1": lambda: c("gine_mlp_fwd1", p(z), p(w1), p(b1), p(a1), p(part), N, D, s),
        "fwd2": lambda: c("gine_mlp_fwd2", p(a1), p(bn_save), p(w2), p(b2), p(x), p(y), p(mask),
                          N, D, 2, s),
        "bwd2": lambda: c("gine_mlp_bwd2", p(dy), None, p(mask), p(a1), p(bn_save), p(w2),
                          p(dbn), p(part), N, D, 2, s),
        "bwd1": lambda: c("gine_mlp_bwd1", p(dbn), p(a1), p(bn_save), p(coef), p(w1), p(dz), N,
                          D, s),
    }
    buf = (ctypes.c_longlong * 4096)()
    n = ctypes.c_int(0)
    names = {0: "start", 1: "tile top", 2: "staged", 3: "mfma done", 4: "epilogue done",
             5: "partials"}
    for name, fn in kernels.items():
        fn()
        lib.gine_debug_rg_prof(buf, ctypes.byref(n))  # reset
        for _ in range(4):  # back to back (warm clocks/caches); the last launch is read
            fn()
        lib.gine_debug_rg_prof(buf, ctypes.byref(n))
        ev = [(buf[2 * i], buf[2 * i + 1]) for i in range(n.value)]
        starts = [i for i, (tag, _) in enumerate(ev) if tag == 0]
        ev = ev[starts[-1]:]
        t0 = ev[0][1]
        line = " | ".join(f"{names[tag]} {t - t0}" for tag, t in ev)
        print(f"{name}: {line}")


if __name__ == "__main__":
    main()
