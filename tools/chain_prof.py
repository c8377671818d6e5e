"""Phase profile of the doubly folded chain kernels (k_chain F2D forward / B2D backward) at
cfg2's shape: every workgroup's s_memtime stamps (gine_chain.hip GINE_CHAIN_PROFILE).
    GINE_HIP_LIB=.../var/chainprof/libgine_hip.so python tools/chain_prof.py [--nodes 16000]
    python tools/chain_prof.py --no-stamps        # launch times of the shipped library"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402

NAMES = ["frags issued", "tile 1 staged", "tile 1 stage 1", "tile 1 sync", "tile 1 stage 2",
         "tile 2 staged", "tile 2 stage 1", "tile 2 sync", "tile 2 stage 2", "to end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16000)
    ap.add_argument("--F", type=int, default=35)
    ap.add_argument("--no-stamps", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, D, F = a.nodes, 128, a.F
    torch.manual_seed(0)
    r, dh0 = torch.randn(N, D, device=dev), torch.randn(N, D, device=dev)
    x = torch.randn(N, F, device=dev)
    wfold = torch.randn(2 * D * (F + D) + D, device=dev) / D ** 0.5
    wfold2 = torch.randn(D * D + D, device=dev) / D ** 0.5
    u, h0, dt, dr = (torch.empty(N, D, device=dev) for _ in range(4))
    P, st = _lib.ptr, _lib.stream_handle(dev)

    def fwd():
        _lib.call("gine_chain_fwd_folded2", P(r), P(x), P(wfold), P(wfold2), P(u), P(h0), N, D,
                  F, st)

    def bwd():
        _lib.call("gine_chain_bwd_folded2", P(dh0), P(u), P(wfold), P(wfold2), P(dt), P(dr), N,
                  D, F, st)

    for name, fn in (("forward (F2D)", fwd), ("backward (B2D)", bwd)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / 20 * 1e3:.2f} us per launch (20 back to back)")
        if a.no_stamps:
            continue
        lib = _lib.load()
        buf = (ctypes.c_longlong * (1024 * 16))()
        fn()
        torch.cuda.synchronize()
        lib.gine_debug_chain_prof(buf)
        t = np.frombuffer(buf, dtype=np.int64).reshape(1024, 16).astype(np.float64)
        live = (t[:, 11] > 0) & (t[:, 11] > t[:, 11].max() - 1e5)
        t = t[live]
        two = t[:, 9] > t[:, 5]
        rt = (t[:, 11:13] - t[:, 11].min()) * 10.0
        print(f"  {len(t)} workgroups ({int(two.sum())} with two tiles); realtime ns: entry "
              f"median {np.median(rt[:, 0]):.0f} max {rt[:, 0].max():.0f}; end median "
              f"{np.median(rt[:, 1]):.0f} max {rt[:, 1].max():.0f}")
        prev = 0
        for i, nm in enumerate(NAMES):
            j = i + 1
            sel = two if j >= 6 and j <= 9 else np.ones_like(two)
            if j == 10:
                d = t[:, 10] - np.where(two, t[:, 9], t[:, 5])
            else:
                d = t[sel, j] - t[sel, j - 1]
            print(f"    {nm:16s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f} ticks")


if __name__ == "__main__":
    main()
