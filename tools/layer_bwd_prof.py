"""Phase profile of the one-launch node-MLP backward (gine_mlp_bwd_layer) at cfg2 size.
    GINE_HIP_LIB=.../var/layerbwdprof/libgine_hip.so python tools/layer_bwd_prof.py
Thread 0's stamps per workgroup (csrc/gine_mlpbwd.hip GINE_LAYER_PROFILE), shader-clock ticks
after the workgroup's entry (median / p90 over workgroups), and the 100 MHz realtime clock
every XCD shares for entry / arrival / release / end across workgroups."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402
from raincast_gnn import functional as Fn  # noqa: E402
from test_gpu_layer_bwd import _inputs, _run, DEV, D  # noqa: E402

NAMES = {1: "tiles staged", 2: "W2 planes", 3: "tile 1 done", 4: "tile 2 done",
         5: "sums in acc", 6: "barrier passed", 7: "W1 planes", 8: "totals read",
         9: "coef ready", 10: "da1 staged", 11: "end"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16000)
    a = ap.parse_args()
    N = a.nodes
    t = _inputs(N, seed=1)
    acc = torch.zeros(Fn._count64("gine_bn_acc_words", D), dtype=torch.int64, device=DEV)
    lib = _lib.load()
    stamps = hasattr(lib, "gine_debug_bwd_layer_prof")
    buf = (ctypes.c_longlong * (1024 * 24))()
    for _ in range(5):
        _run("layer", t, acc, N, 2)
    torch.cuda.synchronize()
    if stamps:
        lib.gine_debug_bwd_layer_prof(buf)
        full = np.frombuffer(buf, dtype=np.int64).reshape(1024, 24).astype(np.float64)
        live = (full[:, 16] > 0) & (full[:, 16] > full[:, 16].max() - 1e5)
        full = full[live]
        print(f"N={N}: {len(full)} workgroups; ticks after entry (median / p90)")
        for i, nm in NAMES.items():
            d = full[:, i] - full[:, 0]
            print(f"  {nm:15s} {np.median(d):8.0f} {np.percentile(d, 90):8.0f}")
        rt = (full[:, 16:20] - full[:, 16].min()) * 10.0
        print(f"  realtime ns: entry median {np.median(rt[:, 0]):.0f} max {rt[:, 0].max():.0f}; "
              f"arrival median {np.median(rt[:, 1]):.0f} max {rt[:, 1].max():.0f}; release "
              f"min {rt[:, 2].min():.0f} max {rt[:, 2].max():.0f}; end median "
              f"{np.median(rt[:, 3]):.0f} max {rt[:, 3].max():.0f}")
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
        _run("layer", t, acc, N, 2)
    en.record()
    torch.cuda.synchronize()
    print(f"  launch time (HIP events, 20 back to back, with allocations): "
          f"{st.elapsed_time(en) / 20 * 1e3:.2f} us")


if __name__ == "__main__":
    main()
