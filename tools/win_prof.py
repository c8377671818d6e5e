"""Phase profile of the window message-passing backward (every workgroup's s_memtime stamps).
    GINE_HIP_LIB=.../libgine_hip_winprof.so python tools/win_prof.py [--config 2]
Phases per workgroup: 0 entry -> 1 own rows issued -> 2 window staged (barrier) -> 3 edges
done (barrier) -> 4 block reduction -> 5 partials written."""
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
from raincast_gnn.graph import GineGraph  # noqa: E402
from helpers import knn_batch_graph  # noqa: E402

CONFIGS = {2: (500, 10, 32), 3: (2000, 16, 64), 5: (10000, 32, 8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    D = 128
    n, k, B = CONFIGS[a.config]
    ei, ea, N = knn_batch_graph(n, k, B, seed=0)
    from raincast_gnn.data import relabel_edges, station_order
    ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // B], n))
    ei, ea = ei.to(dev), ea.to(dev)
    x, dz, dres = (torch.randn(N, D, device=dev) for _ in range(3))
    lw, lb = torch.randn(D, device=dev), torch.randn(D, device=dev)
    eps = torch.tensor([0.1], device=dev)
    g = GineGraph(ei, ea, N)
    plan = g.window_plan("out", D)
    assert plan is not None, "no window plan"
    nb = int(plan.num_tiles) * (D // int(plan.slice_channels))
    lib = _lib.load()
    buf = (ctypes.c_longlong * (4096 * 8))()
    for _ in range(5):
        Fn.mp_backward(dz, x, g, lw, lb, eps, dres=dres)
    torch.cuda.synchronize()
    lib.gine_debug_win_prof(buf)
    t = np.frombuffer(buf, dtype=np.int64).reshape(4096, 8)[:min(nb, 4096), :6].astype(np.float64)
    t0 = t[:, 0].min()
    rel = t - t0
    ph = np.diff(t, axis=1)
    names = ["rows issued", "staged", "edges", "reduce", "write"]
    print(f"cfg{a.config}: {nb} workgroups, tiles {int(plan.num_tiles)}, slice "
          f"{int(plan.slice_channels)}; s_memtime ticks")
    print(f"  span entry->last end {rel[:, 5].max():.0f}; entry spread: median "
          f"{np.median(rel[:, 0]):.0f} max {rel[:, 0].max():.0f}")
    for i, nm in enumerate(names):
        print(f"  {nm:12s} median {np.median(ph[:, i]):8.0f}  p90 {np.percentile(ph[:, i], 90):8.0f}"
              f"  max {ph[:, i].max():8.0f}")
    print(f"  whole block  median {np.median(t[:, 5] - t[:, 0]):8.0f}  max "
          f"{(t[:, 5] - t[:, 0]).max():8.0f}")


if __name__ == "__main__":
    main()
