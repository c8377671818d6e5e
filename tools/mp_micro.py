"""Message-passing microbenchmark: gather kernels vs LDS-staged window kernels.

Times gine_mp_fwd / gine_mp_bwd (and the *_win forms) standalone with HIP events on the
bench configurations' graphs, plus the algorithmic-bytes rate (B_f, B_b).
    python tools/mp_micro.py [--configs 1,2,3,5] [--tiles 128,64] [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from raincast_gnn import functional as Fn  # noqa: E402
from raincast_gnn import graph as G, options  # noqa: E402
from raincast_gnn.graph import GineGraph  # noqa: E402
from helpers import knn_batch_graph  # noqa: E402

CONFIGS = {1: (500, 10, 1), 2: (500, 10, 32), 3: (2000, 16, 64), 5: (10000, 32, 8)}


def morton_batch_graph(n, k, batch, seed=0):
    """knn_batch_graph with the stations renumbered along a Z-order curve of (lat, lon):
    graph neighbours become index neighbours (locality experiment)."""
    from raincast_gnn import data as rdata
    lat, lon = rdata.synthetic_stations(n, seed)
    qa = ((lat - 43.0) / 12.0 * 65535).astype(np.int64)
    qo = ((lon + 5.0) / 22.0 * 65535).astype(np.int64)
    key = np.zeros(n, dtype=np.int64)
    for b in range(16):
        key |= ((qa >> b) & 1) << (2 * b + 1) | ((qo >> b) & 1) << (2 * b)
    order = np.argsort(key, kind="stable")
    ei, ea = rdata.knn_edge_index_and_attr(rdata.haversine_matrix(lat[order], lon[order]), k)
    eis = [ei + g * n for g in range(batch)]
    return torch.cat(eis, 1), torch.cat([ea] * batch), n * batch


EAGER = False


def timed(fn, reps):
    if EAGER:  # counter collection: plain launches
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return float("nan")
    """Per-call time of `fn` replayed from a HIP graph of `reps` calls (no host overhead)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(5):
        graph.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / (5 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,5")
    ap.add_argument("--tiles", default="128,64,32")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--morton", action="store_true", help="Z-order station numbering")
    ap.add_argument("--rcm", action="store_true",
                    help="stations in the engine's locality order (reverse Cuthill-McKee, "
                         "raincast_gnn.data.station_order), as bench.py runs them")
    ap.add_argument("--slice", type=int, default=0, help="force a window slice width")
    ap.add_argument("--eager", action="store_true", help="no graphs (for rocprofv3 --pmc)")
    args = ap.parse_args()
    global EAGER
    EAGER = args.eager
    dev = torch.device("cuda:0")
    D = args.D
    out = []
    for c in (int(v) for v in args.configs.split(",")):
        n, k, B = CONFIGS[c]
        ei, ea, N = (morton_batch_graph if args.morton else knn_batch_graph)(n, k, B, seed=0)
        if args.rcm:
            from raincast_gnn.data import relabel_edges, station_order
            ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // B], n))
        E = ei.size(1)
        ei, ea = ei.to(dev), ea.to(dev)
        x = torch.randn(N, D, device=dev)
        dz = torch.randn(N, D, device=dev)
        dres = torch.randn(N, D, device=dev)
        lw, lb = torch.randn(D, device=dev), torch.randn(D, device=dev)
        eps = torch.tensor([0.1], device=dev)
        bf = 4 * (2 * N * D + 2 * E + N + 1)
        bb = 4 * (3 * N * D + 2 * E + N + 1)   # SURVEY 8(d) B_b
        variants = [("gather", "0", 128)] + [(f"win{t}", "all", t)
                                             for t in (int(v) for v in args.tiles.split(",") if v)]
        for name, on, tiles in variants:
            options.MP_WINDOW = on
            options.WINDOW_NODES = tiles
            if args.slice:
                G.WINDOW_SLICES = (args.slice,)
            g = GineGraph(ei, ea, N)
            plan = g.window_plan("in", D)
            if on == "all" and plan is None:
                print(f"cfg{c} {name}: no window plan", flush=True)
                continue
            tf = timed(lambda: Fn.mp_forward(x, g, lw, lb, eps), args.reps)
            # backward = the mp kernel + its fixed-order finalize (two launches)
            tb = timed(lambda: Fn.mp_backward(dz, x, g, lw, lb, eps, dres=dres), args.reps)
            rec = {"cfg": c, "variant": name, "N": N, "E": E, "fwd_us": round(tf, 3),
                   "bwd_us": round(tb, 3), "fwd_GBps": round(bf / tf / 1e3, 1),
                   "bwd_GBps": round(bb / tb / 1e3, 1),
                   "tiles": None if plan is None else int(plan.num_tiles),
                   "slice": None if plan is None else int(plan.slice_channels)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    return out


if __name__ == "__main__":
    main()
