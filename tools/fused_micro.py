"""Fused gather + Linear1 (gine_mp_fwd_mlp1) against the unfused pair, HIP-graph replay.
    python tools/fused_micro.py [--configs 1,2,3] [--reps 50]
GINE_HIP_LIB selects an experiment build (make variant ... VDEFS=-DGINE_FUSED_DBG=1|2)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from raincast_gnn import _lib, functional as Fn  # noqa: E402
from raincast_gnn.graph import GineGraph  # noqa: E402
from helpers import knn_batch_graph  # noqa: E402
from mp_micro import CONFIGS, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rcm", action="store_true", help="stations in the locality order")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    D = 128
    for c in (int(v) for v in args.configs.split(",")):
        n, k, b = CONFIGS[c]
        ei, ea, N = knn_batch_graph(n, k, b, seed=0)
        if args.rcm:
            from raincast_gnn.data import relabel_edges, station_order
            ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // b], n))
        g = GineGraph(ei.to(dev), ea.to(dev), N)
        x = torch.randn(N, D, device=dev)
        lw, lb = torch.randn(D, device=dev), torch.randn(D, device=dev)
        eps = torch.tensor([0.1], device=dev)
        w1, b1 = torch.randn(D, D, device=dev) / 11, torch.randn(D, device=dev)
        z, a1 = torch.empty_like(x), torch.empty_like(x)
        P = Fn._count("gine_mlp_num_partials", N, D)
        part = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
        p = _lib.ptr

        def S():  # the current stream: the capture stream inside timed()
            return _lib.stream_handle(dev)

        def fused():
            _lib.call("gine_mp_fwd_mlp1", p(x), p(g.in_rowptr), p(g.in_src), p(g.in_attr),
                      p(lw), p(lb), p(eps), p(w1), p(b1), p(z), p(a1), p(part), N, D,
                      g.max_in_degree, 0, S())

        def mp():
            _lib.call("gine_mp_fwd", p(x), p(g.in_rowptr), p(g.in_src), p(g.in_attr), p(lw),
                      p(lb), p(eps), p(z), N, D, 0, S())

        def fwd1():
            _lib.call("gine_mlp_fwd1", p(z), p(w1), p(b1), p(a1), p(part), N, D, S())

        def pair():
            mp()
            fwd1()

        rec = {"cfg": c, "N": N, "E": int(ei.size(1)), "max_deg": g.max_in_degree}
        for name, fn in (("fused", fused), ("mp_fwd", mp), ("fwd1", fwd1), ("pair", pair)):
            if name == "fused" and g.max_in_degree > _lib.MP_FUSED_MAX_DEGREE:
                continue
            rec[name + "_us"] = round(timed(fn, args.reps), 3)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
