"""What a BatchNorm finish launch costs inside a replayed graph: the layer's forward chain
(fused gather+Linear1, BN finish, Linear2) timed with and without the finish launch
(the latter reads a stale bn_save: timing only).
    python tools/bnfin_cost.py [--reps 50]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from raincast_gnn import _lib, functional as Fn  # noqa: E402
from raincast_gnn.graph import GineGraph  # noqa: E402
from helpers import knn_batch_graph  # noqa: E402
from mp_micro import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    D = 128
    ei, ea, N = knn_batch_graph(500, 10, 32, seed=0)
    g = GineGraph(ei.to(dev), ea.to(dev), N)
    x = torch.randn(N, D, device=dev)
    lw, lb, eps = torch.randn(D, device=dev), torch.randn(D, device=dev), torch.zeros(1, device=dev)
    w1, b1, w2, b2 = (torch.randn(D, D, device=dev) / 11, torch.randn(D, device=dev),
                      torch.randn(D, D, device=dev) / 11, torch.randn(D, device=dev))
    gamma, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    rm, rv = torch.zeros(D, device=dev), torch.ones(D, device=dev)
    z, a1, y = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    mask = torch.empty(N, D, dtype=torch.uint8, device=dev)
    P = Fn._count("gine_mlp_num_partials", N, D)
    part = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
    bn_save = torch.ones(4, D, device=dev)
    p = _lib.ptr

    def S():
        return _lib.stream_handle(dev)

    def fused():
        _lib.call("gine_mp_fwd_mlp1", p(x), p(g.in_rowptr), p(g.in_src), p(g.in_attr), p(lw),
                  p(lb), p(eps), p(w1), p(b1), p(z), p(a1), p(part), N, D, g.max_in_degree, 2,
                  S())

    def fin():
        _lib.call("gine_bn_fwd_finalize", p(part), P, p(gamma), p(beta), p(rm), p(rv), None,
                  p(bn_save), N, D, 0.1, 1e-5, 1, 0, S())

    def fwd2():
        _lib.call("gine_mlp_fwd2", p(a1), p(bn_save), p(w2), p(b2), p(x), p(y), p(mask), N, D,
                  2, S())

    t3 = timed(lambda: (fused(), fin(), fwd2()), a.reps)
    t2 = timed(lambda: (fused(), fwd2()), a.reps)
    tf = timed(fin, a.reps)
    print(f"fused+fin+fwd2 {t3:.2f} us   fused+fwd2 {t2:.2f} us   -> finish costs "
          f"{t3 - t2:.2f} us in the chain (alone, back to back: {tf:.2f} us)")


if __name__ == "__main__":
    main()
