"""Host-side cost of the drop-in GINE stack (bench.py --dropin's gine_step: 4 GINEConv +
torch ReLU / residual, forward + backward, a fresh device edge_index each step): wall time
per step, the time the host spends issuing it (no synchronisation inside the loop except the
graph cache's content check), and a cProfile of the issuing side.
    python tools/dropin_prof.py [--steps 50] [--same-edges]"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

import torch  # noqa: E402

from raincast_gnn.data import collate, synthetic_samples  # noqa: E402
from raincast_gnn.dropin import reference_struct_from_params  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--same-edges", action="store_true",
                    help="pass the same device edge_index every step (identity hits)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = BENCH_CONFIGS[2]
    params = cfg.params()
    torch.manual_seed(42)
    model = reference_struct_from_params(params).to(dev).train()
    host = collate(synthetic_samples(cfg.num_stations, cfg.graphs_per_gpu, k=cfg.k, seed=1000))
    D = params["gnn_hidden"]
    x0 = torch.randn(host.num_nodes, D, device=dev, requires_grad=True)
    gy = torch.randn(host.num_nodes, D, device=dev)
    ei_dev, ea_dev = host.edge_index.to(dev), host.edge_attr.to(dev)

    def step():
        ei = ei_dev if a.same_edges else host.edge_index.to(dev)
        ea = ea_dev if a.same_edges else host.edge_attr.to(dev)
        out = model.conv(x0, ei, ea)
        out.backward(gy)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print(f"steps {a.steps}: wall {t_wall / a.steps * 1e3:.3f} ms/step, host issue "
          f"{t_issue / a.steps * 1e3:.3f} ms/step (same_edges={a.same_edges})")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
