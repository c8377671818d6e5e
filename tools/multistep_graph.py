"""What capturing S consecutive training steps in one HIP graph would buy (the replay boundary,
DESIGN.md §6): per-step GPU time of S-step graphs vs the one-step graph bench.py replays, and
the final loss after the same number of steps (the steps are the same work either way).
    python tools/multistep_graph.py [--config 2] [--steps 240] [--per-graph 1,2,4]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402


def run(cfg, dev, per_graph, steps):
    tr = bench.Trainer(cfg, dev, 0, 1, cfg.graphs_per_gpu)
    for _ in range(3):
        tr.eager_step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            loss = tr.fwd_bwd()
            tr.opt.step()
    assert tr.opt.views_intact()
    for _ in range(max(1, 300 // per_graph)):  # clock settle, as bench.py
        g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps // per_graph):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps, loss.item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--per-graph", default="1,2,4,1")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = BENCH_CONFIGS[a.config]
    for s in map(int, a.per_graph.split(",")):
        us, loss = run(cfg, dev, s, a.steps)
        print(f"{s} step(s) per graph: {us:.1f} us per step  "
              f"({cfg.graphs_per_gpu / us * 1e6:.0f} graphs/s), last loss {loss:.6f}", flush=True)


if __name__ == "__main__":
    main()
