"""Host issue time vs GPU time of the captured cfg2 training step: is the gap between two
replays (k_adamw end -> next step's first kernel, ≈8.8 µs in profiles/r06_s33's trace) the
host's replay call or the runtime's graph boundary?
    python tools/replay_gap.py [--config 2] [--reps 200]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = BENCH_CONFIGS[a.config]
    tr = bench.Trainer(cfg, dev, 0, 1, cfg.graphs_per_gpu)
    for _ in range(3):
        tr.eager_step()
    torch.cuda.synchronize()
    tr.capture()
    for _ in range(300):  # clock settle, as bench.py
        tr.step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for label in ("back to back", "one at a time"):
        host = []
        e0.record(s)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            h0 = time.perf_counter()
            tr.step()
            host.append(time.perf_counter() - h0)
            if label == "one at a time":
                torch.cuda.synchronize()
        e1.record(s)
        e1.synchronize()
        wall = time.perf_counter() - t0
        host.sort()
        print(f"{label}: GPU {e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us/step, wall "
              f"{wall * 1e6 / a.reps:.1f} us/step, host replay call p50 "
              f"{host[len(host) // 2] * 1e6:.1f} us p90 {host[int(0.9 * len(host))] * 1e6:.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
