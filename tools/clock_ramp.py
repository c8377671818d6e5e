"""The cfg2 step's time per block of 10 graph replays from right after capture until it is
steady: how long the GPU's clock takes to reach its training-steady state after the
bench's CPU-heavy preparation (the driver's 20-step line is timed inside that ramp).
    python tools/clock_ramp.py [--seconds 2] [--idle-ms 0]"""
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
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before the replays")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = BENCH_CONFIGS[2]
    tr = bench.Trainer(cfg, dev, 0, 1, cfg.graphs_per_gpu, "split", False, "locality")
    for _ in range(5):
        tr.eager_step()
    torch.cuda.synchronize()
    tr.capture()
    torch.cuda.synchronize()
    if a.idle_ms:
        time.sleep(a.idle_ms / 1e3)
    s = torch.cuda.current_stream(dev)
    t0 = time.perf_counter()
    rows = []
    while time.perf_counter() - t0 < a.seconds:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            tr.step()
        e1.record(s)
        e1.synchronize()
        rows.append((time.perf_counter() - t0, e0.elapsed_time(e1) / 10))
    for i, (t, ms) in enumerate(rows):
        if i < 40 or i % 20 == 0:
            print(f"block {i:4d}  t {t * 1e3:8.1f} ms  step {ms:.4f} ms")
    tail = sorted(ms for _, ms in rows[len(rows) // 2:])
    print(f"steady (median of the second half): {tail[len(tail) // 2]:.4f} ms; blocks {len(rows)}")


if __name__ == "__main__":
    main()
