"""The jobs of the end-of-backward gradient batch (gine_grad_finalize_batch) in one cfg2
training step, and the launch time of the batch and of each job alone (HIP events, the
buffers still alive: timed inside the flush that launches them).
    python tools/gradbatch_jobs.py [--config 2] [--reps 20]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from raincast_gnn import _lib  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = BENCH_CONFIGS[a.config]
    tr = bench.Trainer(cfg, dev, 0, 1, cfg.graphs_per_gpu)
    for _ in range(2):
        tr.eager_step()
    torch.cuda.synchronize()
    real = _lib.call
    seen = []

    def timed(fn):
        s = torch.cuda.current_stream(dev)
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            fn()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.reps

    def spy(name, *args):
        if name != "gine_grad_finalize_batch" or seen:
            return real(name, *args)
        arr, n, stream = args
        jobs = [arr[i] for i in range(n)]
        seen.append(1)
        real(name, *args)
        one = lambda j: (lambda: real(name, (_lib.GradJob * 1)(j), 1, stream))
        print(f"batch of {n} jobs: {timed(lambda: real(name, *args)):.2f} us", flush=True)
        for i, j in enumerate(jobs):
            kind = "mp" if j.kind == _lib.GRAD_JOB_MP else "slab"
            desc = (f"rows {j.rows} x 3*{j.channels} fp64" if kind == "mp" else
                    f"rows {j.rows} x per {[j.per[z] for z in range(j.nz)]} fp32, "
                    f"cstride {j.cstride}")
            mb = (j.rows * 3 * j.channels * 8 if kind == "mp" else
                  j.rows * sum(j.per[z] for z in range(j.nz)) * 4) / 1e6
            print(f"  job {i}: {kind:4s} {desc}  ({mb:.2f} MB)  alone {timed(one(j)):.2f} us",
                  flush=True)

    _lib.call = spy
    try:
        tr.eager_step()
        torch.cuda.synchronize()
    finally:
        _lib.call = real


if __name__ == "__main__":
    main()
