"""Per-kernel floor of a dependent chain of tiny kernels on this GPU: eager launches vs one
HIP-graph replay, no profiler.  Tells how much of a training step is dispatch overhead.
    python tools/launch_floor.py [--kernels 100] [--reps 50]
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=100)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    small = torch.zeros(64, device=dev)
    big = torch.zeros(16000 * 128, device=dev)

    def chain(t):
        for _ in range(a.kernels):
            t.add_(1.0)

    for name, t in (("64 floats", small), ("16000x128 floats", big)):
        for _ in range(3):
            chain(t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            chain(t)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / (a.reps * a.kernels) * 1e6

        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain(t)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            chain(t)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / (a.reps * a.kernels) * 1e6
        print(f"{name}: eager {eager:.2f} us/kernel, graph replay {graph:.2f} us/kernel "
              f"({a.kernels} dependent kernels per chain)")

    # a tiny kernel right behind a bandwidth-heavy one (the finalize-after-GEMM pattern)
    def alt(n_tiny):
        for _ in range(a.kernels // 2):
            big.add_(1.0)
            for _ in range(n_tiny):
                small.add_(1.0)

    for n_tiny in (0, 1, 2):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            alt(n_tiny)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            alt(n_tiny)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        per_pair = (time.perf_counter() - t0) / (a.reps * (a.kernels // 2)) * 1e6
        print(f"graph: 1 big (16000x128 add) + {n_tiny} tiny kernels: {per_pair:.2f} us per group")


if __name__ == "__main__":
    main()
