#!/usr/bin/env python3
"""bench.py with engine path selections overridden (raincast_gnn.options; the product path
reads no environment switches), for A/B runs on one box:
    python tools/bench_with.py ENGINE_IN_MP=0 MP_FUSED=0 -- --config 5 --steps 20 --no-cpu
Values: 0/1 for booleans, strings otherwise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

from raincast_gnn import options  # noqa: E402

argv = sys.argv[1:]
split = argv.index("--") if "--" in argv else len(argv)
for kv in argv[:split]:
    k, v = kv.split("=", 1)
    cur = getattr(options, k)
    setattr(options, k, (v not in ("0", "false", "False")) if isinstance(cur, bool)
            else type(cur)(v))
sys.argv = [os.path.join(ROOT, "bench.py")] + argv[split + 1:]
import bench  # noqa: E402

bench.main()
