#!/usr/bin/env python3
"""bench.py with engine path selections overridden (raincast_gnn.options; the product path
reads no environment switches), for A/B runs on one box:
    python tools/bench_with.py ENGINE_IN_MP=0 MP_FUSED=0 -- --config 5 --steps 20 --no-cpu
    python tools/bench_with.py chain.FOLD2=0 -- --steps 50 --no-cpu   (module.NAME: that
    raincast_gnn module's switch)
Values: 0/1 for booleans, strings otherwise."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

from raincast_gnn import options  # noqa: E402

argv = sys.argv[1:]
split = argv.index("--") if "--" in argv else len(argv)
for kv in argv[:split]:
    k, v = kv.split("=", 1)
    mod = options
    if "." in k:
        m, k = k.rsplit(".", 1)
        mod = importlib.import_module(f"raincast_gnn.{m}")
    cur = getattr(mod, k)
    setattr(mod, k, (v not in ("0", "false", "False")) if isinstance(cur, bool)
            else type(cur)(v))
sys.argv = [os.path.join(ROOT, "bench.py")] + argv[split + 1:]
import bench  # noqa: E402

bench.main()
