"""Diagnostic (CPU, no GPU): why full-size gradients cannot match at 1e-5.

Runs the CPU restatement of the reference's training step (oracle/, test infrastructure) at
a benchmark config in fp32 and in fp64 on the same weights and batch, and prints
* the distribution of the fp32 layer-input gradient's error against fp64, and
* how many ReLU decisions come out differently in fp32 and fp64 at the sites it can see
  (DeepSet phi[0], each GINE layer's edge message and outer ReLU).
A handful of decisions out of ~10^8 flip; each switches one gradient entry between 0 and
the upstream gradient, and message passing spreads it to the neighbours: the reference's
own fp32 gradient is then 1e-4..1e-2 away from the exact one (max-norm), which is why the
full-size parity tests use the reference's envelope (tests/helpers.py).
    python tools/relu_flips.py [cfg] [graphs]
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import gine_cpu as O  # noqa: E402
from raincast_gnn.data import synthetic_batch  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402


def main(cfg=2, graphs=None):
    c = BENCH_CONFIGS[cfg]
    p = c.params()
    graphs = graphs or c.graphs_per_gpu
    torch.manual_seed(42)
    ref = O.OracleGNN(35, p["gnn_hidden"], p["gnn_layers"], p["loss"], p["grad_u"], p["u"],
                      p["xi"])
    batch = synthetic_batch(c.num_stations, graphs, k=c.k, seed=100 + cfg)

    def cast(dt):
        r = copy.deepcopy(ref).to(dt)
        b = copy.copy(batch)
        b.x, b.ensemble, b.edge_attr = (t.to(dt) for t in (batch.x, batch.ensemble,
                                                           batch.edge_attr))
        return r, b

    def grad(dt):
        r, b = cast(dt)
        store = {}
        h = r.dim_red(torch.cat([b.x, r.deepset(b.ensemble)], 1))
        h.register_hook(lambda g: store.__setitem__("g", g.double()))
        x = h
        for i, conv in enumerate(r.conv.convolutions):
            y = torch.relu(conv(x, b.edge_index, b.edge_attr))
            x = y if i == 0 else x + y
        r.crps(O.postprocess(r.aggr(x), r.loss, r.grad_u), batch.y).backward()
        return store["g"]

    def acts(dt):
        r, b = cast(dt)
        out = []
        with torch.no_grad():
            out.append(("deepset phi[0]", r.deepset.phi[0](b.ensemble)))
            x = r.dim_red(torch.cat([b.x, r.deepset(b.ensemble)], 1))
            src = b.edge_index[0]
            for i, conv in enumerate(r.conv.convolutions):
                out.append((f"layer {i} edge message", x[src] + conv.lin(b.edge_attr)))
                cv = conv(x, b.edge_index, b.edge_attr)
                out.append((f"layer {i} outer ReLU", cv))
                y = torch.relu(cv)
                x = y if i == 0 else x + y
        return out

    print(f"{c.name} ({c.experiment}), {graphs} graphs x {c.num_stations} stations, "
          f"k={c.k}, {p['gnn_layers']} layers, {torch.get_num_threads()} threads")
    g32, g64 = grad(torch.float32), grad(torch.float64)
    e = ((g32 - g64).abs() / g64.abs().max()).flatten().numpy()
    print("fp32 oracle layer-0 input gradient vs fp64, |err| / max|g|: "
          + ", ".join(f"q{q}={np.quantile(e, q):.2e}" for q in (0.5, 0.99, 0.9999, 1.0)))
    print(f"  entries > 1e-5: {(e > 1e-5).sum()} / {e.size}")
    total = flipped = 0
    for (name, u), (_, v) in zip(acts(torch.float32), acts(torch.float64)):
        f = int(((u > 0) != (v > 0)).sum())
        total, flipped = total + u.numel(), flipped + f
        print(f"  {name:24s} {u.numel():>10d} ReLU decisions, {f} differ fp32 vs fp64")
    print(f"total: {flipped} of {total} decisions differ")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
