"""Generate tests/golden/gine_golden.npz: golden vectors of the GINE hot path.

    python tests/golden/make_gine_golden.py

torch_geometric is not importable here (no network), so these vectors come
from the CPU restatement of PyG's op sequence (oracle/gine_cpu.py) -- the GINE path stays
"parity unpinned" against the reference itself.  What they pin: the oracle against drift
(tests/test_golden.py recomputes them on CPU) and the HIP path against fixed numbers
(tests/test_gpu_golden.py), on the edge cases the reference can produce:
  (i)  message-passing forward z for both host roundings of the K=1 edge Linear
       (fma: MKL on Intel; muladd: MKL on AMD EPYC -- tools/probe_cpu_rounding.py)
  (ii) message-passing backward: dx (bit-exact per rounding) and dlin_w, dlin_b, deps in
       fp64
  (iii) one full GINE layer (GINEConv + Linear/BatchNorm1d(train)/ReLU/Linear, models/gnn.py
       :21-29) at D=128 on a 500-station k=10 graph, fp64 outputs and gradients.
Graph construction follows utils/data.py:261-284 (raincast_gnn.data).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]

from helpers import knn_batch_graph, radius_graph  # noqa: E402
from oracle import gine_cpu as O  # noqa: E402

OUT = os.path.join(HERE, "gine_golden.npz")


def mp_cases():
    """(name, edge_index, edge_attr, num_nodes, D)."""
    out = []
    ei, ea, n = knn_batch_graph(7, 1, 1, seed=11)
    out.append(("knn7_k1", ei, ea, n, 4))
    ei, ea, n = knn_batch_graph(64, 4, 3, seed=12)
    out.append(("knn64_k4_b3", ei, ea, n, 64))
    ei, ea, n = knn_batch_graph(500, 10, 1, seed=13)
    out.append(("knn500_k10", ei, ea, n, 128))
    ei, ea, n = radius_graph(50, 1.0, seed=14)          # max_dist=1: self-loops only
    out.append(("selfloops_only", ei, ea, n, 64))
    # node 3 receives nothing and sends nothing; node 5 only sends
    ei = torch.tensor([[0, 1, 2, 5, 5, 0, 1, 2, 4], [1, 2, 0, 0, 4, 0, 1, 2, 4]])
    ea = torch.linspace(0.5, 2.5, ei.size(1)).reshape(-1, 1)
    out.append(("isolated_node", ei, ea, 6, 4))
    out.append(("no_edges", torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, 1), 7, 4))
    return out


def lin_rounded(a, w, b, rounding):
    """Linear(1, D)(a) with the host rounding made explicit (a [E,1], w [D,1], b [D])."""
    if rounding == "fma":
        return (a.double() @ w.double().T + b.double()).float()
    return a * w.reshape(1, -1) + b


def aggregate_rounded(x, ei, ea, w, b, eps, rounding):
    """oracle.gine_aggregate with the edge Linear's rounding fixed (differentiable in x)."""
    src, dst = ei[0], ei[1]
    m = (x.index_select(0, src) + lin_rounded(ea.reshape(-1, 1), w, b, rounding)).relu()
    agg = x.new_zeros(x.size(0), m.size(1)).scatter_add_(0, dst.view(-1, 1).expand_as(m), m)
    return agg + (1 + eps) * x


def make_mp(arrays):
    for i, (name, ei, ea, n, D) in enumerate(mp_cases()):
        g = torch.Generator().manual_seed(100 + i)
        x = torch.randn(n, D, generator=g)
        w = torch.randn(D, 1, generator=g) * 0.5
        b = torch.randn(D, generator=g) * 0.5
        eps = torch.tensor([0.1 * (i + 1)])
        dz = torch.randn(n, D, generator=g)
        p = f"mp/{name}/"
        arrays.update({p + "x": x, p + "edge_index": ei, p + "edge_attr": ea, p + "lin_w": w,
                       p + "lin_b": b, p + "eps": eps, p + "dz": dz})
        for rounding in ("fma", "muladd"):
            xr = x.clone().requires_grad_(True)
            z = aggregate_rounded(xr, ei, ea, w, b, eps, rounding)
            z.backward(dz)
            arrays[p + f"z_{rounding}"] = z.detach()
            arrays[p + f"dx_{rounding}"] = xr.grad
        # parameter gradients in fp64 (reductions: compared at fp32 tolerance)
        w64, b64, e64 = (t.double().requires_grad_(True) for t in (w, b, eps))
        O.gine_aggregate(x.double(), ei, ea.double(), w64, b64, e64).backward(dz.double())
        arrays[p + "dlin_w64"] = w64.grad.reshape(-1)
        arrays[p + "dlin_b64"] = b64.grad
        arrays[p + "deps64"] = e64.grad


def make_layer(arrays):
    ei, ea, n = knn_batch_graph(500, 10, 1, seed=21)
    D = 128
    torch.manual_seed(22)
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = O.OracleGINEConv(mlp, train_eps=True, edge_dim=1)
    conv.eps.data.fill_(0.15)
    conv = conv.double().train()
    g = torch.Generator().manual_seed(23)
    x = torch.randn(n, D, generator=g).double()    # fp32 values, exact in fp64
    dy = torch.randn(n, D, generator=g).double()
    p = "layer/"
    for k, v in conv.state_dict().items():  # the state BEFORE the training-mode forward
        if v.dtype == torch.float64:
            arrays[p + "param/" + k] = v.float().clone()
    xr = x.clone().requires_grad_(True)
    y = conv(xr, ei, ea.double())
    y.backward(dy)
    arrays.update({p + "x": x.float(), p + "edge_index": ei, p + "edge_attr": ea,
                   p + "dy": dy.float(), p + "y64": y.detach(), p + "dx64": xr.grad})
    for k, prm in conv.named_parameters():
        arrays[p + "grad64/" + k] = prm.grad
    bn = conv.nn[1]
    arrays[p + "running_mean64"] = bn.running_mean.clone()
    arrays[p + "running_var64"] = bn.running_var.clone()


def main():
    arrays = {}
    make_mp(arrays)
    make_layer(arrays)
    np.savez_compressed(OUT, **{k: v.detach().numpy() for k, v in arrays.items()})
    print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
