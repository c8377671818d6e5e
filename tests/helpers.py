"""Shared graph builders and comparison helpers for the test-suite."""
from __future__ import annotations

import numpy as np
import torch

from raincast_gnn import data as rdata


def knn_batch_graph(n: int, k: int, batch: int = 1, seed: int = 0):
    ei, ea = rdata.station_graph(n, k=k, seed=seed)
    eis = [ei + g * n for g in range(batch)]
    return torch.cat(eis, 1), torch.cat([ea] * batch), n * batch


def radius_graph(n: int, max_dist: float, seed: int = 0):
    lat, lon = rdata.synthetic_stations(n, seed)
    ei, ea = rdata.build_edge_index_and_attr(rdata.haversine_matrix(lat, lon), max_dist)
    return ei, ea, n


def random_graph(n: int, e: int, seed: int = 0, skew: bool = True):
    """Unsorted multigraph with hub sources (power-law out-degree) and isolated nodes."""
    rng = np.random.default_rng(seed)
    if skew:
        w = 1.0 / np.arange(1, n + 1) ** 1.2
        src = rng.choice(n, size=e, p=w / w.sum())
    else:
        src = rng.integers(0, n, e)
    dst = rng.integers(0, max(n - 2, 1), e)  # last nodes never receive: isolated targets
    ei = torch.tensor(np.stack([src, dst]), dtype=torch.long)
    ea = torch.from_numpy(rng.uniform(0.5, 4.0, (e, 1)).astype(np.float32))
    return ei, ea, n


def special_graphs():
    """(name, edge_index, edge_attr, num_nodes) edge cases the reference can produce."""
    out = []
    ei, ea, n = knn_batch_graph(64, 4, 1, seed=3)
    out.append(("knn64_k4", ei, ea, n))
    ei, ea, n = knn_batch_graph(500, 10, 2, seed=0)
    out.append(("knn500_k10_b2", ei, ea, n))
    # max_dist=1 (trained_models/24h_normal_mixed/params.json:6): self-loops only
    ei, ea, n = radius_graph(50, 1.0, seed=1)
    out.append(("selfloops_only", ei, ea, n))
    ei, ea, n = radius_graph(80, 150.0, seed=2)
    out.append(("radius80_150km", ei, ea, n))
    out.append(("no_edges", torch.zeros(2, 0, dtype=torch.long), torch.zeros(0, 1), 7))
    ei, ea, n = random_graph(200, 3000, seed=4)
    out.append(("hubs_unsorted", ei, ea, n))
    ei, ea, n = random_graph(1, 5, seed=5, skew=False)
    out.append(("single_node_multi_loops", torch.zeros(2, 5, dtype=torch.long), ea, 1))
    return out


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.abs().max().item()
    num = (a - b).abs().max().item()
    if den == 0.0:
        return num
    return num / den


def assert_close_tiebreak(gpu, cpu32, cpu64, tol=1e-5, name=""):
    """GPU vs CPU fp32 oracle within ``tol`` (max-norm relative); if not, the GPU must be at
    least as close to the fp64 oracle as the fp32 CPU oracle is (x2 slack)."""
    e32 = rel_err(gpu, cpu32)
    if e32 <= tol:
        return e32
    e_gpu = rel_err(gpu, cpu64)
    e_cpu = rel_err(cpu32, cpu64)
    assert e_gpu <= max(tol, 2.0 * e_cpu), (
        f"{name}: rel err vs cpu32 {e32:.3e}, gpu vs fp64 {e_gpu:.3e}, cpu32 vs fp64 {e_cpu:.3e}")
    return e32
