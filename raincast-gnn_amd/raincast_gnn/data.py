"""Station graphs and batches (host side, numpy/torch; cold path).

* :func:`build_edge_index_and_attr` -- the reference's radius graph, utils/data.py:261-284:
  edges (row -> col) where dist <= max_dist off the diagonal, in ``np.where`` (row-major)
  order, ``edge_attr = (dist / max_dist_over_edges) ** -1``, then N self-loops with
  attribute 1.0 appended at the end.
* :func:`knn_edge_index_and_attr` -- the synthetic k-NN variant used for the benchmark
  configs: for every station i its k nearest j != i (ties -> lower index)
  give edges j -> i; same ordering / attribute / self-loop conventions as above.
* :func:`collate` -- PyG ``Batch.from_data_list`` semantics (train.py:155-156): node tensors
  concatenated graph-major, graph g's edge_index offset by the nodes before it.
* :func:`synthetic_batch` -- a whole synthetic training batch of the 24h_mixed shape
  (35 features, 11 ensemble members, precipitation targets with NaNs).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

EARTH_RADIUS_KM = 6371.0088
NUM_FEATURES = 35      # utils/data.py:80-89 feature columns minus station_id/time/number
NUM_MEMBERS = 11       # reforecast ensemble members


def synthetic_stations(num_stations: int, seed: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Latitudes ~ U(43, 55), longitudes ~ U(-5, 17) (the EUPPBench domain)."""
    rng = np.random.default_rng(seed)
    lat = rng.uniform(43.0, 55.0, num_stations)
    lon = rng.uniform(-5.0, 17.0, num_stations)
    return lat, lon


def haversine_matrix(lat: np.ndarray, lon: np.ndarray) -> np.ndarray:
    """Pairwise great-circle distance (km) as float32 [N, N] (utils/data.py:248-259 uses
    geodesic distances; haversine stands in -- only the graph shape matters here)."""
    la, lo = np.radians(lat), np.radians(lon)
    dlat = la[:, None] - la[None, :]
    dlon = lo[:, None] - lo[None, :]
    a = np.sin(dlat / 2) ** 2 + np.cos(la)[:, None] * np.cos(la)[None, :] * np.sin(dlon / 2) ** 2
    d = 2 * EARTH_RADIUS_KM * np.arcsin(np.sqrt(np.clip(a, 0.0, 1.0)))
    np.fill_diagonal(d, 0.0)
    return d.astype(np.float32)


def _finish(row: np.ndarray, col: np.ndarray, dist_vals: np.ndarray, n: int):
    max_val = dist_vals.max() if dist_vals.size > 0 else 1.0
    inv_dist = (dist_vals / max_val) ** -1
    edge_index = torch.tensor(np.stack([row, col]), dtype=torch.long)
    edge_attr = torch.tensor(inv_dist, dtype=torch.float32).unsqueeze(-1)
    loops = torch.arange(n, dtype=torch.long).unsqueeze(0).repeat(2, 1)
    edge_index = torch.cat([edge_index, loops], dim=1)
    edge_attr = torch.cat([edge_attr, torch.ones((n, 1), dtype=torch.float32)], dim=0)
    return edge_index, edge_attr


def build_edge_index_and_attr(dist_mat: np.ndarray, max_dist: float):
    """Radius graph exactly as utils/data.py:261-284 builds it."""
    D = dist_mat.copy()
    np.fill_diagonal(D, np.inf)
    row, col = np.where(D <= max_dist)
    return _finish(row, col, D[row, col], dist_mat.shape[0])


def knn_edge_index_and_attr(dist_mat: np.ndarray, k: int):
    """k-NN graph in the reference's edge conventions (src = neighbour j, dst = station i)."""
    n = dist_mat.shape[0]
    D = dist_mat.astype(np.float32, copy=True)
    np.fill_diagonal(D, np.inf)
    kk = min(k, max(n - 1, 0))
    if kk == 0:
        empty = np.zeros(0, dtype=np.int64)
        return _finish(empty, empty, np.zeros(0, dtype=np.float32), n)
    nbr = np.argsort(D, axis=1, kind="stable")[:, :kk]           # ties -> lower index
    dst = np.repeat(np.arange(n, dtype=np.int64), kk)
    src = nbr.reshape(-1).astype(np.int64)
    order = np.lexsort((dst, src))                               # sorted by (src, dst)
    src, dst = src[order], dst[order]
    return _finish(src, dst, D[dst, src], n)


@dataclass
class GraphBatch:
    """The fields of a PyG ``Data``/``Batch`` the model reads (gnn.py:129-141, train.py:65)."""

    x: torch.Tensor
    ensemble: torch.Tensor
    edge_index: torch.Tensor
    edge_attr: torch.Tensor
    y: torch.Tensor
    batch: torch.Tensor | None = None
    ptr: torch.Tensor | None = None
    num_graphs: int = 1
    extra: dict = field(default_factory=dict)

    @property
    def num_nodes(self) -> int:
        return self.x.size(0)

    def to(self, device, non_blocking: bool = False) -> "GraphBatch":
        mv = lambda t: None if t is None else t.to(device, non_blocking=non_blocking)  # noqa: E731
        extra = {k: mv(v) if isinstance(v, torch.Tensor) else v for k, v in self.extra.items()}
        return GraphBatch(mv(self.x), mv(self.ensemble), mv(self.edge_index), mv(self.edge_attr),
                          mv(self.y), mv(self.batch), mv(self.ptr), self.num_graphs, extra)


def collate(graphs: list[GraphBatch]) -> GraphBatch:
    """Block-diagonal union (PyG Batch.from_data_list): graph-major node order."""
    offs, eis, counts = 0, [], []
    for g in graphs:
        eis.append(g.edge_index + offs)
        counts.append(g.num_nodes)
        offs += g.num_nodes
    counts_t = torch.tensor(counts, dtype=torch.long)
    batch = torch.repeat_interleave(torch.arange(len(graphs)), counts_t)
    ptr = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(counts_t, 0)])
    return GraphBatch(
        x=torch.cat([g.x for g in graphs]), ensemble=torch.cat([g.ensemble for g in graphs]),
        edge_index=torch.cat(eis, dim=1), edge_attr=torch.cat([g.edge_attr for g in graphs]),
        y=torch.cat([g.y for g in graphs]), batch=batch, ptr=ptr, num_graphs=len(graphs))


def synthetic_targets(rng: np.random.Generator, n: int, nan_frac: float = 0.01) -> np.ndarray:
    """y = log(r + 0.01): r = 0 w.p. 0.6 else Gamma(0.7, scale 3) mm; ``nan_frac`` missing."""
    r = np.where(rng.random(n) < 0.6, 0.0, rng.gamma(0.7, 3.0, n))
    y = np.log(r + 0.01).astype(np.float32)
    y[rng.random(n) < nan_frac] = np.nan
    return y


def station_graph(num_stations: int, k: int | None = 10, max_dist: float | None = None,
                  seed: int = 0):
    """edge_index / edge_attr of one synthetic station set (k-NN, or radius if max_dist)."""
    lat, lon = synthetic_stations(num_stations, seed)
    dist = haversine_matrix(lat, lon)
    if max_dist is not None:
        return build_edge_index_and_attr(dist, max_dist)
    return knn_edge_index_and_attr(dist, k)


def synthetic_samples(num_stations: int, num_graphs: int, k: int = 10, seed: int = 0,
                      in_channels: int = NUM_FEATURES, members: int = NUM_MEMBERS,
                      max_dist: float | None = None) -> list[GraphBatch]:
    """``num_graphs`` samples (times) sharing one static station graph (utils/data.py:300)."""
    edge_index, edge_attr = station_graph(num_stations, k, max_dist, seed)
    rng = np.random.default_rng(seed + 1)
    out = []
    for _ in range(num_graphs):
        x = torch.from_numpy(rng.standard_normal((num_stations, in_channels), dtype=np.float32))
        ens = torch.from_numpy(
            rng.standard_normal((num_stations, members, in_channels), dtype=np.float32))
        y = torch.from_numpy(synthetic_targets(rng, num_stations))
        out.append(GraphBatch(x, ens, edge_index, edge_attr, y))
    return out


def synthetic_batch(num_stations: int, num_graphs: int, k: int = 10, seed: int = 0,
                    **kw) -> GraphBatch:
    return collate(synthetic_samples(num_stations, num_graphs, k, seed, **kw))


# -----------------------------------------------------------------------------------------
# engine node order (station relabelling for neighbour locality)
# -----------------------------------------------------------------------------------------
def station_order(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Locality order of one station graph: ``order[i]`` = the station placed at position i
    (reverse Cuthill-McKee over the symmetrised edge list, ``gine_graph_order_locality`` in
    include/gine_hip.h; deterministic).  The reference's dataset order (utils/data.py:261-284)
    scatters each station's k nearest neighbours over the whole index range; in this order
    every edge stays within a short index band, so the window-staged message-passing tiles
    (raincast_gnn.graph.plan_windows) stage a fraction of the graph instead of all of it."""
    from . import _lib
    n = int(num_nodes)
    ei = edge_index.detach().to("cpu", torch.int64)
    if ei.dim() != 2 or ei.size(0) != 2:
        raise ValueError(f"edge_index must have shape [2, E], got {tuple(ei.shape)}")
    if ei.numel() and (int(ei.min()) < 0 or int(ei.max()) >= n):
        raise ValueError("edge_index holds node ids outside [0, num_nodes)")
    src, dst = ei[0], ei[1]
    rowptr = torch.zeros(n + 1, dtype=torch.int32)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=n), 0).to(torch.int32)
    nbr = src[torch.argsort(dst, stable=True)].to(torch.int32).contiguous()
    order = torch.empty(n, dtype=torch.int32)
    _lib.call("gine_graph_order_locality", rowptr.data_ptr(), nbr.data_ptr() if nbr.numel() else None,
              n, order.data_ptr())
    return order.to(torch.int64)


def inverse_order(order: torch.Tensor) -> torch.Tensor:
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel(), device=order.device, dtype=order.dtype)
    return inv


def block_node_order(order: torch.Tensor, num_graphs: int) -> torch.Tensor:
    """Row map of a batch of ``num_graphs`` graphs sharing one station order: row r of the
    relabelled batch is row ``block_node_order(...)[r]`` of the collated (reference) batch."""
    n = order.numel()
    offs = torch.arange(num_graphs, device=order.device, dtype=order.dtype) * n
    return (order.view(1, -1) + offs.view(-1, 1)).reshape(-1)


def relabel_edges(edge_index: torch.Tensor, order: torch.Tensor) -> torch.Tensor:
    """Node ids of a block-diagonal edge list (graphs of ``order.numel()`` stations each)
    mapped to the relabelled positions; the edge ORDER is kept, so every node's in- and
    out-edges stay in their original relative order -- the order CPU ``scatter_add_`` and
    ``index_add_`` accumulate in, hence bit-identical per-node z and dx."""
    n = order.numel()
    inv = inverse_order(order.to(edge_index.device))
    return inv[edge_index % n] + (edge_index // n) * n


def relabel_stations(batch: GraphBatch, order: torch.Tensor) -> GraphBatch:
    """``batch`` (B graphs of one station set, collated graph-major) in the engine's node
    order: the stations of every graph permuted by ``order`` and the edge list relabelled.
    Graph membership (``batch``/``ptr``) is unchanged; ``extra["node_order"]`` maps rows back
    (:func:`restore_node_order`).  Per-node model outputs are those of the reference order,
    only stored at other rows; reductions over nodes (BatchNorm statistics, the loss mean,
    parameter gradients) see the same terms in another order."""
    n, B = order.numel(), batch.num_graphs
    if batch.num_nodes != n * B:
        raise ValueError(f"batch of {batch.num_nodes} nodes is not {B} graphs x {n} stations")
    dev = batch.x.device
    rows = block_node_order(order.to(dev), B)
    extra = dict(batch.extra)
    prev = extra.get("node_order")
    extra["node_order"] = rows if prev is None else prev.to(dev)[rows]
    return GraphBatch(
        x=batch.x[rows], ensemble=batch.ensemble[rows],
        edge_index=relabel_edges(batch.edge_index, order), edge_attr=batch.edge_attr,
        y=batch.y[rows], batch=batch.batch, ptr=batch.ptr, num_graphs=B, extra=extra)


def restore_node_order(t: torch.Tensor, batch: GraphBatch) -> torch.Tensor:
    """Per-node rows of a relabelled batch's output back in the reference (collated) order."""
    rows = batch.extra.get("node_order")
    if rows is None:
        return t
    out = torch.empty_like(t)
    out[rows.to(t.device)] = t
    return out
