"""Device-resident dataset and batching for a static station graph.

The reference builds ONE edge list per station set and shares it by every sample
(utils/data.py:300, 330-335); PyG's DataLoader then collates each batch on the host
(train.py:155-156: ``Batch.from_data_list``) and ``batch.to(device)`` copies it, edge_index
included, every step (train.py:62).  Here the samples live in HBM as stacked tensors
([T, N, F] features, [T, N, M, F] ensemble, [T, N] targets) and a batch is a device gather
by sample index.  The block-diagonal edge list of a batch of B graphs depends only on B,
so it is built once per B and the SAME tensor object is returned for every batch of that
size: the engine's graph cache (raincast_gnn/graph.py, keyed on tensor identity) then
sorts it into its two CSRs once for the whole run instead of once per step.

With ``relabel=False`` node order, edge order and attributes are exactly PyG collation's
(tests/test_batching.py compares with :func:`raincast_gnn.data.collate`).  By default the
stations are stored in the engine's locality order (:func:`raincast_gnn.data.station_order`,
reverse Cuthill-McKee): every graph of a batch has its stations permuted the same way and
the edge list relabelled with its edge order kept, so each node's result is the one the
reference order gives (bit for bit through the message passing), stored at another row;
``batch.extra["node_order"]`` maps the rows back (:func:`raincast_gnn.data.restore_node_order`).
"""
from __future__ import annotations

import torch

from .data import GraphBatch, block_node_order, relabel_edges, station_order


class DeviceDataset:
    """Samples of one station graph, stacked on ``device``."""

    def __init__(self, samples: list[GraphBatch], device, relabel: bool = True):
        if not samples:
            raise ValueError("empty dataset")
        base = samples[0]
        for s in samples:
            if s.edge_index is not base.edge_index and not torch.equal(s.edge_index,
                                                                      base.edge_index):
                raise ValueError("all samples must share one station graph (utils/data.py:300)")
        self.device = torch.device(device)
        self.num_stations = base.num_nodes
        self.x = torch.stack([s.x for s in samples]).to(self.device)
        self.ensemble = torch.stack([s.ensemble for s in samples]).to(self.device)
        self.y = torch.stack([s.y for s in samples]).to(self.device)
        self.edge_index = base.edge_index.to(self.device)
        self.edge_attr = base.edge_attr.to(self.device)
        self.order = None   # station at each stored position (None: the dataset's order)
        if relabel and self.num_stations > 1:
            order = station_order(base.edge_index, self.num_stations).to(self.device)
            self.order = order
            self.x = self.x.index_select(1, order)
            self.ensemble = self.ensemble.index_select(1, order)
            self.y = self.y.index_select(1, order)
            self.edge_index = relabel_edges(self.edge_index, order)
        self._blocks: dict[int, tuple] = {}

    def __len__(self) -> int:
        return self.x.size(0)

    def subset(self, indices) -> "DeviceDataset":
        """The samples ``indices`` (any order) as a dataset sharing this one's graph
        (``torch.utils.data.Subset`` after ``random_split``, train.py:150)."""
        idx = torch.as_tensor(indices, dtype=torch.long).to(self.device)
        out = DeviceDataset.__new__(DeviceDataset)
        out.device, out.num_stations = self.device, self.num_stations
        out.x = self.x.index_select(0, idx)
        out.ensemble = self.ensemble.index_select(0, idx)
        out.y = self.y.index_select(0, idx)
        out.edge_index, out.edge_attr, out.order = self.edge_index, self.edge_attr, self.order
        out._blocks = self._blocks   # same station graph: share the per-size edge lists
        return out

    def block_graph(self, num_graphs: int):
        """(edge_index, edge_attr, batch, ptr, node_order) of ``num_graphs`` copies of the
        station graph, built once per size and returned as the same tensors afterwards
        (node_order: row map back to the collated order, None without relabelling)."""
        hit = self._blocks.get(num_graphs)
        if hit is None:
            n, E = self.num_stations, self.edge_index.size(1)
            offs = (torch.arange(num_graphs, device=self.device, dtype=torch.long) * n)
            ei = (self.edge_index.unsqueeze(1) + offs.view(1, -1, 1)).reshape(2, num_graphs * E)
            ea = self.edge_attr.repeat(num_graphs, 1)
            batch = torch.arange(num_graphs, device=self.device).repeat_interleave(n)
            ptr = torch.arange(num_graphs + 1, device=self.device, dtype=torch.long) * n
            rows = block_node_order(self.order, num_graphs) if self.order is not None else None
            hit = (ei.contiguous(), ea.contiguous(), batch, ptr, rows)
            self._blocks[num_graphs] = hit
        return hit

    def batch(self, indices: torch.Tensor) -> GraphBatch:
        """The collated batch of samples ``indices`` (a device or host LongTensor)."""
        idx = indices.to(self.device, dtype=torch.long)
        B, n = idx.numel(), self.num_stations
        ei, ea, batch, ptr, rows = self.block_graph(B)
        F = self.x.size(-1)
        extra = {} if rows is None else {"node_order": rows}
        return GraphBatch(
            x=self.x.index_select(0, idx).reshape(B * n, F),
            ensemble=self.ensemble.index_select(0, idx).reshape(B * n, *self.ensemble.shape[2:]),
            edge_index=ei, edge_attr=ea,
            y=self.y.index_select(0, idx).reshape(B * n),
            batch=batch, ptr=ptr, num_graphs=B, extra=extra)


class DeviceLoader:
    """Epoch iterator over a :class:`DeviceDataset` (train.py:155-156: ``shuffle=True``,
    ``batch_size`` from params.json).  The permutation is drawn from a seeded CPU generator
    (``torch.randperm``, as PyG's DataLoader's RandomSampler does), so the batch order is the
    same whatever the dataset's device.  With ``world > 1`` every rank walks the same global
    batches and yields its contiguous shard of graphs (:func:`~raincast_gnn.distributed.
    shard_range`).  ``batch_size`` must then be a multiple of ``world``, so every full batch
    gives every rank the same number of graphs and the equal-weight gradient average (DDP's
    semantics) is the mean of equal shards; only a short last batch can split unevenly, and
    one with fewer graphs than ranks is skipped by all."""

    def __init__(self, dataset: DeviceDataset, batch_size: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False, rank: int = 0, world: int = 1):
        self.dataset, self.batch_size = dataset, int(batch_size)
        self.shuffle, self.drop_last = shuffle, drop_last
        self.rank, self.world = int(rank), int(world)
        if self.world > 1 and self.batch_size % self.world != 0:
            raise ValueError(f"batch_size {self.batch_size} is not a multiple of the {self.world} "
                             f"data-parallel ranks: shards would be unequal in every step")
        self._gen = torch.Generator()
        self._gen.manual_seed(seed)

    def __len__(self) -> int:
        T = len(self.dataset)
        return T // self.batch_size if self.drop_last else -(-T // self.batch_size)

    def __iter__(self):
        from .distributed import shard_range
        T = len(self.dataset)
        order = torch.randperm(T, generator=self._gen) if self.shuffle else torch.arange(T)
        for i in range(0, T, self.batch_size):
            idx = order[i:i + self.batch_size]
            if self.drop_last and idx.numel() < self.batch_size:
                return
            if self.world > 1:
                if idx.numel() < self.world:  # some rank would get no graph: every rank
                    continue                  # skips it (they all see the same order)
                lo, hi = shard_range(idx.numel(), self.rank, self.world)
                idx = idx[lo:hi]
            yield self.dataset.batch(idx)
