"""Device-resident batching (raincast_gnn/batching.py) reproduces PyG collation exactly and
reuses one edge list per batch size (so the engine sorts it once per run)."""
import torch

from raincast_gnn.batching import DeviceDataset, DeviceLoader
from raincast_gnn.data import (collate, relabel_stations, restore_node_order, station_order,
                               synthetic_samples)


def test_device_batch_equals_collate():
    samples = synthetic_samples(60, 9, k=5, seed=3)
    ds = DeviceDataset(samples, "cpu", relabel=False)
    idx = torch.tensor([4, 0, 7, 7, 2])
    got = ds.batch(idx)
    ref = collate([samples[i] for i in idx.tolist()])
    for name in ("x", "ensemble", "edge_index", "edge_attr", "batch", "ptr"):
        assert torch.equal(getattr(got, name), getattr(ref, name)), name
    assert torch.equal(got.y.isnan(), ref.y.isnan())
    assert torch.equal(torch.nan_to_num(got.y), torch.nan_to_num(ref.y))
    assert got.num_graphs == ref.num_graphs == 5


def test_edge_list_reused_per_batch_size_and_loader_covers_epoch():
    samples = synthetic_samples(30, 10, k=4, seed=1)
    ds = DeviceDataset(samples, "cpu")
    a = ds.batch(torch.tensor([0, 1, 2]))
    b = ds.batch(torch.tensor([5, 6, 7]))
    assert a.edge_index is b.edge_index and a.edge_attr is b.edge_attr
    loader = DeviceLoader(ds, batch_size=4, shuffle=True, seed=0)
    seen = []
    for batch in loader:
        seen.append(batch.num_graphs)
    assert seen == [4, 4, 2] and len(loader) == 3
    assert len(DeviceLoader(ds, 4, drop_last=True)) == 2


def test_relabelled_batch_maps_back_to_collate():
    """Default layout: stations in locality order; the row map restores the collated batch
    and the edge list is the collated one relabelled, edge order kept."""
    samples = synthetic_samples(60, 9, k=5, seed=3)
    ds = DeviceDataset(samples, "cpu")
    idx = torch.tensor([4, 0, 7, 7, 2])
    got = ds.batch(idx)
    ref = collate([samples[i] for i in idx.tolist()])
    rows = got.extra["node_order"]
    assert sorted(rows.tolist()) == list(range(ref.num_nodes))
    for name in ("x", "ensemble"):
        assert torch.equal(restore_node_order(getattr(got, name), got), getattr(ref, name))
    assert torch.equal(restore_node_order(got.y, got).isnan(), ref.y.isnan())
    assert torch.equal(rows[got.edge_index], ref.edge_index)
    assert torch.equal(got.edge_attr, ref.edge_attr)
    assert torch.equal(got.batch, ref.batch) and torch.equal(got.ptr, ref.ptr)
    # the same as relabelling the collated batch directly
    again = relabel_stations(ref, ds.order)
    assert torch.equal(again.x, got.x) and torch.equal(again.edge_index, got.edge_index)
    assert torch.equal(again.extra["node_order"], rows)


def test_station_order_narrows_the_edge_band():
    """Reverse Cuthill-McKee (gine_graph_order_locality): a permutation, deterministic,
    and every edge of a k-NN station graph within a short index band."""
    from raincast_gnn.data import station_graph
    for n, k in ((500, 10), (2000, 16)):
        ei, _ = station_graph(n, k)
        order = station_order(ei, n)
        assert sorted(order.tolist()) == list(range(n))
        assert torch.equal(order, station_order(ei, n))
        inv = torch.empty_like(order)
        inv[order] = torch.arange(n)
        band = (inv[ei[0]] - inv[ei[1]]).abs().max().item()
        assert band < n // 8, (n, band)
    # edge cases: no edges, a single station, self-loops only, two components
    assert station_order(torch.zeros(2, 0, dtype=torch.long), 3).tolist() == [2, 1, 0]
    assert station_order(torch.zeros(2, 1, dtype=torch.long), 1).tolist() == [0]
    two = torch.tensor([[0, 1, 3, 4], [1, 0, 4, 3]])
    o = station_order(two, 5)
    assert sorted(o.tolist()) == list(range(5))
