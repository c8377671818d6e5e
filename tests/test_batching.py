"""Device-resident batching (raincast_gnn/batching.py) reproduces PyG collation exactly and
reuses one edge list per batch size (so the engine sorts it once per run)."""
import torch

from raincast_gnn.batching import DeviceDataset, DeviceLoader
from raincast_gnn.data import collate, synthetic_samples


def test_device_batch_equals_collate():
    samples = synthetic_samples(60, 9, k=5, seed=3)
    ds = DeviceDataset(samples, "cpu")
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
