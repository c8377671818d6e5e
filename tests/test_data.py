"""CPU: graph construction and batching conventions (utils/data.py:261-284, PyG collate)."""
import numpy as np
import torch

from raincast_gnn import data as D
from raincast_gnn.params import BENCH_CONFIGS, EXPERIMENTS


def test_radius_graph_layout():
    lat, lon = D.synthetic_stations(60, seed=3)
    dist = D.haversine_matrix(lat, lon)
    ei, ea = D.build_edge_index_and_attr(dist, 200.0)
    n = 60
    E = ei.size(1) - n
    src, dst = ei[0, :E].numpy(), ei[1, :E].numpy()
    assert np.all(src != dst)
    key = src * n + dst
    assert np.all(np.diff(key) > 0)                         # np.where row-major order
    assert torch.equal(ei[:, E:], torch.arange(n).repeat(2, 1))  # self-loops last
    assert torch.all(ea[E:] == 1.0)
    d = dist[src, dst]
    assert np.allclose(ea[:E, 0].numpy(), (d / d.max()) ** -1)
    assert ea.dtype == torch.float32 and ei.dtype == torch.int64
    assert ea[:E].min() >= 1.0
    # symmetric distances -> symmetric radius graph
    assert set(zip(src, dst)) == set(zip(dst, src))


def test_self_loop_only_config():
    """24h_normal_mixed uses max_dist=1 km: effectively a self-loop-only graph."""
    assert EXPERIMENTS["24h_normal_mixed"]["max_dist"] == 1
    ei, ea = D.station_graph(100, max_dist=1.0, seed=0)
    assert torch.equal(ei, torch.arange(100).repeat(2, 1))
    assert torch.all(ea == 1.0)


def test_knn_graph_layout():
    n, k = 120, 7
    ei, ea = D.station_graph(n, k=k, seed=1)
    E = n * k
    assert ei.size(1) == E + n
    indeg = torch.bincount(ei[1], minlength=n)
    assert torch.all(indeg == k + 1)
    src, dst = ei[0, :E].numpy(), ei[1, :E].numpy()
    assert np.all(np.diff(src * n + dst) > 0)
    lat, lon = D.synthetic_stations(n, seed=1)
    dist = D.haversine_matrix(lat, lon)
    for i in (0, 17, 119):
        nb = src[dst == i]
        order = np.argsort(np.where(np.arange(n) == i, np.inf, dist[i]), kind="stable")[:k]
        assert set(nb) == set(order)


def test_collate_block_diagonal():
    samples = D.synthetic_samples(50, 3, k=4, seed=2)
    b = D.collate(samples)
    assert b.num_graphs == 3 and b.num_nodes == 150
    E1 = samples[0].edge_index.size(1)
    for g in range(3):
        assert torch.equal(b.edge_index[:, g * E1:(g + 1) * E1], samples[g].edge_index + 50 * g)
    assert torch.equal(b.ptr, torch.tensor([0, 50, 100, 150]))
    assert torch.equal(b.batch, torch.arange(3).repeat_interleave(50))
    assert b.ensemble.shape == (150, D.NUM_MEMBERS, D.NUM_FEATURES)
    assert not torch.isnan(b.x).any()


def test_synthetic_targets():
    y = D.synthetic_targets(np.random.default_rng(0), 20000)
    nan = np.isnan(y)
    assert 0.005 < nan.mean() < 0.02
    zero = y[~nan] == np.float32(np.log(0.01))
    assert 0.55 < zero.mean() < 0.65


def test_bench_configs_shapes():
    c2 = BENCH_CONFIGS[2]
    assert (c2.num_stations, c2.k, c2.graphs_per_gpu) == (500, 10, 32)
    p = c2.params()
    assert p["gnn_hidden"] == 128 and p["gnn_layers"] == 4 and p["loss"] == "MixedLoss"
    assert BENCH_CONFIGS[5].params()["gnn_layers"] == 3
