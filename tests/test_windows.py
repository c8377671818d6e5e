"""CPU: the window planner of the LDS-staged message passing (gine_graph_plan_windows).

The planner is host code of the C-ABI library (no device), so it runs here.  Checked: the
tiles partition the nodes in order, every node's neighbours lie inside its tile's window,
the size limits hold, graph boundaries of a PyG batch are never straddled, and graphs whose
nodes reach too far get no plan (the gather kernels take them).
"""
import ctypes

import numpy as np
import pytest
import torch

from helpers import knn_batch_graph, random_graph
from raincast_gnn import _lib


def csr(ei: torch.Tensor, n: int, key: int):
    """Stable CSR of edge_index by row `key` (1: in-edges by destination, 0: out-edges)."""
    k = ei[key].numpy()
    other = ei[1 - key].numpy()
    perm = np.argsort(k, kind="stable")
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(k, minlength=n))]).astype(np.int32)
    return rowptr, other[perm].astype(np.int32)


def plan(rowptr, nbr, n, max_rows, max_nodes, max_edges):
    tb = np.empty(n + 1, np.int32)
    lo = np.empty(max(n, 1), np.int32)
    rows = np.empty(max(n, 1), np.int32)
    maxima = np.zeros(3, np.int32)
    nt = ctypes.c_int32(-1)
    nbr = nbr if nbr.size else np.zeros(1, np.int32)
    _lib.call("gine_graph_plan_windows", rowptr.ctypes.data, nbr.ctypes.data, n, max_rows,
              max_nodes, max_edges, tb.ctypes.data, lo.ctypes.data, rows.ctypes.data,
              ctypes.byref(nt), maxima.ctypes.data)
    T = nt.value
    return T, tb[:T + 1], lo[:T], rows[:T], maxima


def check_plan(rowptr, nbr, n, T, tb, lo, rows, maxima, max_rows, max_nodes, max_edges):
    assert T > 0
    assert tb[0] == 0 and tb[-1] == n and np.all(np.diff(tb) > 0)
    assert np.all(np.diff(tb) <= max_nodes)
    assert np.all(rows <= max_rows) and maxima[0] == rows.max()
    tile_edges = rowptr[tb[1:]] - rowptr[tb[:-1]]
    assert np.all(tile_edges <= max_edges) and maxima[1] == tile_edges.max()
    assert maxima[2] == np.diff(tb).max()
    for t in range(T):
        seg = nbr[rowptr[tb[t]]:rowptr[tb[t + 1]]]
        if seg.size:
            assert lo[t] == seg.min() and lo[t] + rows[t] - 1 == seg.max()
        else:
            assert rows[t] == 0


@pytest.mark.parametrize("key", [1, 0])
def test_plan_batched_knn_aligns_with_graphs(key):
    ei, ea, n = knn_batch_graph(500, 10, 6, seed=0)
    rowptr, nbr = csr(ei, n, key)
    T, tb, lo, rows, mx = plan(rowptr, nbr, n, 512, 128, 1900)
    check_plan(rowptr, nbr, n, T, tb, lo, rows, mx, 512, 128, 1900)
    assert T == 6 * 4  # 128 + 128 + 128 + 116 nodes per 500-node graph
    graph_of_tile = tb[:-1] // 500
    assert np.all((tb[1:] - 1) // 500 == graph_of_tile)      # no tile straddles graphs
    assert np.all(lo // 500 == graph_of_tile)                 # windows inside the graph
    assert np.all((lo + rows - 1) // 500 == graph_of_tile)


@pytest.mark.parametrize("max_nodes,max_rows,max_edges", [(8, 256, 64), (64, 200, 4000),
                                                          (1, 200, 5000)])
def test_plan_random_multigraph(max_nodes, max_rows, max_edges):
    ei, ea, n = random_graph(200, 3000, seed=4)
    for key in (1, 0):
        rowptr, nbr = csr(ei, n, key)
        T, tb, lo, rows, mx = plan(rowptr, nbr, n, max_rows, max_nodes, max_edges)
        deg = np.diff(rowptr)
        if deg.max() > max_edges:
            assert T == 0
            continue
        check_plan(rowptr, nbr, n, T, tb, lo, rows, mx, max_rows, max_nodes, max_edges)


def test_plan_refuses_when_a_node_reaches_too_far():
    ei = torch.tensor([[0, 900, 5], [3, 3, 4]])
    rowptr, nbr = csr(ei, 1000, 1)
    T, *_ = plan(rowptr, nbr, 1000, 512, 128, 1000)
    assert T == 0                         # node 3 gathers rows 0 and 900
    T, *_ = plan(rowptr, nbr, 1000, 1024, 128, 1000)
    assert T > 0
    T, *_ = plan(rowptr, nbr, 1000, 1024, 128, 1)
    assert T == 0                         # node 3 has two in-edges


def test_plan_edge_cases():
    rowptr = np.zeros(8, np.int32)      # 7 nodes, no edges
    T, tb, lo, rows, mx = plan(rowptr, np.zeros(0, np.int32), 7, 512, 4, 100)
    assert T == 2 and list(tb) == [0, 4, 7] and list(rows) == [0, 0] and mx[0] == 0
    T, *_ = plan(np.zeros(1, np.int32), np.zeros(0, np.int32), 0, 512, 4, 100)
    assert T == 0
    lib = _lib.load()
    n = ctypes.c_int32(0)
    arr = np.zeros(8, np.int32)
    p = arr.ctypes.data
    assert lib.gine_graph_plan_windows(p, p, 7, 0, 4, 10, p, p, p, ctypes.byref(n), p) == 1
    assert lib.gine_graph_plan_windows(None, p, 7, 8, 4, 10, p, p, p, ctypes.byref(n), p) == 1


def test_window_entry_points_validate_on_host():
    lib = _lib.load()
    plan_ = _lib.WindowPlan(None, None, None, 0, 32, 0, 0, 1)
    assert lib.gine_mp_fwd_win(*([None] * 8), 100, 128, 0, ctypes.byref(plan_), None) == 1
    good = np.zeros(4, np.int32).ctypes.data
    plan_ = _lib.WindowPlan(good, good, good, 1, 24, 10, 10, 10)   # bad slice width
    assert lib.gine_mp_fwd_win(*([None] * 8), 100, 96, 0, ctypes.byref(plan_), None) == 1
    plan_ = _lib.WindowPlan(good, good, good, 1, 32, 4096, 10, 10)  # window too big for LDS
    assert lib.gine_mp_fwd_win(*([None] * 8), 100, 128, 0, ctypes.byref(plan_), None) == 1
    plan_ = _lib.WindowPlan(good, good, good, 1, 8, 10, 10, 10)     # 16 slices > 8
    assert lib.gine_mp_fwd_win(*([None] * 8), 100, 128, 0, ctypes.byref(plan_), None) == 1
    assert lib.gine_mp_bwd_win_finalize(None, 4, 128, 32, None, None, None, None) == 1
    assert lib.gine_mp_bwd_win_finalize(good, 4, 128, 48, good, good, good, None) == 1


@pytest.mark.parametrize("max_nodes", [128, 100, 40])
def test_plan_window_slots_balance_degrees(max_nodes):
    """gine_graph_plan_window_slots: per tile a permutation of its nodes; positions [0, 64)
    hold the heaviest nodes, position 64 + g the (g+1)-th lightest, so the lane group that
    runs the heaviest node runs the lightest one second."""
    ei, ea, n = knn_batch_graph(500, 10, 3, seed=1)
    rowptr, nbr = csr(ei, n, 0)
    T, tb, lo, rows, mx = plan(rowptr, nbr, n, 512, max_nodes, 1900)
    slot = np.full(n, -1, np.int16)
    _lib.call("gine_graph_plan_window_slots", rowptr.ctypes.data, tb.ctypes.data, T,
              slot.ctypes.data)
    deg = np.diff(rowptr)
    for t in range(T):
        n0, m = tb[t], tb[t + 1] - tb[t]
        s = slot[n0:n0 + m].astype(np.int64)
        assert sorted(s.tolist()) == list(range(m))          # a permutation of the tile
        d = deg[n0 + s]
        first = min(m, 64)
        assert np.all(np.diff(d[:first]) <= 0)                # heaviest first
        if m > 64:
            assert np.all(np.diff(d[64:]) >= 0)               # then lightest first
            assert d[:first].min() >= d[64:].max()
            pair = d[:m - 64] + d[64:]
            naive = deg[n0:n0 + m - 64] + deg[n0 + 64:n0 + m]
            assert pair.max() <= naive.max()
    bad = np.array([0, 200], np.int32)                        # a tile wider than 128 nodes
    with pytest.raises(_lib.GineError):
        _lib.call("gine_graph_plan_window_slots", np.zeros(201, np.int32).ctypes.data,
                  bad.ctypes.data, 1, np.zeros(200, np.int16).ctypes.data)
