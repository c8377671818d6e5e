"""CPU, 2 processes over gloo: the data-parallel path.

Parity under DP: the all-reduced gradient on every rank equals the mean over shards of the
per-shard gradients (each shard with its own BatchNorm statistics), computed with the CPU
oracle model -- the DP machinery (flat gradient buffer, one all-reduce, parameter broadcast,
graph sharding) is device-agnostic.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raincast_gnn.distributed import FlatGradReducer, broadcast_parameters, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_grads(model, batch):
    model.zero_grad(set_to_none=True)
    loss = model.crps(model(batch), batch.y)
    loss.backward()
    return torch.cat([p.grad.reshape(-1) for p in model.parameters()])


def _worker(rank, world, port, result_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import gine_cpu as O
    from raincast_gnn.data import collate, synthetic_samples
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
    model = O.OracleGNN(35, 32, 2, "MixedLoss", "False", 1.71, 0.5)
    broadcast_parameters(model)
    samples = synthetic_samples(40, 6, k=5, seed=11)
    lo, hi = shard_range(len(samples), rank, world)
    batch = collate(samples[lo:hi])
    params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
    red = FlatGradReducer(model.parameters())
    red.zero_()
    loss = model.crps(model(batch), batch.y)
    loss.backward()
    assert red.check_views()
    red.all_reduce_()
    torch.save({"flat": red.flat.clone(), "params": params0},
               os.path.join(result_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_allreduce_equals_mean_of_shard_grads(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["flat"], res[1]["flat"])
    for k in res[0]["params"]:  # broadcast made the start point identical
        assert torch.equal(res[0]["params"][k], res[1]["params"][k]), k
    # single-process reference: mean over shards of per-shard gradients
    from oracle import gine_cpu as O
    from raincast_gnn.data import collate, synthetic_samples
    model = O.OracleGNN(35, 32, 2, "MixedLoss", "False", 1.71, 0.5)
    model.load_state_dict(res[0]["params"], strict=False)
    samples = synthetic_samples(40, 6, k=5, seed=11)
    grads = []
    for r in range(world):
        lo, hi = shard_range(len(samples), r, world)
        grads.append(_shard_grads(model, collate(samples[lo:hi])))
    expect = torch.stack(grads).mean(0)
    err = (res[0]["flat"] - expect).abs().max() / expect.abs().max()
    assert err <= 1e-5, err  # thread-count-dependent CPU BLAS sums between processes


def test_shard_range_covers_batch():
    for n in (1, 7, 32, 256):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(h - l for l, h in got) - min(h - l for l, h in got) <= 1


def _overlap_worker(rank, world, port, result_dir):
    """The overlapped form: the GINE stack's and the head's gradients (the tail of the flat
    buffer) are all-reduced as soon as autograd has differentiated the stack's input, while
    the backward of the dense front continues; all_reduce_() reduces the front and joins."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import gine_cpu as O
    from raincast_gnn.data import collate, synthetic_samples
    torch.manual_seed(100 + rank)
    model = O.OracleGNN(35, 32, 2, "MixedLoss", "False", 1.71, 0.5)
    broadcast_parameters(model)
    samples = synthetic_samples(40, 6, k=5, seed=11)
    lo, hi = shard_range(len(samples), rank, world)
    batch = collate(samples[lo:hi])
    red = FlatGradReducer(model.parameters())
    tail = list(model.conv.parameters()) + list(model.aggr.parameters())
    red.overlap_after(model.conv, tail)
    fired = []
    model.conv.register_forward_pre_hook(lambda m, i: fired.append(i[0].requires_grad))
    outs = []
    for _ in range(2):                     # two steps: the hook re-arms every forward
        red.zero_()
        loss = model.crps(model(batch), batch.y)
        loss.backward()
        started = red._tail_started
        red.all_reduce_()
        assert not red._tail_started
        outs.append((started, red.flat.clone()))
    # a plain (non-overlapped) reduction of the same step for comparison
    red2 = FlatGradReducer(model.parameters())
    red2.zero_()
    model.crps(model(batch), batch.y).backward()
    red2.all_reduce_()
    torch.save({"outs": outs, "plain": red2.flat.clone(), "fired": fired},
               os.path.join(result_dir, f"ov{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_overlapped_tail_allreduce_equals_plain(tmp_path):
    world = 2
    mp.spawn(_overlap_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    res = [torch.load(tmp_path / f"ov{r}.pt", weights_only=True) for r in range(world)]
    for r in res:
        for started, flat in r["outs"]:
            assert started, "the tail's collective must start inside the backward"
            assert torch.equal(flat, r["plain"])   # same sums, same division
        assert all(r["fired"])
    assert torch.equal(res[0]["plain"], res[1]["plain"])


def test_overlap_after_rejects_a_tail_that_is_not_the_end():
    from oracle import gine_cpu as O
    model = O.OracleGNN(35, 16, 2, "MixedLoss", "False", 1.71, 0.5)
    red = FlatGradReducer(model.parameters())
    with pytest.raises(ValueError, match="end of the flat buffer"):
        red.overlap_after(model.conv, list(model.conv.parameters()))   # aggr follows it
    red.overlap_after(model.conv, list(model.conv.parameters()) + list(model.aggr.parameters()))


def _bail_worker(rank, world, port, result_dir):
    """Rank 1's tail hook bails (as when a tail gradient is outside the flat buffer) while
    rank 0's starts the tail's collective inside the backward: every rank must still issue
    the same collective sequence (tail, then front), and the sums must equal the plain
    reduction's (distributed.py _start_tail)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import gine_cpu as O
    from raincast_gnn.data import collate, synthetic_samples
    torch.manual_seed(7)
    model = O.OracleGNN(35, 32, 2, "MixedLoss", "False", 1.71, 0.5)
    broadcast_parameters(model)
    samples = synthetic_samples(40, 6, k=5, seed=11)
    lo, hi = shard_range(len(samples), rank, world)
    batch = collate(samples[lo:hi])
    red = FlatGradReducer(model.parameters())
    red.overlap_after(model.conv, list(model.conv.parameters()) + list(model.aggr.parameters()))
    if rank == 1:
        red._start_tail = lambda grad: None  # the hook bails on this rank only
    red.zero_()
    model.crps(model(batch), batch.y).backward()
    started = red._tail_started
    red.all_reduce_()
    red2 = FlatGradReducer(model.parameters())
    red2.zero_()
    model.crps(model(batch), batch.y).backward()
    red2.all_reduce_()
    torch.save({"started": started, "flat": red.flat.clone(), "plain": red2.flat.clone()},
               os.path.join(result_dir, f"bail{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_tail_hook_bailing_on_one_rank_keeps_the_collective_order(tmp_path):
    world = 2
    mp.spawn(_bail_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"bail{r}.pt", weights_only=True) for r in range(world)]
    assert res[0]["started"] and not res[1]["started"]
    for r in res:
        assert torch.equal(r["flat"], r["plain"])
    assert torch.equal(res[0]["flat"], res[1]["flat"])


def _barrier_check_worker(rank, world, port, result_dir):
    """check_grid_barriers is collective: a failure word on rank 0 only makes BOTH ranks raise
    (instead of rank 1 blocking in its next collective while rank 0 raised)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ctypes
    from raincast_gnn import _lib
    from raincast_gnn import functional as Fn

    class FakeBn:
        num_features = 128
    words = ctypes.c_int64(0)
    _lib.call("gine_bn_acc_words", 128, ctypes.byref(words))
    idx = ctypes.c_int64(0)
    _lib.call("gine_bn_acc_barrier_failures_index", 128, ctypes.byref(idx))
    acc = torch.zeros(int(words.value), dtype=torch.int64)
    if rank == 0:
        acc[int(idx.value)] = 3
    fake = FakeBn()  # (_BN_ACC holds its modules weakly)
    Fn._BN_ACC[fake] = {("cpu", "fwd"): acc}
    raised = None
    try:
        Fn.check_grid_barriers()
    except _lib.GineError as e:
        raised = str(e)
    Fn._BN_ACC.clear()
    Fn.check_grid_barriers()  # reset: nothing pending on any rank
    torch.save({"raised": raised, "acc_sum": int(acc.abs().sum())},
               os.path.join(result_dir, f"chk{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_grid_barrier_check_raises_on_every_rank(tmp_path):
    world = 2
    mp.spawn(_barrier_check_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    res = [torch.load(tmp_path / f"chk{r}.pt", weights_only=True) for r in range(world)]
    assert "grid barrier timed out" in res[0]["raised"] and res[0]["acc_sum"] == 0
    assert "another rank" in res[1]["raised"]
