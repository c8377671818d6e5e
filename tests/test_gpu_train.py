"""GPU: the training driver (raincast_gnn/train.py; reference train.py:55-208) on the HIP
engine against the same loop on the CPU oracle, and engine-level data parallelism.

* Two epochs (sanity forward, shuffled train batches with HIP-graph replays after the first
  two steps of each batch size, validation, best checkpoint) follow the oracle's loss
  trajectory: per-epoch train and validation losses against the fp64 oracle's within
  1e-5 relative or twice the fp32 oracle's own drift from it (all run AdamW, lr 1e-4, on the
  same batches in the same order).
* The checkpoint is a reference state_dict: it loads into the oracle (strict) and gives the
  engine's validation loss.
* Data parallelism: two ranks (gloo, both on cuda:0) running the engine; the all-reduced
  gradient in the flat buffer equals the mean over shards of the oracle's per-shard
  gradients (1e-5, fp64 tie-break), and both ranks hold the same bits.
"""
import copy
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from helpers import assert_close_tiebreak
from raincast_gnn import train as T
from raincast_gnn.batching import DeviceDataset, DeviceLoader
from raincast_gnn.data import synthetic_samples
from raincast_gnn.models import gnn_from_params
from raincast_gnn.optim import FlatAdamW
from raincast_gnn.params import EXPERIMENTS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


class _Oracle(torch.nn.Module):
    def __init__(self, params):
        super().__init__()
        from oracle import gine_cpu as O
        self.net = O.OracleGNN(35, params["gnn_hidden"], params["gnn_layers"], params["loss"],
                               params["grad_u"], params["u"], params["xi"])
        self.loss_fn = type("L", (), {"crps": staticmethod(self.net.crps)})()

    def forward(self, data):
        dt = self.net.dim_red.weight.dtype
        if data.x.dtype != dt:   # the fp64 trajectory: inputs promoted like the weights
            import copy as _copy
            data = _copy.copy(data)
            data.x, data.ensemble, data.edge_attr = (t.to(dt) for t in (
                data.x, data.ensemble, data.edge_attr))
        return self.net(data)


def test_two_epochs_follow_oracle_trajectory(tmp_path):
    params = dict(EXPERIMENTS["24h_mixed"])
    samples = synthetic_samples(60, 14, k=6, seed=21)
    split = torch.Generator().manual_seed(0)
    gpu_full = DeviceDataset(samples, DEV)
    cpu_full = DeviceDataset(samples, "cpu")
    gtr, gva = T.split_train_val(gpu_full, generator=split)
    ctr, cva = T.split_train_val(cpu_full, generator=torch.Generator().manual_seed(0))

    torch.manual_seed(42)
    model = gnn_from_params(params)
    ref = _Oracle(params)
    ref.net.load_state_dict(model.state_dict(), strict=True)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(DEV)
    opt = FlatAdamW(model.parameters(), lr=params["lr"])
    ropt = torch.optim.AdamW(ref.parameters(), lr=params["lr"])
    runner = T.StepRunner(model, opt, graphed=True)
    got = T.fit(model, opt, DeviceLoader(gtr, 4, seed=3), DeviceLoader(gva, 4, shuffle=False),
                DEV, 2, ckpt_dir=str(tmp_path / "gpu"), run_id="g",
                example=gtr.batch(torch.tensor([0])), runner=runner)
    assert len(runner._graphs) == 1               # batch size 4 replayed from a HIP graph
    want = T.fit(ref, ropt, DeviceLoader(ctr, 4, seed=3), DeviceLoader(cva, 4, shuffle=False),
                 "cpu", 2, ckpt_dir=str(tmp_path / "cpu"), run_id="c",
                 example=ctr.batch(torch.tensor([0])))
    # The trajectory's own conditioning: AdamW's first steps move every parameter by about
    # lr * sign(g), so a gradient entry within rounding of zero -- which any change of
    # summation order can flip -- moves its parameter by 2 lr either way, and two fp32 runs
    # of the same loop drift apart by more than the one-step tolerance.  The bar is the
    # reference restatement's own fp32 drift from the fp64 trajectory (x2), or 1e-5 if
    # larger; the engine is compared with the fp64 trajectory.
    ref64 = _Oracle(params).double()
    ref64.net.load_state_dict({k: v.double() if v.is_floating_point() else v
                               for k, v in init.items()}, strict=True)
    want64 = T.fit(ref64, torch.optim.AdamW(ref64.parameters(), lr=params["lr"]),
                   DeviceLoader(ctr, 4, seed=3), DeviceLoader(cva, 4, shuffle=False), "cpu", 2,
                   ckpt_dir=str(tmp_path / "cpu64"), run_id="c64",
                   example=ctr.batch(torch.tensor([0])))
    for key in ("train", "val"):
        for a, b, c in zip(got["history"][key], want["history"][key], want64["history"][key]):
            env = abs(b - c)
            assert abs(a - c) <= max(TOL * abs(c), 2.0 * env), (key, a, b, c)
    # BatchNorm bookkeeping: sanity forward + every step, as the reference
    nbt = [int(b) for n, b in model.named_buffers() if n.endswith("num_batches_tracked")]
    rnbt = [int(b) for n, b in ref.net.named_buffers() if n.endswith("num_batches_tracked")]
    assert nbt == rnbt and nbt[0] == 1 + 2 * len(DeviceLoader(gtr, 4))
    # the engine's best checkpoint is a reference state_dict
    state = torch.load(got["best_ckpt_path"], weights_only=True)
    chk = _Oracle(params)
    chk.net.load_state_dict(state, strict=True)
    val = T.evaluate(chk, DeviceLoader(cva, 4, shuffle=False), "cpu")
    assert abs(val - got["best_val_loss"]) <= TOL * abs(val)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _dp_worker(rank, world, port, out_dir, overlap=False):
    import torch.distributed as dist
    from raincast_gnn.data import collate
    from raincast_gnn.distributed import FlatGradReducer, broadcast_parameters, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from raincast_gnn.distributed import note_device_sharing
    assert note_device_sharing()   # both ranks on cuda:0: the grid-barrier layer stays off
    params = dict(EXPERIMENTS["24h_mixed"])
    torch.manual_seed(100 + rank)               # different init per rank: broadcast fixes it
    model = gnn_from_params(params).to(dev).train()
    broadcast_parameters(model)
    start = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    samples = synthetic_samples(80, 6, k=6, seed=31)
    lo, hi = shard_range(len(samples), rank, world)
    batch = collate(samples[lo:hi]).to(dev)
    opt = FlatAdamW(model.parameters(), lr=params["lr"])
    red = FlatGradReducer(model.parameters(), flat=opt.flat_grad, offsets=opt._offsets)
    if overlap:  # the GINE stack's + head's tail reduced from inside the backward
        red.overlap_after(model.conv, list(model.conv.parameters())
                          + list(model.aggr.parameters()))
    runner = T.StepRunner(model, opt, graphed=False, reducer=red)
    runner._fwd_bwd(batch)
    assert red._tail_started == overlap
    red.all_reduce_()
    torch.cuda.synchronize()
    torch.save({"flat": opt.flat_grad.cpu(), "start": start, "offsets": list(opt._offsets),
                "names": [n for n, _ in model.named_parameters()]},
               os.path.join(out_dir, f"rank{rank}{'_ov' if overlap else ''}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_engine_data_parallel_gradient_is_mean_of_shards(tmp_path):
    world = 2
    mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["flat"], res[1]["flat"])
    for k in res[0]["start"]:
        assert torch.equal(res[0]["start"][k], res[1]["start"][k]), k
    from raincast_gnn.data import collate
    from raincast_gnn.distributed import shard_range
    params = dict(EXPERIMENTS["24h_mixed"])
    samples = synthetic_samples(80, 6, k=6, seed=31)
    means = {}
    for dt in (torch.float32, torch.float64):
        ref = _Oracle(params)
        ref.net.load_state_dict(res[0]["start"], strict=True)
        ref = ref.to(dt)
        grads = []
        for r in range(world):
            lo, hi = shard_range(len(samples), r, world)
            b = copy.copy(collate(samples[lo:hi]))
            b.x, b.ensemble, b.edge_attr = (t.to(dt) for t in (b.x, b.ensemble, b.edge_attr))
            ref.zero_grad(set_to_none=True)
            ref.loss_fn.crps(ref(b), b.y).backward()
            grads.append(torch.cat([p.grad.reshape(-1) for p in ref.net.parameters()]))
        means[dt] = torch.stack(grads).mean(0)
    off = 0  # into the packed oracle gradient; FlatAdamW's slices are aligned (gaps zero)
    names = res[0]["names"]
    shapes = [p.shape for p in _Oracle(params).net.parameters()]
    for name, shp, foff in zip(names, shapes, res[0]["offsets"]):
        n = int(torch.Size(shp).numel())
        sl = slice(off, off + n)
        off += n
        if name.endswith(".eps") or name.endswith(".nn.0.bias"):
            continue  # conditioning-scaled / analytically-zero: covered in test_gpu_parity
        assert_close_tiebreak(res[0]["flat"][foff:foff + n], means[torch.float32][sl],
                              means[torch.float64][sl], TOL, name)
    assert off == means[torch.float32].numel()
    covered = torch.zeros(res[0]["flat"].numel(), dtype=torch.bool)
    for shp, foff in zip(shapes, res[0]["offsets"]):
        covered[foff:foff + int(torch.Size(shp).numel())] = True
    assert not res[0]["flat"][~covered].any()  # the alignment gaps hold no gradient


@pytest.mark.timeout(300)
def test_engine_data_parallel_overlapped_tail_same_bits(tmp_path):
    """The overlapped reduction (distributed.FlatGradReducer.overlap_after: the deferred GINE
    and head reductions launched from inside the backward, their tail of the flat buffer
    reduced on a side stream) gives the same bits as the plain one, 2 gloo ranks."""
    world = 2
    for ov in (False, True):
        mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path), ov), nprocs=world,
                 join=True)
    for r in range(world):
        a = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)["flat"]
        b = torch.load(tmp_path / f"rank{r}_ov.pt", weights_only=True)["flat"]
        assert torch.equal(a, b)
