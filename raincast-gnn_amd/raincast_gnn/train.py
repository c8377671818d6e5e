"""Training driver on the engine: the counterpart of the reference's train.py.

Same procedure as train.py:55-208, with the data path of this package (device-resident
samples, :mod:`raincast_gnn.batching`) instead of PyG's host DataLoader:

* :func:`split_train_val` -- ``random_split(dataset, [n - int(0.1 n), int(0.1 n)])``
  (train.py:147-150);
* :func:`sanity_forward` -- the ``with torch.no_grad(): model(example_data)`` check of
  train.py:181-183, which runs in TRAIN mode and so bumps every BatchNorm's running
  statistics and ``num_batches_tracked`` once before epoch 1;
* :func:`train_one_epoch` / :func:`evaluate` -- train.py:55-74 / 76-91: the epoch loss is
  the mean over batches of each batch's loss, summed on the host in the reference's order
  (``total_loss += loss.item()``) but read back once per epoch instead of once per step;
* :func:`fit` -- the epoch loop with the best-validation checkpoint
  (``torch.save(model.state_dict(), dir/models/run_<id>-best.ckpt)``, train.py:188-208);
  the state_dict keys are the reference's, so the file loads into models/gnn.py's GNN.

:class:`StepRunner` is the training step (forward, loss, backward, optimizer -- and with
data parallelism the gradient all-reduce between backward and the optimizer).  After two
eager steps of a batch size it captures that size's step as a HIP graph and replays it,
copying each batch into the graph's static input buffers (the edge list of a batch size is
one cached tensor, see batching.DeviceDataset.block_graph, so the graph's CSR is built once).
Replays take the same trajectory as eager steps (tests/test_gpu_parity.py:
test_graph_capture_replay_matches_eager).

Data parallelism: every rank iterates the same global batch order and takes
its contiguous shard of graphs (``DeviceLoader(rank=, world=)``); gradients are averaged by
one all-reduce of the flat gradient buffer; validation runs on every rank over the whole
validation set after the BatchNorm running statistics are broadcast from rank 0.  That
broadcast reproduces DistributedDataParallel's buffer semantics at every point where the
buffers are read: DDP overwrites each rank's buffers with rank 0's at the start of every
forward, and a training-mode forward does not read them, so rank 0's buffers -- the ones
DDP would save -- evolve from rank 0's batches alone, exactly as here.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import random
import sys

import numpy as np
import torch
import torch.distributed as dist

from . import gradbuf
from .batching import DeviceDataset, DeviceLoader
from .data import GraphBatch

log = logging.getLogger("raincast_gnn.train")


def set_seed(seed: int) -> None:
    """train.py:44-50."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def split_train_val(dataset: DeviceDataset, val_fraction: float = 0.1,
                    generator: torch.Generator | None = None):
    """``random_split(dataset, [n_train, n_val])`` with n_val = int(0.1 * n) (train.py:
    147-150): one permutation of the sample indices, the first n_train train, the rest val."""
    n = len(dataset)
    n_val = int(val_fraction * n)
    perm = torch.randperm(n, generator=generator)
    return dataset.subset(perm[:n - n_val]), dataset.subset(perm[n - n_val:])


def _world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_buffers(model: torch.nn.Module, src: int = 0) -> None:
    """Every rank takes rank ``src``'s buffers (BatchNorm running statistics)."""
    if _world() == 1:
        return
    with torch.no_grad():
        for b in model.buffers():
            dist.broadcast(b, src=src)


class StepRunner:
    """One training step per call; eager for the first ``warmup`` steps of each batch size,
    then a captured HIP graph per batch size (``graphed=True``, CUDA/HIP devices only).

    ``optimizer`` is a :class:`raincast_gnn.optim.FlatAdamW` (one kernel over the flat
    buffer) or any torch optimizer (``capturable=True`` for graph capture).  ``reducer`` is a
    :class:`raincast_gnn.distributed.FlatGradReducer` over the same gradients (data
    parallelism).  ``allreduce``: "split" (default) launches the all-reduce between the
    fwd+bwd graph and the optimizer graph; "graph" captures it inside the one step graph
    (RCCL only; the capture of a collective has only run at world 1 so far, and costs
    0.534 -> 0.548 ms per cfg2 step when split, DESIGN.md 5 -- the same choice and default
    as ``bench.py --allreduce``).  gloo groups always split (their collectives cannot be
    captured).
    """

    def __init__(self, model, optimizer, graphed: bool = True, warmup: int = 2,
                 reducer=None, allreduce: str = "split"):
        if allreduce not in ("split", "graph"):
            raise ValueError(f"allreduce={allreduce!r}: expected 'split' or 'graph'")
        self.model, self.opt, self.reducer = model, optimizer, reducer
        self.graphed, self.warmup, self.allreduce = graphed, warmup, allreduce
        if (reducer is not None and allreduce == "graph" and dist.is_initialized()
                and dist.get_backend() == "nccl" and reducer.offsets is not None
                and hasattr(model, "conv") and hasattr(model, "aggr")):
            # the GINE stack's and the head's gradients reduced on a side stream under the
            # rest of the backward (distributed.FlatGradReducer.overlap_after)
            reducer.overlap_after(model.conv, list(model.conv.parameters())
                                  + list(model.aggr.parameters()))
        self._seen: dict[int, int] = {}
        self._graphs: dict[int, tuple] = {}

    # -- the step ----------------------------------------------------------------------
    def _zero(self):
        self.opt.zero_grad(set_to_none=True)

    def _fwd_bwd(self, batch):
        self._zero()
        loss = self.model.loss_fn.crps(self.model(batch), batch.y)
        gradbuf.loss_backward(loss)
        if hasattr(self.opt, "gather_grads"):
            self.opt.gather_grads()   # the flat gradient buffer complete (all-reduce payload)
        return loss

    def _reduce(self):
        if self.reducer is not None:
            self.reducer.all_reduce_()

    def eager(self, batch) -> torch.Tensor:
        loss = self._fwd_bwd(batch)
        self._reduce()
        self.opt.step()
        return loss.detach()

    def __call__(self, batch: GraphBatch) -> torch.Tensor:
        """Run one step on ``batch``; returns the loss (a device scalar owned by the
        caller)."""
        n = batch.num_graphs
        dev = batch.x.device
        if not self.graphed or dev.type != "cuda":
            return self.eager(batch)
        seen = self._seen.get(n, 0)
        self._seen[n] = seen + 1
        if seen < self.warmup:
            return self.eager(batch)
        if n not in self._graphs:
            self._capture(batch)
        g_fb, g_opt, static, loss = self._graphs[n]
        if static.edge_index is not batch.edge_index:
            return self.eager(batch)  # a different graph: not what was captured
        static.x.copy_(batch.x)
        static.ensemble.copy_(batch.ensemble)
        static.y.copy_(batch.y)
        g_fb.replay()
        if g_opt is not None:
            self._reduce()
            g_opt.replay()
        return loss.detach().clone()

    def _capture(self, batch):
        static = GraphBatch(batch.x.clone(), batch.ensemble.clone(), batch.edge_index,
                            batch.edge_attr, batch.y.clone(), batch.batch, batch.ptr,
                            batch.num_graphs)
        collective = self.reducer is not None and _world() > 1
        # allreduce="graph" with RCCL: the all-reduce inside the step graph (between the
        # backward and the optimizer); otherwise two graphs with the all-reduce launched
        # between them (gloo collectives cannot be captured)
        in_graph = collective and self.allreduce == "graph" and dist.get_backend() == "nccl"
        split = collective and not in_graph
        torch.cuda.synchronize()
        g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_fb):
            loss = self._fwd_bwd(static)
            if in_graph:
                self._reduce()
            if not split:
                self.opt.step()
        g_opt = None
        if split:
            g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_opt):
                self.opt.step()
        self._graphs[batch.num_graphs] = (g_fb, g_opt, static, loss)


def _mean_over_ranks(v: float, dev) -> float:
    if _world() == 1:
        return v
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.item() / _world()


def train_one_epoch(model, loader, optimizer, device, logger=None, runner=None) -> float:
    """train.py:55-74: train mode, one optimizer step per batch, mean batch loss."""
    model.train()
    runner = runner or StepRunner(model, optimizer, graphed=False)
    losses = [runner(b.to(device) if b.x.device != torch.device(device) else b)
              for b in loader]
    if not losses:
        raise ValueError(
            "the training loader yielded no batch (a data-parallel loader skips batches with "
            "fewer graphs than ranks: use at least one graph per rank per batch)")
    total = 0.0
    for v in torch.stack(losses).double().cpu().tolist():  # train.py:72 order, one readback
        total += v
    from .functional import check_grid_barriers
    check_grid_barriers()  # (synchronised by the readback above)
    avg = _mean_over_ranks(total / len(losses), losses[0].device)
    (logger or log).info(f"  [Train] Loss: {avg:.6f}")
    return avg


@torch.no_grad()
def evaluate(model, loader, device, logger=None) -> float:
    """train.py:76-91: eval mode (BatchNorm from running statistics), mean batch loss."""
    model.eval()
    losses = [model.loss_fn.crps(model(b.to(device)), b.to(device).y) for b in loader]
    if not losses:
        raise ValueError("the validation loader yielded no batch")
    total = 0.0
    for v in torch.stack(losses).double().cpu().tolist():
        total += v
    avg = total / len(losses)
    (logger or log).info(f"  [Val] Loss: {avg:.6f}")
    return avg


@torch.no_grad()
def sanity_forward(model, example: GraphBatch, device) -> torch.Tensor:
    """train.py:181-183: one forward of a single sample with the model still in train mode
    (the reference never calls ``eval()`` before it), so BatchNorm uses batch statistics
    and updates its running buffers once."""
    return model(example.to(device))


def fit(model, optimizer, train_loader, val_loader, device, max_epochs: int,
        ckpt_dir: str | None = None, run_id: str = "0", example: GraphBatch | None = None,
        logger=None, runner: StepRunner | None = None) -> dict:
    """train.py:179-208: sanity forward, then per epoch train + validate, saving the
    state_dict whenever the validation loss improves.  Returns the loss history and the
    best checkpoint."""
    logger = logger or log
    rank = dist.get_rank() if _world() > 1 else 0
    if example is not None:
        sanity_forward(model, example, device)
    runner = runner or StepRunner(model, optimizer)
    best, best_path = float("inf"), None
    history = {"train": [], "val": []}
    if ckpt_dir is not None:
        os.makedirs(ckpt_dir, exist_ok=True)
    logger.info(f"Starting training for {max_epochs} epochs...")
    for epoch in range(1, max_epochs + 1):
        logger.info(f"=== Epoch {epoch}/{max_epochs} ===")
        history["train"].append(train_one_epoch(model, train_loader, optimizer, device,
                                                logger, runner))
        broadcast_buffers(model)
        val = evaluate(model, val_loader, device, logger)
        history["val"].append(val)
        if val < best:
            best = val
            if ckpt_dir is not None:
                best_path = os.path.join(ckpt_dir, f"run_{run_id}-best.ckpt")
                if rank == 0:
                    torch.save({k: v.detach().cpu().clone()
                                for k, v in model.state_dict().items()}, best_path)
                logger.info(f"[Checkpoint] New best val_loss: {val:.6f}. Saved to {best_path}")
    logger.info("Training completed.")
    return {"history": history, "best_val_loss": best, "best_ckpt_path": best_path}


# ---------------------------------------------------------------------------------------
# command line (train.py:27-208 with synthetic station data: the EUPPBench ETL is out of
# scope)
# ---------------------------------------------------------------------------------------
def main(argv=None) -> dict:
    from .data import synthetic_samples
    from .distributed import (FlatGradReducer, broadcast_parameters, env_rank,
                              note_device_sharing)
    from .models import gnn_from_params
    from .optim import FlatAdamW
    from .params import load_params

    ap = argparse.ArgumentParser(description="Train the station-graph GNN on the engine.")
    ap.add_argument("--dir", required=True, help="directory with params.json; logs/models")
    ap.add_argument("--run_id", required=True)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--stations", type=int, default=122, help="synthetic station count")
    ap.add_argument("--samples", type=int, default=64, help="synthetic samples (times)")
    ap.add_argument("--k", type=int, default=10, help="k-NN graph (None: radius max_dist)")
    ap.add_argument("--radius", action="store_true", help="radius graph of params max_dist")
    ap.add_argument("--epochs", type=int, default=None, help="override max_epochs")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph replay")
    ap.epilog = ("Data parallel (torchrun, one process per GPU): the world size must divide "
                 "params.json's batch_size, so every rank gets an equal shard of each batch.")
    ap.add_argument("--allreduce", choices=("split", "graph"), default="split",
                    help="data-parallel all-reduce between the step's two graphs (split) or "
                         "captured inside one (graph, RCCL); see StepRunner")
    args = ap.parse_args(argv)

    rank, local_rank, world = env_rank()
    config = load_params(os.path.join(args.dir, "params.json"))
    bs = config["batch_size"]
    if world > 1 and bs % world:
        # DeviceLoader's condition (equal shards in every full batch), reported up front
        raise SystemExit(f"params.json batch_size {bs} is not a multiple of the {world} "
                         f"data-parallel ranks; run with a world size that divides it "
                         f"(24h_mixed: batch_size 8 -> 1, 2, 4 or 8 GPUs)")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl")
    os.makedirs(os.path.join(args.dir, "logs"), exist_ok=True)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(message)s",
                        handlers=[logging.FileHandler(os.path.join(
                            args.dir, "logs", f"train_{args.run_id}.log"), mode="w"),
                            logging.StreamHandler(sys.stdout)])
    set_seed(args.seed)
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    note_device_sharing()
    samples = synthetic_samples(args.stations, args.samples, k=args.k, seed=args.seed,
                                max_dist=config.get("max_dist", 100.0) if args.radius else None)
    full = DeviceDataset(samples, device)
    train_set, val_set = split_train_val(full)
    log.info(f"Dataset sizes => Train: {len(train_set)}, Val: {len(val_set)}")
    train_loader = DeviceLoader(train_set, bs, shuffle=True, seed=args.seed, rank=rank,
                                world=world)
    val_loader = DeviceLoader(val_set, bs, shuffle=False)
    model = gnn_from_params(config, in_channels=samples[0].x.size(1)).to(device)
    broadcast_parameters(model)
    opt = FlatAdamW(model.parameters(), lr=config["lr"])
    reducer = (FlatGradReducer(model.parameters(), flat=opt.flat_grad, offsets=opt._offsets)
               if world > 1 else None)
    runner = StepRunner(model, opt, graphed=not args.eager, reducer=reducer,
                        allreduce=args.allreduce)
    out = fit(model, opt, train_loader, val_loader, device,
              args.epochs or config["max_epochs"], os.path.join(args.dir, "models"),
              args.run_id, example=train_set.batch(torch.tensor([0])), runner=runner)
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
