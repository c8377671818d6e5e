#!/usr/bin/env python3
"""Training-throughput benchmark of the station-graph GNN on MI355X.

Metric (BASELINE.json): training graphs/s (+ edges aggregated/s), 24h_mixed config.
One step = one full training step exactly as train.py:55-74 does it -- DeepSet + dim_red +
4 GINE layers (HIP engine) + head + PostProcess + MixedLoss + backward + AdamW -- on one
pre-collated batch resident in HBM.  N=1 runs configs[1] (500-station k=10 graphs, 32 per
GPU); with N>1 every rank runs its own 32 graphs (weak scaling) and the gradient is
averaged with one RCCL all-reduce per step, captured in the step's HIP graph.  The same run
also measures cfg4 (global batch 256 split over the N ranks: strong scaling) and reports
it as ``strong_scaling_cfg4``.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints ONE JSON line.  Per-kernel timings (HIP events on the launch stream) and the
CPU baseline (oracle, rank 0, N=1 only) are measured in the same process.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "raincast-gnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from raincast_gnn import functional as Fn  # noqa: E402
from raincast_gnn import gradbuf, options  # noqa: E402
from raincast_gnn.data import relabel_stations, synthetic_batch  # noqa: E402
from raincast_gnn.data import station_order as station_order_of  # noqa: E402
from raincast_gnn.distributed import (FlatGradReducer, broadcast_parameters, env_rank,  # noqa: E402
                                      note_device_sharing)
from raincast_gnn.graph import get_graph  # noqa: E402
from raincast_gnn.models import gnn_from_params  # noqa: E402
from raincast_gnn.optim import FlatAdamW  # noqa: E402
from raincast_gnn.params import BENCH_CONFIGS  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 matrix peak (dense)
# what the node-MLP products actually execute: split-bf16x3 (gine_bf16x3.hpp), six
# v_mfma_f32_32x32x16_bf16 per fp32-class product on the bf16 rate (16x fp32, dense): the
# ceiling of an fp32-class flop on the instructions the kernels run
BF16X3_EXEC_PEAK_TFLOPS = round(16 * FP32_MFMA_PEAK_TFLOPS / 6, 1)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=sorted(BENCH_CONFIGS))
    ap.add_argument("--hidden", type=int, default=None,
                    help="gnn_hidden override (the D=64 sweep of BASELINE.md:47 / the north "
                         "star's 64-dim features); default: params.json's 128")
    ap.add_argument("--no-graph", action="store_true", help="eager steps (no HIP graph)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the cfg4 strong-scaling line (global batch 256) that the "
                         "default cfg2 run adds")
    ap.add_argument("--allreduce", choices=("graph", "split"), default="split",
                    help="split (default): fwd+bwd graph, the RCCL all-reduce launched "
                         "between it and the optimizer graph -- keeps multi-rank runs off "
                         "the collective-capture path, which has never run with more than "
                         "one rank; costs the two cross-stream hops of an eager collective "
                         "(0.548 vs 0.534 ms per cfg2 step at world 1, profiles/r03_s08); "
                         "graph: the all-reduce captured inside the step's HIP graph, the "
                         "GINE stack's and head's gradients reduced on a side stream under "
                         "the rest of the backward (RCCL only; a failed capture exits "
                         "non-zero)")
    ap.add_argument("--station-order", choices=("locality", "dataset"), default="locality",
                    help="locality: the batch in the engine's station order (reverse "
                         "Cuthill-McKee, raincast_gnn.data.station_order -- the device "
                         "loader's layout); dataset: the reference's collated order")
    ap.add_argument("--force-allreduce", action="store_true",
                    help="run the all-reduce even with one rank (rehearsal of the capture)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm, the benchmark) | gloo (multi-rank rehearsal on "
                         "one GPU: ranks share the device)")
    ap.add_argument("--dropin", action="store_true",
                    help="time the drop-in path instead: the reference's model structure in "
                         "torch with raincast_gnn's GINEConv, train.py's loop (batch.to(device) "
                         "and loss.item() every step); 1 GPU")
    ap.add_argument("--settle-steps", type=int, default=100,
                    help="replays of the captured step after capture, before the timed steps "
                         "(same count on every rank): the GPU clock ramps for ~25 ms after the "
                         "CPU-bound preparation (cfg2 step 0.474 -> 0.436 ms over the first 50 "
                         "replays, profiles/r06_s18_clock_ramp.txt), so a 20-step region "
                         "right after capture would time the ramp, not the training step; "
                         "0 times the ramp")
    ap.add_argument("--no-head-fold", action="store_true",
                    help="A/B: the output head in a launch of its own instead of the last GINE "
                         "layer's (options.HEAD_FOLD)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: ranks over gloo build their shards and time the gradient "
                         "all-reduce alone (launcher / rank / shard / JSON plumbing; no GPU "
                         "step, no HIP call)")
    return ap.parse_args()


# -----------------------------------------------------------------------------------------
# training step
# -----------------------------------------------------------------------------------------
class Trainer:
    def __init__(self, cfg, device, rank, world, graphs_per_rank, allreduce="graph",
                 force_allreduce=False, station_order="locality"):
        self.cfg, self.device, self.world = cfg, device, world
        self.allreduce = allreduce
        self.collective = world > 1 or force_allreduce
        params = cfg.params()
        self.params = params
        torch.manual_seed(42)
        self.model = gnn_from_params(params).to(device).train()
        broadcast_parameters(self.model)
        batch = synthetic_batch(cfg.num_stations, graphs_per_rank, k=cfg.k, seed=1000 + rank)
        if station_order == "locality":
            # the layout DeviceDataset stores samples in (raincast_gnn/batching.py): every
            # graph's stations in reverse Cuthill-McKee order, edges relabelled, edge order
            # kept; collation itself stays outside the timed step, as in the reference
            graph0 = batch.edge_index[:, :batch.edge_index.size(1) // graphs_per_rank]
            batch = relabel_stations(batch, station_order_of(graph0, cfg.num_stations))
        self.batch = batch.to(device)
        # AdamW (train.py:185, torch defaults betas/eps/weight_decay) over one flat buffer;
        # the same flat gradient buffer is what the data-parallel all-reduce reduces
        self.opt = FlatAdamW(self.model.parameters(), lr=params["lr"])
        self.reducer = FlatGradReducer(self.model.parameters(), flat=self.opt.flat_grad,
                                       force=force_allreduce, offsets=self.opt._offsets)
        self.overlap = False
        if (self.collective and allreduce == "graph" and dist.is_initialized()
                and dist.get_backend() == "nccl"):
            # the GINE stack's and the head's gradients (the tail of the flat buffer) are
            # all-reduced on a side stream as soon as the stack's backward is done, under
            # the dense chain's and the DeepSet's backward (captured as a fork of the graph)
            self.reducer.overlap_after(self.model.conv, list(self.model.conv.parameters())
                                       + list(self.model.aggr.parameters()))
            self.overlap = True
        self.graph_fb = self.graph_opt = None
        self.loss = None
        self.allreduce_in_graph = False
        self.ar_events = None  # a list: (start, end) HIP events around each split all-reduce

    def fwd_bwd(self):
        self.opt.zero_grad()            # set_to_none: kernels write grads into flat slices
        pred = self.model(self.batch)
        loss = self.model.loss_fn.crps(pred, self.batch.y)
        gradbuf.loss_backward(loss)      # (no seed-fill launch)
        self.opt.gather_grads()         # flat_grad complete before the all-reduce
        return loss

    def eager_step(self):
        loss = self.fwd_bwd()
        self.reducer.all_reduce_()
        self.opt.step()
        return loss

    def capture(self):
        """The whole step as ONE HIP graph -- fwd + bwd, the RCCL gradient all-reduce (when
        there is a collective) and AdamW -- or, with a gloo group or ``allreduce="split"``,
        fwd+bwd and AdamW as two graphs with the all-reduce launched between them.

        The form is decided here, before any capture starts: only RCCL ("nccl") collectives
        are captured.  A capture that fails is fatal -- a failed capture leaves its stream
        invalidated, so nothing may run on it afterwards (the 2-rank abort of commit
        3462363); the error is printed and the process exits non-zero."""
        in_graph = not self.collective or (
            self.allreduce == "graph" and dist.get_backend() == "nccl")
        if in_graph:
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    self.loss = self.fwd_bwd()
                    if self.collective:
                        self.reducer.all_reduce_()
                    self.opt.step()
            except Exception as e:
                log(f"FATAL: capture of the training step "
                    f"{'with the RCCL all-reduce ' if self.collective else ''}failed "
                    f"({type(e).__name__}: {e}); the capture stream is invalid, exiting "
                    f"(run with --allreduce split to keep the collective out of the graph)")
                raise SystemExit(3) from e
            self.graph_fb, self.graph_opt = g, None
            self.allreduce_in_graph = self.collective
            assert self.opt.views_intact()
            return
        self.graph_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_fb):
            self.loss = self.fwd_bwd()
        self.graph_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_opt):
            self.opt.step()
        assert self.opt.views_intact()

    def step(self):
        if self.graph_fb is None:
            return self.eager_step()
        timed = self.ar_events is not None and self.collective and self.graph_opt is not None
        if timed:
            stream = torch.cuda.current_stream(self.device)
            ev = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
            ev[0].record(stream)
        self.graph_fb.replay()
        if self.graph_opt is not None:
            if timed:
                ev[1].record(stream)
                sync_ms = None
                if dist.get_backend(self.reducer.group) != "nccl":
                    # gloo reduces host copies: the wait for the fwd+bwd graph, timed apart
                    # from the collective itself
                    t0 = time.perf_counter()
                    stream.synchronize()
                    sync_ms = (time.perf_counter() - t0) * 1e3
                t0 = time.perf_counter()
                self.reducer.all_reduce_()
                host_ms = (time.perf_counter() - t0) * 1e3  # the call's host time (gloo: whole)
                ev[2].record(stream)
                self.ar_events.append(ev + (host_ms, sync_ms))
            else:
                self.reducer.all_reduce_()
            self.graph_opt.replay()
        return self.loss


# -----------------------------------------------------------------------------------------
# per-kernel timing (HIP events on the stream the kernels are launched on)
# -----------------------------------------------------------------------------------------
def time_kernels(tr: Trainer, reps: int):
    dev = tr.device
    b = tr.batch
    conv = tr.model.conv.convolutions[1]
    N, D = b.num_nodes, tr.params["gnn_hidden"]
    E = b.edge_index.size(1)
    g = get_graph(b.edge_index, b.edge_attr.float(), N)
    torch.manual_seed(0)
    x = torch.randn(N, D, device=dev)
    dz = torch.randn(N, D, device=dev)
    lw = conv.lin.weight.detach().reshape(-1).contiguous()
    lb = conv.lin.bias.detach().contiguous()
    ep = conv.eps.detach().contiguous()
    l1, bn, _, l2 = conv.nn
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    S = [sh]  # launch stream of the timed lambdas (switched to the capture stream below)
    from raincast_gnn._lib import call, ptr
    lin = Fn.edge_linear_flag()
    P = Fn._count("gine_mlp_num_partials", N, D)
    partials = torch.empty(P, 2, D, dtype=torch.float64, device=dev)
    a1 = torch.empty_like(x)
    y = torch.empty_like(x)
    dbn = torch.empty_like(x)
    mask = torch.empty(N, D, dtype=torch.uint8, device=dev)
    bn_save = torch.empty(4, D, device=dev)
    coef = torch.empty(3, D, device=dev)
    w1, b1, w2, b2 = (t.detach().contiguous() for t in (l1.weight, l1.bias, l2.weight, l2.bias))
    C = Fn._count("gine_mlp_wgrad_num_chunks", N, D)
    slab = torch.empty(2 * C * (D * D + D), device=dev)
    dw1, dw2 = torch.empty(D, D, device=dev), torch.empty(D, D, device=dev)
    db1, db2 = torch.empty(D, device=dev), torch.empty(D, device=dev)
    win = g.window_plan("out", D)
    win_part = (torch.empty(win.num_tiles, 3, D, dtype=torch.float64, device=dev)
                if win is not None else None)
    Pm = Fn._count("gine_mp_bwd_num_partials", N, D)
    mp_part = torch.empty(Pm, 3, D, dtype=torch.float64, device=dev)
    dx = torch.empty_like(x)
    lw_g, lb_g, eps_g = torch.empty(D, device=dev), torch.empty(D, device=dev), torch.empty(1, device=dev)
    z = Fn.mp_forward(x, g, lw, lb, ep)
    rm = torch.zeros(D, device=dev)
    rv = torch.ones(D, device=dev)
    call("gine_mlp_fwd1", ptr(z), ptr(w1), ptr(b1), ptr(a1), ptr(partials), N, D, sh)
    call("gine_bn_fwd_finalize", ptr(partials), P, ptr(bn.weight), ptr(bn.bias), ptr(rm),
         ptr(rv), None, ptr(bn_save), N, D, 0.1, 1e-5, 1, 0, sh)
    call("gine_mlp_fwd2", ptr(a1), ptr(bn_save), ptr(w2), ptr(b2), ptr(x), ptr(y), ptr(mask),
         N, D, 2, sh)
    call("gine_mlp_bwd2", ptr(dz), None, ptr(mask), ptr(a1), ptr(bn_save), ptr(w2), ptr(dbn),
         ptr(partials), N, D, 2, sh)
    call("gine_bn_bwd_finalize", ptr(partials), P, ptr(bn.weight), ptr(bn_save), None, None,
         ptr(coef), N, D, 1, sh)

    kernels = {
        "gine_mp_fwd": (lambda: call("gine_mp_fwd", ptr(x), ptr(g.in_rowptr), ptr(g.in_src),
                                     ptr(g.in_attr), ptr(lw), ptr(lb), ptr(ep), ptr(z), N, D,
                                     lin, S[0]),
                        {"bytes": 4 * (2 * N * D + 2 * E + N + 1)}),
        # the backward the training step runs: LDS-staged window kernel when the graph
        # has a plan (GINE_MP_WINDOW policy, raincast_gnn/graph.py), else the gather kernel
        "gine_mp_bwd": (
            (lambda: call("gine_mp_bwd_win", ptr(dz), ptr(x), ptr(g.out_rowptr),
                          ptr(g.out_dst), ptr(g.out_attr), ptr(lw), ptr(lb), ptr(ep), ptr(dz),
                          ptr(dx), ptr(win_part), N, D, 1 | lin, ctypes.byref(win), S[0]))
            if win is not None else
            (lambda: call("gine_mp_bwd", ptr(dz), ptr(x), ptr(g.out_rowptr), ptr(g.out_dst),
                          ptr(g.out_attr), ptr(lw), ptr(lb), ptr(ep), ptr(dz), ptr(dx),
                          ptr(mp_part), N, D, 1 | lin, S[0])),
            {"bytes": 4 * (3 * N * D + 2 * E + N + 1)}),   # 8(d) B_b, as the roofline
        "gine_mlp_fwd1": (lambda: call("gine_mlp_fwd1", ptr(z), ptr(w1), ptr(b1), ptr(a1),
                                       ptr(partials), N, D, S[0]),
                          {"flops": 2 * N * D * D, "bytes": 8 * N * D}),
        "gine_mlp_fwd2": (lambda: call("gine_mlp_fwd2", ptr(a1), ptr(bn_save), ptr(w2), ptr(b2),
                                       ptr(x), ptr(y), ptr(mask), N, D, 2, S[0]),
                          {"flops": 2 * N * D * D, "bytes": 13 * N * D}),
        "gine_mlp_bwd2": (lambda: call("gine_mlp_bwd2", ptr(dz), None, ptr(mask), ptr(a1),
                                       ptr(bn_save), ptr(w2), ptr(dbn), ptr(partials), N, D, 2,
                                       S[0]),
                          {"flops": 2 * N * D * D, "bytes": 13 * N * D}),
        "gine_mlp_bwd1": (lambda: call("gine_mlp_bwd1", ptr(dbn), ptr(a1), ptr(bn_save),
                                       ptr(coef), ptr(w1), ptr(dx), N, D, S[0]),
                          {"flops": 2 * N * D * D, "bytes": 12 * N * D}),
        # what the step runs: dz = da1 W1 beside dW1 = da1^T z, dW2 = do^T r (+ biases)
        "gine_mlp_bwd1_wgrad": (lambda: call("gine_mlp_bwd1_wgrad", ptr(dz), None, ptr(mask),
                                             ptr(a1), ptr(bn_save), ptr(dbn), ptr(coef), ptr(z),
                                             ptr(w1), ptr(dx), ptr(slab), None, None, None,
                                             None, N, D, 2, S[0]),
                                {"flops": 6 * N * D * D, "bytes": 4 * 5 * N * D + 5 * N * D}),
        "gine_mlp_wgrad": (lambda: call("gine_mlp_wgrad", ptr(dz), None, ptr(mask), ptr(a1),
                                        ptr(bn_save), ptr(dbn), ptr(coef), ptr(z), ptr(slab),
                                        ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), N, D, 2, S[0]),
                           {"flops": 4 * N * D * D, "bytes": 4 * 4 * N * D + 5 * N * D}),
        # the reduction launches between the GEMMs (partials reduced in place; re-running them
        # on their own output only re-sums, shapes unchanged)
        "gine_bn_fwd_finalize": (lambda: call("gine_bn_fwd_finalize", ptr(partials), P,
                                              ptr(bn.weight), ptr(bn.bias), ptr(rm), ptr(rv),
                                              None, ptr(bn_save), N, D, 0.1, 1e-5, 1, 0, S[0]),
                                 {}),
        "gine_mp_bwd_finalize": (lambda: call("gine_mp_bwd_finalize", ptr(mp_part), Pm, D,
                                              ptr(lw_g), ptr(lb_g), ptr(eps_g), S[0]), {}),
    }

    # the LDS-window forward (GINE_MP_WINDOW=all), for comparison with the gather forward
    from raincast_gnn.graph import plan_windows
    fwin = plan_windows(g.in_rowptr, g.in_src, N, dev, 128).get(32)
    if fwin is not None:
        fplan = fwin[0]
        kernels["gine_mp_fwd_win"] = (
            lambda: call("gine_mp_fwd_win", ptr(x), ptr(g.in_rowptr), ptr(g.in_src),
                         ptr(g.in_attr), ptr(lw), ptr(lb), ptr(ep), ptr(z), N, D, lin,
                         ctypes.byref(fplan), S[0]),
            {"bytes": 4 * (2 * N * D + 2 * E + N + 1)})

    def mp_fwd_mlp1():  # the fused forward (gather + Linear1 + BN partials)
        call("gine_mp_fwd_mlp1", ptr(x), ptr(g.in_rowptr), ptr(g.in_src), ptr(g.in_attr),
             ptr(lw), ptr(lb), ptr(ep), ptr(w1), ptr(b1), ptr(z), ptr(a1), ptr(partials), N,
             D, g.max_in_degree, lin, S[0])

    if Fn.fused_forward_ok(g, N, D):  # what the training step's forward runs at this size
        kernels["gine_mp_fwd_mlp1"] = (mp_fwd_mlp1, {
            "flops": 2 * N * D * D, "bytes": 4 * (2 * N * D + 2 * E + N + 1) + 4 * N * D})

    def mp_bwd_mlp_wgrad():  # the window backward + the node-MLP weight-gradient engine
        call("gine_mp_bwd_win_mlp_wgrad", ptr(dz), ptr(x), ptr(g.out_rowptr), ptr(g.out_dst),
             ptr(g.out_attr), ptr(lw), ptr(lb), ptr(ep), ptr(dz), ptr(dx), ptr(win_part), N, D,
             1 | lin, ctypes.byref(win), ptr(dz), None, ptr(mask), ptr(a1), ptr(bn_save),
             ptr(dbn), ptr(coef), ptr(z), ptr(slab), 2, S[0])

    # the one-launch layer forward (fused gather + Linear1 + BN sums | grid barrier | BN
    # finish + Linear2 + residual epilogue) where the step runs it, on an accumulator of its
    # own (each launch is a paired producer + consumer)
    if Fn.fused_forward_ok(g, N, D) and Fn.layer_forward_ok(N, D, g.max_in_degree):
        words = Fn._count64("gine_bn_acc_words", D)
        lacc = torch.zeros(words, dtype=torch.int64, device=dev)
        y_l = torch.empty_like(x)
        bsave_l = torch.empty(4, D, device=dev)
        rm_l, rv_l = torch.zeros(D, device=dev), torch.ones(D, device=dev)

        def mp_fwd_layer():
            call("gine_mp_fwd_layer", ptr(x), ptr(g.in_rowptr), ptr(g.in_src), ptr(g.in_attr),
                 ptr(lw), ptr(lb), ptr(ep), ptr(w1), ptr(b1), ptr(z), ptr(a1), ptr(lacc),
                 ptr(bn.weight), ptr(bn.bias), ptr(rm_l), ptr(rv_l), None, ptr(bsave_l), 0.1,
                 1e-5, 1, ptr(w2), ptr(b2), ptr(y_l), ptr(mask), N, D, g.max_in_degree, lin, 2,
                 *Fn.layer_window_args(g), None, S[0])
        # bytes: the message passing's B_f + a1 and y written, mask, x re-read for the residual
        kernels["gine_mp_fwd_layer"] = (mp_fwd_layer, {
            "flops": 4 * N * D * D,
            "bytes": 4 * (2 * N * D + 2 * E + N + 1) + 4 * N * D + 4 * N * D + N * D + 4 * N * D})

    if Fn.engine_in_mp_ok(g, D) and options.BN_ACC_BWD:
        # the backward's BatchNorm-accumulator pair (dbn GEMM + sums | BN finish + dz GEMM):
        # two launches that must run as a pair on their accumulator, timed together
        bacc = torch.zeros(Fn._count64("gine_bn_acc_words", D), dtype=torch.int64, device=dev)
        dg, dbt = torch.empty(D, device=dev), torch.empty(D, device=dev)

        def mlp_bwd_pair_acc():
            call("gine_mlp_bwd2_acc", ptr(dz), None, ptr(mask), ptr(a1), ptr(bn_save), ptr(w2),
                 ptr(dbn), None, ptr(bacc), N, D, 2, S[0])
            call("gine_mlp_bwd1_bn", ptr(dbn), ptr(a1), ptr(bn_save), ptr(bacc), ptr(bn.weight),
                 ptr(dg), ptr(dbt), ptr(coef), ptr(w1), ptr(dx), N, D, S[0])
        kernels["gine_mlp_bwd_pair_acc"] = (mlp_bwd_pair_acc, {
            "flops": 4 * N * D * D, "bytes": 25 * N * D})

        if Fn.layer_backward_ok(N, D):  # the pair in one launch, as the step runs it
            lbacc = torch.zeros(Fn._count64("gine_bn_acc_words", D), dtype=torch.int64,
                                device=dev)

            def mlp_bwd_layer():
                call("gine_mlp_bwd_layer", ptr(dz), None, ptr(mask), ptr(a1), ptr(bn_save),
                     ptr(w2), ptr(dbn), ptr(lbacc), ptr(bn.weight), ptr(dg), ptr(dbt),
                     ptr(coef), ptr(w1), ptr(dx), N, D, 2, S[0])
            kernels["gine_mlp_bwd_layer"] = (mlp_bwd_layer, {
                "flops": 4 * N * D * D, "bytes": 25 * N * D})

    if Fn.engine_in_mp_ok(g, D):  # what the training step's backward runs at this size
        # bytes: the message-passing backward's B_b (dz, x, dx, CSR, dres = dy) + the
        # engine's other operands read once (mask u8, dbn, a1, z) + its fp32 slab
        kernels["gine_mp_bwd_mlp_wgrad"] = (mp_bwd_mlp_wgrad, {
            "flops": 4 * N * D * D,
            "bytes": 4 * (3 * N * D + 2 * E + N + 1) + 4 * N * D + 13 * N * D
                     + 4 * slab.numel()})
    out = {}
    for name, (fn, work) in kernels.items():
        for _ in range(3):
            fn()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(reps):
            fn()
        ev1.record(stream)
        ev1.synchronize()
        us = ev0.elapsed_time(ev1) * 1e3 / reps
        # the same launches captured in one HIP graph: no host launch gaps, the way the
        # training step runs them
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        graph = torch.cuda.CUDAGraph()
        S[0] = side.cuda_stream
        with torch.cuda.graph(graph, stream=side):
            for _ in range(reps):
                fn()
        S[0] = sh
        stream.wait_stream(side)
        graph.replay()
        ev0.record(stream)
        graph.replay()
        ev1.record(stream)
        ev1.synchronize()
        us_graph = ev0.elapsed_time(ev1) * 1e3 / reps
        rec = {"us": round(us, 3), "us_graph": round(us_graph, 3)}
        if "bytes" in work:
            rec["alg_bytes"] = work["bytes"]
            rec["GBps"] = round(work["bytes"] / us * 1e-3, 1)
        if "flops" in work:
            rec["alg_flops"] = work["flops"]
            rec["TFLOPps"] = round(work["flops"] / us * 1e-6, 2)
        out[name] = rec
    return out


STEP_KERNELS = ("gine_mp_fwd", "gine_mp_bwd", "gine_mlp_fwd1", "gine_mlp_fwd2",
                "gine_mlp_bwd2", "gine_mlp_bwd1_wgrad")  # each runs once per GINE layer
# ... or, where the fused forward applies (raincast_gnn.functional.fused_forward_ok):
FUSED_STEP_KERNELS = ("gine_mp_fwd_mlp1", "gine_mp_bwd", "gine_mlp_fwd2", "gine_mlp_bwd2",
                      "gine_mlp_bwd1_wgrad")


def sec8d_work(N: int, E: int, D: int) -> dict:
    """SURVEY.md 8(d)'s algorithmic quantities per GINE layer: B_f (read h once, src index
    and attribute per edge, rowptr, write z), B_b (read dz, read h for the ReLU mask, write
    dh, dst index + attribute per edge, rowptr) and the node-MLP flops (fwd 4ND^2, bwd
    8ND^2, of which the weight gradients are 4ND^2)."""
    return {"B_f": 4 * (2 * N * D + 2 * E + N + 1), "B_b": 4 * (3 * N * D + 2 * E + N + 1),
            "mlp_fwd_flops": 4 * N * D * D, "mlp_bwd_flops": 8 * N * D * D}


# per entry point: its 8(d) work per launch (bytes, flops) -- only what 8(d) counts:
# message-passing bytes for the gather / scatter kernels, GEMM flops for the node MLP
# (operands of a GEMM re-read from L2, split-K slabs and the residual-gradient read are
# NOT algorithmic work; they show up in `traffic`)
def sec8d_launch_work(name: str, w: dict) -> dict:
    half_fwd, half_bwd = w["mlp_fwd_flops"] // 2, w["mlp_bwd_flops"] // 4
    return {
        "gine_mp_fwd": {"bytes": w["B_f"]}, "gine_mp_fwd_win": {"bytes": w["B_f"]},
        "gine_mp_bwd": {"bytes": w["B_b"]},
        "gine_mp_fwd_mlp1": {"bytes": w["B_f"], "flops": half_fwd},
        "gine_mp_fwd_layer": {"bytes": w["B_f"], "flops": 2 * half_fwd},
        "gine_mlp_bwd_pair_acc": {"flops": 2 * half_bwd},
        "gine_mlp_bwd_layer": {"flops": 2 * half_bwd},
        "gine_mp_bwd_mlp_wgrad": {"bytes": w["B_b"], "flops": 2 * half_bwd},
        "gine_mlp_fwd1": {"flops": half_fwd}, "gine_mlp_fwd2": {"flops": half_fwd},
        "gine_mlp_bwd2": {"flops": half_bwd}, "gine_mlp_bwd1": {"flops": half_bwd},
        "gine_mlp_bwd1_wgrad": {"flops": 3 * half_bwd},
        "gine_mlp_wgrad": {"flops": 2 * half_bwd},
    }.get(name, {})


MALL_BYTES = 256 * 1024 * 1024  # MI355X Infinity Cache (MALL)


def roofline_for(kernels: dict, layers: int, work: dict, config: str = "cfg2"):
    """The dominant kernel of the step (largest time per step among the per-layer kernels
    the training step launches) against SURVEY.md 8(d)'s roofline: its ideal time is
    max(8(d) bytes / 8 TB/s, 8(d) flops / 157.3 TFLOP/s fp32 MFMA), frac = ideal / measured
    average launch time; `achieved` is the binding quantity per second."""
    step = list(FUSED_STEP_KERNELS if "gine_mp_fwd_mlp1" in kernels else STEP_KERNELS)
    if "gine_mp_bwd_mlp_wgrad" in kernels:  # engine in the message-passing launch
        step = [k for k in step if k not in ("gine_mp_bwd", "gine_mlp_bwd1_wgrad")]
        step += ["gine_mlp_bwd1", "gine_mp_bwd_mlp_wgrad"]
    if "gine_mp_fwd_layer" in kernels:  # the whole layer forward in one launch
        step = [k for k in step if k not in ("gine_mp_fwd_mlp1", "gine_mlp_fwd2")]
        step += ["gine_mp_fwd_layer"]
    if "gine_mlp_bwd_pair_acc" in kernels:  # (two launches: a pair, not a roofline line)
        step = [k for k in step if k not in ("gine_mlp_bwd2", "gine_mlp_bwd1")]
    if "gine_mlp_bwd_layer" in kernels:  # the pair in one launch
        step += ["gine_mlp_bwd_layer"]
    timed = [k for k in step if k in kernels]
    # the kernels table also times launches the step does not run (the pair forms, the
    # stand-alone gather / GEMM / finalize entry points): marked, for context only
    for k, rec in kernels.items():
        rec["in_step"] = k in timed
    dominant = max(timed, key=lambda k: kernels[k]["us"])
    out = roof_of(dominant, kernels[dominant], layers, work, config)
    # the other per-layer launches of the step against their own 8(d) floors, for context
    out["per_layer_launches"] = {
        k: {"avg_us": kernels[k]["us"],
            "frac": roof_of(k, kernels[k], layers, work, config)["frac"]}
        for k in timed + [k for k in ("gine_mlp_bwd_pair_acc",) if k in kernels]}
    return out


def roof_of(name: str, rec: dict, layers: int, work: dict, config: str = "cfg2") -> dict:
    wl = sec8d_launch_work(name, work)
    b, f = wl.get("bytes", 0), wl.get("flops", 0)
    t_hbm = b / (HBM_PEAK_GBS * 1e9)
    t_mfma = f / (FP32_MFMA_PEAK_TFLOPS * 1e12)
    sec = rec["us"] * 1e-6
    if t_mfma > t_hbm:
        roof = {"kernel": name, "bound": "mfma", "achieved": round(f / sec * 1e-12, 2),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                # the same flops against the split-bf16x3 instructions' own ceiling (the
                # fp32 peak flatters an MFMA-bound frac by 16/6)
                "peak_executed": BF16X3_EXEC_PEAK_TFLOPS,
                "frac_executed": round(f / sec * 1e-12 / BF16X3_EXEC_PEAK_TFLOPS, 4)}
    else:
        roof = {"kernel": name, "bound": "hbm", "achieved": round(b / sec * 1e-9, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    roof["frac"] = round(max(t_hbm, t_mfma) / sec, 4)
    roof["alg_bytes_per_launch"] = b
    roof["alg_flops_per_launch"] = f
    roof["avg_us"] = rec["us"]
    roof["launches_per_step"] = layers
    t = pmc_traffic(name, config)
    roof["traffic"] = t["bytes"] if t else None
    roof["traffic_source"] = t["source"] if t else None
    roof["traffic_tree"] = t["tree"] if t else None
    return roof


def roofline_step(work: dict, layers: int, ms_per_step: float) -> dict:
    """SURVEY.md 8(d)'s per-step figure: sum over layers of (B_f + B_b) / step time, against
    HBM (the message-passing bytes of the whole step; the rest of the step -- DeepSet,
    dense chain, node-MLP GEMMs, head, loss, optimizer -- is time without 8(d) bytes)."""
    b = (work["B_f"] + work["B_b"]) * layers
    gbs = b / (ms_per_step * 1e-3) * 1e-9
    return {"bytes_per_step": b, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}


def roofline_mp(kernels: dict, layers: int, work: dict, config: str = "cfg2"):
    """The message-passing kernels (the north-star gather / segmented-scatter path) alone
    against HBM, with the measured copy ceiling beside the 8 TB/s spec."""
    out = {}
    for name in ("gine_mp_fwd", "gine_mp_fwd_win", "gine_mp_bwd"):
        if name in kernels:
            out[name] = roof_of(name, kernels[name], layers, work, config)
    return out or None


def copy_ceiling_gbps(device, nbytes=1 << 30, reps=10):
    """Measured HBM ceiling: a 1 GiB device-to-device copy by gine_copy_f4 (16-byte-per-lane
    streaming loads and stores, csrc/gine_probe.hip -- MI355X_MICROARCH.md's measured copy
    form), read + write bytes per second, on the current stream."""
    from raincast_gnn import _lib
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(device)
    s = _lib.stream_handle(device)

    def copy():
        _lib.call("gine_copy_f4", _lib.ptr(src), _lib.ptr(dst), nbytes, s)
    copy()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        copy()
    ev1.record(stream)
    ev1.synchronize()
    sec = ev0.elapsed_time(ev1) * 1e-3 / reps
    ok = torch.equal(dst[:1024], src[:1024]) and torch.equal(dst[-1024:], src[-1024:])
    del src, dst
    if not ok:
        raise RuntimeError("gine_copy_f4 copied wrong data")
    return round(2 * nbytes / sec / 1e9, 1)


# entry point -> the kernels one call launches (names as in the rocprofv3 PMC summary; D=128,
# the residual epilogue of layers >= 1).  A tuple lists alternatives: the first kernel the
# summary holds is the one the configuration ran (gine_mp_bwd: the window kernel where the
# graph has a plan, the gather kernel otherwise -- cfg5).
PMC_KERNELS = {
    "gine_mp_fwd": ["gine::k_mp_fwd<32, 1, "],
    "gine_mp_fwd_mlp1": ["gine::k_mp_fwd_mlp1<"],
    "gine_mp_fwd_layer": ["gine::k_mp_fwd_layer<false, 5>"],
    "gine_mlp_bwd_layer": ["gine::k_mlp_bwd_layer<5>"],
    # (the GPU box's host rounds the edge Linear mul-then-add: FMA = false)
    "gine_mp_bwd_mlp_wgrad": ["gine::k_mp_bwd_win<32, false, true, 5>"],
    "gine_mp_bwd": [("gine::k_mp_bwd_win<32, ", "gine::k_mp_bwd<32, 1, ")],
    "gine_mlp_fwd1": ["gine::k_rowgemm<128, 0, 0, true>"],
    "gine_mlp_fwd2": ["gine::k_rowgemm<128, 1, 5, true>"],
    "gine_mlp_bwd2": ["gine::k_rowgemm<128, 5, 2, false>"],
    "gine_mlp_bwd1": ["gine::k_rowgemm<128, 3, 3, false>"],
    "gine_mlp_bwd1_wgrad": ["gine::k_bwd1_wgrad<5>"],
    "gine_mlp_wgrad": ["gine::k_wgrad_engine<gine::MlpWgradSrc<5>, 64, 8>",
                       "gine::k_slab_sum<true, gine::MlpWgradOut>"],
}


def source_tree_hash() -> str:
    """sha256 (first 16 hex digits) of the sources the library is built from (csrc/*.hip,
    *.hpp, the Makefile, include/gine_hip.h): the tree a PMC traffic summary was collected
    on must be this one for its bytes to be reported (tools/pmc_summary.py --tree-hash)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "raincast-gnn_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))
                   + [os.path.join(csrc, "Makefile"), os.path.join(ROOT, "include", "gine_hip.h")])
    for path in files:
        h.update(os.path.relpath(path, ROOT).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel: str, config: str = "cfg2"):
    """HBM bytes per call of entry point ``kernel`` from the committed rocprofv3 PMC summary
    (profiles/*pmc_traffic.json: per-kernel (2 x FETCH_SIZE + WRITE_SIZE) bytes per launch,
    the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md), summed over the kernels the
    call launches; None when no summary of THIS configuration AND THIS source tree covers
    them (a summary names its configuration in "_config" -- untagged: cfg2 -- and the
    source_tree_hash() it was collected on in "_tree"; a summary of another tree is not
    used)."""
    names = PMC_KERNELS.get(kernel)
    if not names:
        return None
    tree = source_tree_hash()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")),
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("_config", "cfg2") != config or d.get("_tree") != tree:
            continue
        hits = [next((v for alt in (n if isinstance(n, tuple) else (n,))
                      for k, v in d.items() if k.startswith(alt)), None) for n in names]
        if all(h is not None for h in hits):
            return {"bytes": int(sum(hits)), "source": os.path.basename(path), "tree": tree}
    return None


# -----------------------------------------------------------------------------------------
# CPU baseline (oracle, rank 0, N=1)
# -----------------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(cfg, graphs, seconds):
    """The oracle (CPU restatement of the reference's training step) on this host: all
    threads torch uses, then one thread for a quarter of the time."""
    from oracle import gine_cpu as O
    params = cfg.params()
    torch.manual_seed(42)
    model = O.OracleGNN(35, params["gnn_hidden"], params["gnn_layers"], params["loss"],
                        params["grad_u"], params["u"], params["xi"]).train()
    opt = torch.optim.AdamW(model.parameters(), lr=params["lr"])
    batch = synthetic_batch(cfg.num_stations, graphs, k=cfg.k, seed=1000)

    def step():
        opt.zero_grad()
        loss = model.crps(model(batch), batch.y)
        loss.backward()
        opt.step()

    def run(limit):
        step()  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            step()
            n += 1
            el = time.perf_counter() - t0
            if el >= limit or n >= 200:
                return n, el

    # threads: the cores this process may use.  On the GPU pool one GPU's job gets a 16-CPU
    # share (OMP_NUM_THREADS=16 is set there and the pool asks that it be left as is), so
    # torch's intra-op pool is that share even when the affinity mask shows every CPU.
    threads = torch.get_num_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    n, el = run(seconds)
    torch.set_num_threads(1)
    try:
        n1, el1 = run(seconds / 4)
    finally:
        torch.set_num_threads(threads)
    return {"value": round(graphs * n / el, 3), "unit": "graphs/s",
            "cores": threads, "kind": "port",
            "sample": f"{n} full training steps (oracle CPU restatement, fp32) on the cfg "
                      f"{cfg.name} batch of {graphs} graphs x {cfg.num_stations} stations, "
                      f"after 1 warm-up step; {el:.1f} s on {threads} threads; "
                      f"cpu={cpu_model()}",
            "ms_per_step": round(el / n * 1e3, 2),
            "host": {"cpu_count": os.cpu_count(), "affinity_cpus": affinity,
                     "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                     "threads_used": threads,
                     "why": "torch intra-op threads = the job's CPU share (OMP_NUM_THREADS, "
                            "set by the GPU pool: 16 CPUs per GPU); the affinity mask and "
                            "cpu_count show the whole host"},
            "one_thread": {"value": round(graphs * n1 / el1, 3), "unit": "graphs/s",
                           "steps": n1, "seconds": round(el1, 1)}}


# -----------------------------------------------------------------------------------------
def measure(cfg, graphs_per_rank, args, device, rank, world):
    """Build the trainer, warm up, capture, then time ``args.steps`` steps between barriers
    + synchronisations; returns (trainer, max-over-ranks seconds, HIP-event percentiles)."""
    tr = Trainer(cfg, device, rank, world, graphs_per_rank, args.allreduce,
                 args.force_allreduce, args.station_order)
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        for _ in range(max(args.warmup, 2)):
            tr.eager_step()
    torch.cuda.current_stream(device).wait_stream(side)
    torch.cuda.synchronize(device)
    if not args.no_graph:
        tr.capture()
        for _ in range(2):
            tr.step()
    # clock settle (--settle-steps): untimed replays until the GPU runs at its training-steady
    # clock; the same count on every rank (the N > 1 step holds a collective)
    for _ in range(max(0, args.settle_steps)):
        tr.step()
    torch.cuda.synchronize(device)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    # HIP events between steps on the stream the steps run on (distribution only; the
    # reported time is the wall clock between the synchronised barriers)
    stream = torch.cuda.current_stream(device)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    tr.ar_events = []
    thr0 = cpu_throttle()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        tr.step()
        evs[i + 1].record(stream)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    thr = throttle_delta(thr0, cpu_throttle())
    Fn.check_grid_barriers()  # a layer launch whose grid was not co-resident raises here
    in_order = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    per_step = sorted(in_order)
    pct = {q: round(per_step[min(len(per_step) - 1, int(q / 100 * len(per_step)))], 4)
           for q in (10, 50, 90)}
    # the split all-reduce alone (between the fwd+bwd and AdamW graphs), per step: on the
    # stream (HIP events) and on the host (the collective call itself)
    ar_steps = [(b.elapsed_time(c), h, sy, a.elapsed_time(b))
                for a, b, c, h, sy in tr.ar_events]
    ar = sorted(t[0] for t in ar_steps)
    tr.ar_events = None
    pct["allreduce_p50"] = round(ar[len(ar) // 2], 4) if ar else None
    pct["stalls"] = stalled_steps(in_order, ar_steps)
    pct["cpu_throttle"] = thr
    if world > 1:
        own = elapsed
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        st = pct["stalls"]
        pct["per_rank"] = gather_per_rank(pct[50], pct["allreduce_p50"], world, device,
                                          step_max=per_step[-1],
                                          stalls=st["count"] if st else 0,
                                          wall_ms=own / args.steps * 1e3,
                                          events_ms=sum(in_order) / len(in_order),
                                          gpu=device.index if device.type == "cuda" else -1)
        check_rank_devices(pct["per_rank"], args)
    return tr, elapsed, pct


def check_rank_devices(per_rank, args) -> None:
    """RCCL runs one rank per GPU: every rank's device must differ (LOCAL_RANK -> GPU), and
    the group must hold exactly --gpus ranks.  gloo rehearsals may put
    several ranks on one GPU."""
    assert len(per_rank) == args.gpus, (len(per_rank), args.gpus)
    if args.dist_backend == "nccl" and not args.dry_run:
        gpus = [r["gpu"] for r in per_rank]
        assert len(set(gpus)) == len(gpus), f"ranks share a GPU under RCCL: {gpus}"


def stalled_steps(in_order, ar_steps):
    """Steps that took more than 10x the median (and over 1 ms): their index, time, and the
    all-reduce's stream / host time in that step -- so that one stall (seen with two ranks
    sharing one GPU over gloo) is reported beside the wall-clock value instead of silently
    defining it.  None when there is none."""
    if not in_order:
        return None
    med = sorted(in_order)[len(in_order) // 2]
    bad = [i for i, t in enumerate(in_order) if t > max(10 * med, 1.0)]
    if not bad:
        return None
    out = {"threshold_ms": round(max(10 * med, 1.0), 4), "count": len(bad),
           "total_ms": round(sum(in_order[i] for i in bad), 3), "steps": []}
    for i in bad[:8]:
        rec = {"step": i, "ms": round(in_order[i], 3)}
        if i < len(ar_steps):
            ar_ms, host_ms, sync_ms, fb_ms = ar_steps[i]
            rec["fwd_bwd_stream_ms"] = round(fb_ms, 3)  # the fwd+bwd graph on the stream
            if sync_ms is not None:  # host wait for it before the gloo collective
                rec["fwd_bwd_host_wait_ms"] = round(sync_ms, 3)
            rec["allreduce_stream_ms"] = round(ar_ms, 3)
            rec["allreduce_host_ms"] = round(host_ms, 3)
        out["steps"].append(rec)
    rest = [t for i, t in enumerate(in_order) if i not in set(bad)]
    out["ms_per_step_other_steps"] = round(sum(rest) / len(rest), 4) if rest else None
    return out


def _cgroup_file(name: str):
    for d in ("/sys/fs/cgroup", "/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        f = os.path.join(d, name)
        if os.path.exists(f):
            return f
    return None


def cpu_share() -> int:
    """CPUs this job may use: the cgroup quota (cpu.max or cpu.cfs_quota_us / period), else
    OMP_NUM_THREADS, else the affinity mask (os.cpu_count() on the GPU boxes shows the whole
    machine, many times the job's share)."""
    try:
        f = _cgroup_file("cpu.max")
        if f:
            q, per = open(f).read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(per)))
        fq, fp = _cgroup_file("cpu.cfs_quota_us"), _cgroup_file("cpu.cfs_period_us")
        if fq and fp and int(open(fq).read()) > 0:
            return max(1, int(int(open(fq).read()) / int(open(fp).read())))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        return int(omp)
    return len(os.sched_getaffinity(0))


def cpu_throttle():
    """The cgroup's CPU-throttling counters {nr_throttled, throttled_usec} (None when the
    cgroup does not expose them): read before and after the timed steps, their difference
    says whether the job's CPU quota was throttled while it ran."""
    f = _cgroup_file("cpu.stat")
    if not f:
        return None
    out = {}
    try:
        for line in open(f):
            k, v = line.split()[:2]
            if k in ("nr_throttled", "throttled_usec", "throttled_time", "nr_periods"):
                out[k] = int(v)
    except (OSError, ValueError):
        return None
    return out or None


def throttle_delta(a, b):
    if not a or not b:
        return None
    return {k: b[k] - a[k] for k in b if k in a}


def gather_per_rank(step_p50, allreduce_p50, world, device, step_max=None, stalls=0,
                    wall_ms=None, events_ms=None, gpu=-1):
    """Every rank's p50 step time, p50 all-reduce time, slowest step (ms) and stalled-step
    count, for the N > 1 line's decomposition (a tensor all_gather: on the GPU over RCCL, on
    the CPU over gloo)."""
    def opt(v):
        return -1.0 if v is None else float(v)
    mine = torch.tensor([step_p50, opt(allreduce_p50), opt(step_max), float(stalls),
                         opt(wall_ms), opt(events_ms), float(gpu)],
                        device=device if dist.get_backend() == "nccl" else "cpu",
                        dtype=torch.float64)
    every = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)

    def val(x, nd=4):
        return round(x.item(), nd) if x.item() >= 0 else None
    # wall_ms_per_step: this rank's own wall clock between the synchronised barriers (the
    # line's ms_per_step is the max over ranks); events_ms_per_step: the mean of its HIP-event
    # step times -- the two reconcile when the host kept the stream fed
    return [{"rank": r, "step_ms_p50": round(v[0].item(), 4),
             "allreduce_ms_p50": val(v[1]), "step_ms_max": val(v[2]),
             "stalled_steps": int(v[3].item()),
             "wall_ms_per_step": val(v[4]), "events_ms_per_step": val(v[5]),
             "gpu": int(v[6].item()) if v[6].item() >= 0 else None}
            for r, v in enumerate(every)]


# -----------------------------------------------------------------------------------------
# multi-rank launch: one process per GPU
# -----------------------------------------------------------------------------------------
LAUNCH_ENV = "RAINCAST_BENCH_LAUNCHED"


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nranks: int, argv: list) -> int:
    """``python bench.py --gpus N`` without a torchrun environment: start N fresh child
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per GPU)
    and return the worst exit status.  The parent makes no HIP call -- it only waits:
    children inherit stdout, and rank 0 prints the one JSON line.  When a child fails,
    the others get a grace period to finish (or notice the broken group), then are
    terminated by PID."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env[LAUNCH_ENV] = "1"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    try:
        deadline = None
        while any(p.poll() is None for p in procs):
            if deadline is None and any(p.returncode not in (None, 0) for p in procs):
                deadline = time.monotonic() + 60.0
                log("bench launcher: a rank failed; waiting 60 s for the others")
            if deadline is not None and time.monotonic() > deadline:
                stop()
                for p in procs:
                    try:
                        p.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                break
            time.sleep(0.2)
        for p in procs:
            p.wait()
    finally:
        signal.signal(signal.SIGTERM, old)
    rcs = [p.returncode for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log(f"bench launcher: rank exit codes {rcs}")
        # a signal death (negative) counts as failure with the shell's 128+signal code
        return max((128 - rc) if rc < 0 else rc for rc in bad)
    return 0


def dry_run(args, rank: int, world: int) -> None:
    """CPU rehearsal of the N-rank bench: gloo group, per-rank synthetic shard of the
    configuration, the step's gradient all-reduce (the flat fp32 buffer of the model) timed
    between barriers, max over ranks, rank 0's JSON line.  No GPU work."""
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    if os.environ.get("RAINCAST_BENCH_DRY_FAIL_RANK") == str(rank):  # launcher test hook
        raise SystemExit(7)
    cfg = BENCH_CONFIGS[args.config].with_hidden(args.hidden)
    graphs_per_rank = (cfg.graphs_per_gpu // world if args.config == 4 else cfg.graphs_per_gpu)
    params = cfg.params()
    torch.manual_seed(42)
    model = gnn_from_params(params).train()
    broadcast_parameters(model)
    n_params = sum(p.numel() for p in model.parameters())
    reducer = FlatGradReducer(model.parameters())
    shard = synthetic_batch(cfg.num_stations, graphs_per_rank, k=cfg.k, seed=1000 + rank)
    for _ in range(args.warmup):
        reducer.all_reduce_()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    per = []
    for _ in range(args.steps):
        reducer.flat.fill_(float(rank + 1))
        t1 = time.perf_counter()
        reducer.all_reduce_()
        per.append((time.perf_counter() - t1) * 1e3)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ar_p50 = sorted(per)[len(per) // 2] if per else None
    per_rank = gather_per_rank(ar_p50, ar_p50, world, "cpu") if world > 1 else None
    expect = (world + 1) / 2.0  # mean over ranks of (rank + 1)
    assert torch.allclose(reducer.flat, torch.full_like(reducer.flat, expect)), "all-reduce"
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        nodes = torch.tensor([shard.num_nodes], dtype=torch.int64)
        dist.all_reduce(nodes)
        nodes_total = int(nodes)
    else:
        nodes_total = shard.num_nodes
    elapsed = float(t)
    if rank == 0:
        print(json.dumps({
            "metric": "dry run: gradient all-reduce only (no GPU step)",
            "value": round(graphs_per_rank * world * args.steps / elapsed, 2),
            "unit": "graphs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if args.config == 4 else "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic", "dry_run": True,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "rccl_world_size": None, "launcher": os.environ.get(LAUNCH_ENV) == "1",
            "config": {"workload": cfg.name, "global_batch": graphs_per_rank * world,
                       "graphs_per_gpu": graphs_per_rank, "nodes_global": nodes_total,
                       "allreduce_floats": reducer.numel, "parameters": n_params,
                       "parallelism": f"dp{world}"},
            "allreduce_ms_p50": round(ar_p50, 4) if ar_p50 is not None else None,
            "host_threads_per_rank": torch.get_num_threads(), "cpu_share": cpu_share(),
            "per_rank": per_rank}), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def dropin_bench(args, cfg, device) -> dict:
    """The reference's own training loop (train.py:61-71) over the reference's model
    structure with only GINEConv swapped (raincast_gnn.dropin.ReferenceStructGNN: torch
    DeepSet / dim_red / ResGnn activations / aggr / PostProcess / CRPS, torch AdamW): every
    step copies a host batch to the device (``batch.to(device)``: a fresh edge_index tensor
    each step), runs forward, loss, backward, optimizer step and ``loss.item()``.  Host
    batches are pre-collated (the DataLoader's collation is host work that this timing
    leaves out).  The GINE share is the conv stack's forward + backward timed alone on the
    same device inputs, also with a fresh edge_index tensor per step."""
    from raincast_gnn.data import collate, synthetic_samples
    from raincast_gnn.dropin import reference_struct_from_params
    from raincast_gnn.graph import graph_cache
    params = cfg.params()
    graphs = cfg.graphs_per_gpu
    torch.manual_seed(42)
    model = reference_struct_from_params(params).to(device).train()
    opt = torch.optim.AdamW(model.parameters(), lr=params["lr"])
    samples = synthetic_samples(cfg.num_stations, 2 * graphs, k=cfg.k, seed=1000)
    host = [collate(samples[:graphs]), collate(samples[graphs:])]

    def step(i):
        batch = host[i % 2].to(device)                      # train.py:62
        preds = model(batch)                                # train.py:64
        loss = model.loss_fn.crps(preds, batch.y)           # train.py:65
        opt.zero_grad()                                     # train.py:67-69
        loss.backward()
        opt.step()
        return loss.item()                                  # train.py:71

    for i in range(max(args.warmup, 2)):
        step(i)
    torch.cuda.synchronize(device)
    stats0 = dict(graph_cache.stats)
    t0 = time.perf_counter()
    total = 0.0
    for i in range(args.steps):
        total += step(i)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    stats = {k: graph_cache.stats[k] - stats0[k] for k in stats0}

    # the GINE stack alone (4 GINEConv + torch ReLU / residual), forward + backward, with
    # the training loop's set_to_none gradients; every step gets edge tensors of its own
    # (copied to the device before the timed region: a fresh tensor per step as in the
    # loop above, without the host-to-device copy that the whole-step number holds)
    D = params["gnn_hidden"]
    x0 = torch.randn(host[0].num_nodes, D, device=device, requires_grad=True)
    gy = torch.randn(host[0].num_nodes, D, device=device)
    edges = [(host[i % 2].edge_index.to(device), host[i % 2].edge_attr.to(device))
             for i in range(args.steps + 3)]

    def gine_step(i):
        model.conv.zero_grad(set_to_none=True)
        x0.grad = None
        ei, ea = edges[i]
        out = model.conv(x0, ei, ea)
        out.backward(gy)

    for i in range(3):
        gine_step(args.steps + i)
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    for i in range(args.steps):
        gine_step(i)
    torch.cuda.synchronize(device)
    gine_ms = (time.perf_counter() - t1) / args.steps * 1e3
    ms = elapsed / args.steps * 1e3
    return {"metric": "training graphs/s, drop-in path (models/gnn.py structure in torch, "
                      "raincast_gnn GINEConv, train.py loop with batch.to(device) and "
                      "loss.item() every step)",
            "value": round(graphs * args.steps / elapsed, 2), "unit": "graphs/s",
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (host batches)",
            "config": {"workload": f"{cfg.name}-dropin: {graphs} graphs x {cfg.num_stations} "
                                   f"stations, k={cfg.k}, {params['gnn_layers']} GINE layers, "
                                   f"D={D}", "global_batch": graphs},
            "gine_stack_ms_fwd_bwd": round(gine_ms, 4),
            "gine_share_of_step": round(gine_ms / ms, 4),
            "graph_cache_per_timed_steps": stats,
            "mean_loss": total / args.steps}


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, started before anything here touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank, local_rank, world = env_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started {world} rank(s) "
                         f"(WORLD_SIZE); they must agree")
    # the host's CPU share split over the ranks on it, before any GPU call: N ranks x
    # OMP_NUM_THREADS intra-op threads on one share oversubscribe it (the
    # N > 1 rehearsals' host-side stalls inside the collective)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world) or world)
    threads = max(1, cpu_share() // max(1, local_world))
    torch.set_num_threads(threads)
    if args.dry_run:
        return dry_run(args, rank, world)
    if world > 1 or args.force_allreduce:
        if world == 1:  # a forced 1-rank group outside a launcher: its own rendezvous
            for k, v in (("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0"),
                         ("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(_free_port()))):
                os.environ.setdefault(k, v)
        dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and local_rank >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but only {ndev} GPU(s) "
                         f"visible; RCCL needs one GPU per rank")
    device = torch.device("cuda", local_rank % max(1, ndev))
    torch.cuda.set_device(device)
    # ranks sharing one GPU (gloo rehearsals) keep the one-launch layer forward off: its grid
    # barrier needs the whole chip (raincast_gnn.functional.layer_forward_ok)
    note_device_sharing()
    cfg = BENCH_CONFIGS[args.config].with_hidden(args.hidden)
    if args.no_head_fold:
        options.HEAD_FOLD = False
    if args.dropin:
        if world > 1:
            raise SystemExit("--dropin measures the single-GPU drop-in path (--gpus 1)")
        print(json.dumps(dropin_bench(args, cfg, device)), flush=True)
        return
    if args.config == 4:  # global batch fixed -> strong scaling
        graphs_per_rank = cfg.graphs_per_gpu // world
        scaling = "strong"
    else:
        graphs_per_rank = cfg.graphs_per_gpu
        scaling = "weak"
    tr, elapsed, pct = measure(cfg, graphs_per_rank, args, device, rank, world)
    # flag MALL residency when the step's working set is under the 256 MB
    # Infinity Cache -- the peak of live device allocations over the measured steps (inputs,
    # parameters, saved activations, workspaces) is the working-set bound used here
    working_set = torch.cuda.max_memory_allocated(device)
    layers = tr.params["gnn_layers"]
    E_rank = tr.batch.edge_index.size(1)
    loss_val = float(tr.loss.item()) if tr.loss is not None else float("nan")

    graphs_global = graphs_per_rank * world
    edges_global = E_rank * world
    ms = elapsed / args.steps * 1e3
    value = graphs_global * args.steps / elapsed
    edges_per_s = edges_global * layers * args.steps / elapsed

    strong = None
    if args.config == 2 and not args.no_strong:
        # the same model at a fixed global batch of 256 graphs split over
        # the ranks (strong scaling), measured in the same run as the weak-scaling line
        c4 = BENCH_CONFIGS[4].with_hidden(args.hidden)
        g4 = c4.graphs_per_gpu // world
        tr4, el4, pct4 = measure(c4, g4, args, device, rank, world)
        strong = {"config": "cfg4", "global_batch": g4 * world, "graphs_per_gpu": g4,
                  "value": round(g4 * world * args.steps / el4, 2), "unit": "graphs/s",
                  "ms_per_step": round(el4 / args.steps * 1e3, 4),
                  "step_ms_p10_p50_p90": [pct4[10], pct4[50], pct4[90]],
                  "scaling": "strong",
                  "edges_aggregated_per_s": round(tr4.batch.edge_index.size(1) * world
                                                  * layers * args.steps / el4, 1)}
        del tr4
        torch.cuda.empty_cache()

    rccl_world = (dist.get_world_size() if dist.is_initialized()
                  and dist.get_backend() == "nccl" else None)
    if world > 1 and args.dist_backend == "nccl":
        assert rccl_world == args.gpus, (rccl_world, args.gpus)
    kernels = time_kernels(tr, args.kernel_reps) if rank == 0 else {}
    result = None
    if rank == 0:
        work = sec8d_work(tr.batch.num_nodes, E_rank, tr.params["gnn_hidden"])
        roof = roofline_for(kernels, layers, work, cfg.name)
        roof["working_set_bytes"] = int(working_set)
        roof["mall_resident"] = bool(working_set < MALL_BYTES)
        roof_mp = roofline_mp(kernels, layers, work, cfg.name)
        if roof_mp is not None:
            copy_gbs = copy_ceiling_gbps(device)
            for r in roof_mp.values():
                r["measured_copy_GBps"] = copy_gbs
                r["frac_of_measured"] = round(r["achieved"] / copy_gbs, 4)
        roof_step = roofline_step(work, layers, ms)
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(cfg, graphs_per_rank, args.cpu_seconds)
        result = {
            "metric": "training graphs/s (24h_mixed GNN, full train step)",
            "value": round(value, 2), "unit": "graphs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            # untimed replays between the warmup / capture and the timed steps (clock ramp)
            "settle_steps": max(0, args.settle_steps),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
            "dtype": "f32 (split-bf16x3 GEMM products, fp32 accumulate)",
            "data": "synthetic (k-NN station graphs, random-init weights)",
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "rccl_world_size": rccl_world,
            "launcher": ("bench.py --gpus (one child process per GPU)"
                         if os.environ.get(LAUNCH_ENV) == "1" else
                         "torch.distributed.run" if world > 1 else "single process"),
            "config": {"workload": f"{cfg.name}: {cfg.experiment}, {graphs_global} graphs x "
                                   f"{cfg.num_stations} stations, k={cfg.k}, "
                                   f"{layers} GINE layers, D={tr.params['gnn_hidden']}",
                       "global_batch": graphs_global, "graphs_per_gpu": graphs_per_rank,
                       "nodes_per_gpu": tr.batch.num_nodes, "edges_per_gpu": E_rank,
                       "parallelism": f"dp{world}", "hip_graph": not args.no_graph,
                       "station_order": args.station_order,
                       "allreduce_in_graph": tr.allreduce_in_graph,
                       "allreduce_overlap": tr.overlap, "head_fold": options.HEAD_FOLD},
            "edges_aggregated_per_s": round(edges_per_s, 1),
            "step_ms_p10_p50_p90": [pct[10], pct[50], pct[90]],
            # N > 1 decomposition: the gradient all-reduce between the fwd+bwd and AdamW
            # graphs (HIP events on the step's stream; null when it is captured in the
            # graph or there is no collective), and every rank's p50 step
            "allreduce_ms_p50": pct.get("allreduce_p50"),
            "per_rank": pct.get("per_rank"),
            # steps > 10x the median on rank 0 (flagged, still inside `value`)
            "stalled_steps": pct.get("stalls"),
            # host side of the N > 1 line: intra-op threads per rank (the CPU share over the
            # local ranks) and the cgroup's throttling counters over the timed steps
            "host_threads_per_rank": threads, "cpu_share": cpu_share(),
            "cpu_throttle_timed": pct.get("cpu_throttle"),
            "roofline": roof, "roofline_step": roof_step,
            "roofline_message_passing": roof_mp,
            "strong_scaling_cfg4": strong,
            "cpu_baseline": cpu, "kernels": kernels,
            "final_loss": loss_val,
        }
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
