"""GPU: the training step at the benchmark configurations of BASELINE.json / SURVEY.md 8.

Oracle parity (tests/helpers.py: check_training_step -- predictions, loss and the BatchNorm
running statistics within 1e-5 of the CPU oracle, fp64 tie-break; every parameter gradient
within 1e-5, condition-scaled, of the fp64 oracle on the engine's branch: the oracle follows
the engine's ReLU decisions, each one that differs from its own checked against the engine's
per-decision forward rounding bound, EngineTies) on each config's own station graph,
experiment head and layer count, at batch sizes the CPU oracle finishes in seconds:

* cfg2 at full size (32 x 500 stations, k=10): the fused gather + Linear1 forward, the
  LDS-window backward with the weight-gradient engine in the same launch, BatchNorm sums
  by fixed-point accumulators in both directions;
* cfg3's graph (2,000 stations, k=16, 72h_mixed_u: MixedLoss with a learned u) at 4 graphs
  (8,000 nodes: fused forward) and 9 graphs (18,000 nodes: the standalone gather forward,
  no window plan -> the gather backward with dz and the weight gradients in one launch);
* cfg5's graph (10,000 stations, k=32: in-degree 33, above the fused forward's limit;
  3 GINE layers; 120h_normal_mixed) at 1 graph.

With GINE_PARITY_REPORT=<dir> set, each case writes its per-parameter error table and its
decision table there (profiles/r04_*_parity_*.txt).

At the configs' full sizes (cfg3: 64 graphs, 128,000 nodes; cfg4: cfg2's graph at the global
batch of 256 graphs, 128,000 nodes -- what one GPU of the strong-scaling curve runs at N=1,
and the shapes of N=2/4/8 are 128/64/32 graphs of the same graph; cfg5: 8 graphs, 80,000 nodes),
where an oracle step would take minutes, size-independent properties: the step is finite
and bit-identical when re-run from the same state, and the fused and unfused forward
kernels give bit-identical gradients (same z / a1 / BatchNorm integer sums).
"""
import copy
import os

import pytest
import torch

from raincast_gnn import options

from helpers import check_training_step, engine_order_batch
from raincast_gnn.data import synthetic_batch
from raincast_gnn.params import BENCH_CONFIGS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5


def _order(relabel):
    return "locality" if relabel else "dataset"


class _report(list):
    """The tables check_training_step appends, written to $GINE_PARITY_REPORT/<name>.txt."""

    def __init__(self, name):
        super().__init__()
        self.name = name

    def append(self, text):
        super().append(text)
        out = os.environ.get("GINE_PARITY_REPORT")
        if out:
            os.makedirs(out, exist_ok=True)
            with open(os.path.join(out, f"parity_{self.name}.txt"), "w") as f:
                f.write("\n\n".join(self) + "\n")


@pytest.mark.parametrize("cfg,graphs,relabel",
                         [(2, 32, False), (3, 4, False), (3, 9, False), (5, 1, False),
                          (2, 32, True), (3, 9, True), (5, 1, True)],
                         ids=["cfg2-full", "cfg3-b4-fused", "cfg3-b9-gather", "cfg5-b1",
                              "cfg2-full-relabel", "cfg3-b9-relabel-window", "cfg5-b1-relabel"])
def test_training_step_matches_oracle_at_config(cfg, graphs, relabel):
    """relabel: the engine runs the batch in its station locality order (the order the
    benchmark and the device loader use: narrow LDS windows, and at cfg3 a window plan where
    the dataset order has none), predictions mapped back; the oracle runs the reference
    order."""
    c = BENCH_CONFIGS[cfg]
    params = c.params()
    batch = synthetic_batch(c.num_stations, graphs, k=c.k, seed=100 + cfg)
    worst = check_training_step(params, batch, DEV, TOL, relabel=relabel,
                                report=_report(f"cfg{cfg}_b{graphs}_{_order(relabel)}"))
    print(f"{c.name} x{graphs} relabel={relabel}: worst scaled grad err {worst:.2e}")


@pytest.mark.skipif(not os.environ.get("GINE_FULL_PARITY"),
                    reason="full-size oracle steps take minutes of host time: set "
                           "GINE_FULL_PARITY=1 (run by tools/sessions, tables in profiles/)")
@pytest.mark.timeout(1800)
@pytest.mark.parametrize("cfg,graphs", [(5, 8), (3, 64)], ids=["cfg5-full", "cfg3-full"])
def test_training_step_matches_oracle_at_full_config(cfg, graphs):
    """The same oracle parity at the configs' full sizes (cfg5: 8 x 10,000 stations, 80,000
    nodes, 3 layers; cfg3: 64 x 2,000 stations, 128,000 nodes), in the locality order the
    benchmark runs: opt-in (GINE_FULL_PARITY=1), its tables committed under profiles/."""
    c = BENCH_CONFIGS[cfg]
    assert graphs == c.graphs_per_gpu
    batch = synthetic_batch(c.num_stations, graphs, k=c.k, seed=100 + cfg)
    worst = check_training_step(c.params(), batch, DEV, TOL, relabel=True,
                                report=_report(f"cfg{cfg}_b{graphs}_locality"))
    print(f"{c.name} x{graphs} full size: worst scaled grad err {worst:.2e}")


@pytest.mark.parametrize("relabel", [False, True], ids=["dataset-order", "relabel"])
def test_training_step_matches_oracle_at_cfg2_d64(relabel):
    """The D = 64 sweep point of the 24h_mixed benchmark (BASELINE.md:47, the north star's
    64-dim features) at full size: 32 x 500 stations, gnn_hidden = 64.  In the locality
    order the window backward carries the node-MLP weight-gradient engine (32-channel
    slices: 2 per tile) and the BatchNorm backward sums go through the accumulator."""
    c = BENCH_CONFIGS[2].with_hidden(64)
    params = c.params()
    assert params["gnn_hidden"] == 64
    batch = synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k, seed=102)
    worst = check_training_step(params, batch, DEV, TOL, relabel=relabel,
                                report=_report(f"cfg2_d64_b32_{_order(relabel)}"))
    print(f"{c.name} relabel={relabel}: worst scaled grad err {worst:.2e}")


def test_cfg2_d64_uses_the_combined_backward():
    from raincast_gnn import functional as Fn
    from raincast_gnn.graph import GineGraph
    c = BENCH_CONFIGS[2]
    b = engine_order_batch(synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k, seed=1))
    g = GineGraph(b.edge_index.to(DEV), b.edge_attr.to(DEV), b.num_nodes)
    plan = g.window_plan("out", 64)
    assert plan is not None and plan.slice_channels == 32
    assert Fn.engine_in_mp_ok(g, 64)


def _grads_after_step(model, batch):
    model.zero_grad(set_to_none=True)
    loss = model.loss_fn.crps(model(batch), batch.y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_full_size_step_deterministic_and_fused_equal(cfg, monkeypatch):
    from raincast_gnn.models import gnn_from_params
    c = BENCH_CONFIGS[cfg]
    torch.manual_seed(42)
    base = gnn_from_params(c.params()).to(DEV).train()
    batch = synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k, seed=1000).to(DEV)
    assert batch.num_nodes == c.num_stations * c.graphs_per_gpu

    def run(mode):
        monkeypatch.setattr(options, "MP_FUSED", mode)
        return _grads_after_step(copy.deepcopy(base), batch)

    l0, g0 = run("1")       # what the training step runs at this size
    l1, g1 = run("1")
    assert torch.isfinite(l0) and all(torch.isfinite(g).all() for g in g0)
    assert torch.equal(l0, l1) and all(torch.equal(a, b) for a, b in zip(g0, g1))
    # cfg3 / cfg4: in-degree 17 / 11 -> the fused forward applies once the size gate is lifted;
    # cfg5: in-degree 33 is beyond it, so "all" must fall back to the same kernels
    l2, g2 = run("all")
    l3, g3 = run("0")
    assert torch.equal(l2, l3) and all(torch.equal(a, b) for a, b in zip(g2, g3))
    assert torch.equal(l0, l3) and all(torch.equal(a, b) for a, b in zip(g0, g3))


def test_device_collation_on_gpu_matches_collate():
    """Row a9: DeviceDataset.batch on the HIP device equals PyG-style collation."""
    from raincast_gnn.batching import DeviceDataset
    from raincast_gnn.data import collate, synthetic_samples
    samples = synthetic_samples(500, 12, k=10, seed=5)
    ds = DeviceDataset(samples, DEV, relabel=False)
    idx = torch.tensor([11, 3, 3, 0, 7, 9], device=DEV)
    got = ds.batch(idx)
    ref = collate([samples[i] for i in idx.tolist()])
    for name in ("x", "ensemble", "edge_index", "edge_attr", "batch", "ptr"):
        a = getattr(got, name)
        assert a.device.type == "cuda", name
        assert torch.equal(a.cpu(), getattr(ref, name)), name
    assert torch.equal(got.y.isnan().cpu(), ref.y.isnan())
    assert torch.equal(torch.nan_to_num(got.y).cpu(), torch.nan_to_num(ref.y))
    assert got.num_graphs == ref.num_graphs == 6
    # ...and the model gives the same bits on either batch
    from raincast_gnn.models import gnn_from_params
    from raincast_gnn.params import EXPERIMENTS
    torch.manual_seed(0)
    m = gnn_from_params(EXPERIMENTS["24h_mixed"]).to(DEV).eval()
    with torch.no_grad():
        assert torch.equal(m(got), m(ref.to(DEV)))


def test_relabelled_batch_gives_the_same_per_node_bits_in_eval():
    """The station relabelling changes where a node's row is stored, not its value: in eval
    mode (BatchNorm from running statistics, no reduction over nodes) every prediction of
    the relabelled batch equals the collated batch's bit for bit once mapped back --
    DeepSet, Linears and head are per node, and each node's message passing sums its edges
    in the same (original) order."""
    from raincast_gnn.batching import DeviceDataset
    from raincast_gnn.data import collate, restore_node_order, synthetic_samples
    from raincast_gnn.models import gnn_from_params
    from raincast_gnn.params import EXPERIMENTS
    samples = synthetic_samples(500, 12, k=10, seed=5)
    ds = DeviceDataset(samples, DEV)            # default: engine (locality) order
    assert ds.order is not None
    idx = torch.tensor([11, 3, 3, 0, 7, 9], device=DEV)
    got = ds.batch(idx)
    ref = collate([samples[i] for i in idx.tolist()]).to(DEV)
    assert torch.equal(restore_node_order(got.x, got), ref.x)
    rows = got.extra["node_order"]
    assert torch.equal(rows[got.edge_index], ref.edge_index)   # same edges, same order
    torch.manual_seed(0)
    m = gnn_from_params(EXPERIMENTS["24h_mixed"]).to(DEV)
    with torch.no_grad():
        m.train()
        m(ref)                                   # non-trivial running statistics
        m.eval()
        assert torch.equal(restore_node_order(m(got), got), m(ref))


@pytest.mark.parametrize("cfg,hidden", [(2, None), (2, 64), (3, None), (4, None), (5, None)],
                         ids=["cfg2", "cfg2-D64", "cfg3", "cfg4", "cfg5"])
def test_relabelled_full_size_step_deterministic_and_close(cfg, hidden):
    """The benchmark's batch (full size, engine order) against the same batch in the
    reference order on the engine: both steps finite and deterministic; the loss and the
    predictions equal within 1e-5 (only the order of node reductions differs)."""
    from raincast_gnn.data import restore_node_order
    from raincast_gnn.models import gnn_from_params
    c = BENCH_CONFIGS[cfg].with_hidden(hidden)
    torch.manual_seed(42)
    base = gnn_from_params(c.params()).to(DEV).train()
    batch = synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k, seed=1000)
    rb = engine_order_batch(batch).to(DEV)
    batch = batch.to(DEV)

    def run(b):
        m = copy.deepcopy(base)
        pred = m(b)
        loss = m.loss_fn.crps(pred, b.y)
        loss.backward()
        torch.cuda.synchronize()
        return (restore_node_order(pred.detach(), b), loss.detach(),
                [p.grad.detach().clone() for p in m.parameters()])

    p0, l0, g0 = run(rb)
    p1, l1, g1 = run(rb)
    assert torch.isfinite(l0) and all(torch.isfinite(g).all() for g in g0)
    assert torch.equal(l0, l1) and all(torch.equal(a, b) for a, b in zip(g0, g1))
    pr, lr, _ = run(batch)
    assert abs(l0.item() - lr.item()) <= TOL * abs(lr.item())
    assert (p0 - pr).abs().max().item() <= TOL * pr.abs().max().item()
