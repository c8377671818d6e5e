"""Diagnostic (GPU box): where does gradient error vs an fp64 oracle come from?

For one training step of a GNN config it prints, per parameter and per GINE-layer
input gradient, the max-norm relative error of the HIP path and of the fp32 CPU oracle
against the fp64 oracle.  Not a test: a measuring tool for DESIGN.md.
    python tools/diag_grads.py [experiment] [graphs]
    python tools/diag_grads.py --cfg 2 [graphs]     (a benchmark config's graph and head)
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from helpers import rel_err  # noqa: E402


def fro_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    den = b.norm().item()
    return (a - b).norm().item() / den if den else (a - b).norm().item()
from oracle import gine_cpu as O  # noqa: E402
from raincast_gnn.data import synthetic_batch  # noqa: E402
from raincast_gnn.models import GNN  # noqa: E402
from raincast_gnn.params import EXPERIMENTS  # noqa: E402


def run(experiment="120h_normal_mixed", graphs=2, stations=500, k=10, layers=None):
    p = dict(EXPERIMENTS[experiment])
    if layers is not None:
        p["gnn_layers"] = layers
    torch.manual_seed(42)
    model = GNN(35, p["gnn_hidden"], p["gnn_hidden"], p["gnn_layers"], loss=p["loss"],
                grad_u=p["grad_u"], u=p["u"], xi=p["xi"])
    ref = O.OracleGNN(35, p["gnn_hidden"], p["gnn_layers"], p["loss"], p["grad_u"], p["u"], p["xi"])
    ref.load_state_dict(model.state_dict())
    batch = synthetic_batch(stations, graphs, k=k, seed=7)
    dev = torch.device("cuda:0")

    def forward(m, b, store, gpu):
        if gpu:  # the path the training step runs (fused DeepSet + dense chain)
            x = m._front(b)
        else:
            emb = m.deepset(b.ensemble)
            x = m.dim_red(torch.cat([b.x, emb], dim=1))
        for i, conv in enumerate(m.conv.convolutions):
            x.register_hook(lambda g, i=i: store.__setitem__(i, g.detach().double().cpu()))
            if gpu:
                x = (conv.forward_relu(x, b.edge_index, b.edge_attr) if i == 0 else
                     conv.forward_residual_relu(x, b.edge_index, b.edge_attr))
            else:
                y = torch.relu(conv(x, b.edge_index, b.edge_attr))
                x = y if i == 0 else x + y
        out = m.aggr(x)
        return m.postprocess(out) if gpu else O.postprocess(out, m.loss, m.grad_u)

    g_gpu, g32, g64 = {}, {}, {}
    model = model.to(dev).train()
    bd = batch.to(dev)
    loss = model.loss_fn.crps(forward(model, bd, g_gpu, True), bd.y)
    loss.backward()
    outs = {}
    g32b = {}
    nthr = torch.get_num_threads()
    for name, dt, store in (("cpu32", torch.float32, g32), ("cpu64", torch.float64, g64),
                            ("cpu32_1t", torch.float32, g32b)):
        torch.set_num_threads(1 if name == "cpu32_1t" else nthr)
        r = copy.deepcopy(ref).to(dt)
        b = copy.copy(batch)
        b.x, b.ensemble, b.edge_attr = (t.to(dt) for t in (batch.x, batch.ensemble, batch.edge_attr))
        lo = r.crps(forward(r, b, store, False), batch.y)
        lo.backward()
        outs[name] = r
    torch.set_num_threads(nthr)
    print(f"{experiment}: loss gpu {loss.item():.10f}")
    print("layer input-grad rel err vs fp64:  gpu | cpu32 | cpu32 1 thread")
    for i in sorted(g64):
        print(f"  layer {i}: {rel_err(g_gpu[i], g64[i]):.2e} | {rel_err(g32[i], g64[i]):.2e}"
              f" | {rel_err(g32b[i], g64[i]):.2e}")
    p32, p64 = dict(outs["cpu32"].named_parameters()), dict(outs["cpu64"].named_parameters())
    p32b = dict(outs["cpu32_1t"].named_parameters())
    print("param-grad rel err vs fp64, max-norm: gpu | cpu32 | cpu32 1 thread;  "
          "Frobenius: gpu | cpu32 | cpu32 1 thread  (rows where gpu > 1e-6)")
    for name, prm in model.named_parameters():
        g, c, b = prm.grad.cpu(), p32[name].grad, p32b[name].grad
        eg, ec, eb = (rel_err(t, p64[name].grad) for t in (g, c, b))
        fg, fc, fb = (fro_err(t, p64[name].grad) for t in (g, c, b))
        if eg > 1e-6:
            print(f"  {name:40s} {eg:.2e} | {ec:.2e} | {eb:.2e};  {fg:.2e} | {fc:.2e} | {fb:.2e}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--cfg":
        from raincast_gnn.params import BENCH_CONFIGS
        c = BENCH_CONFIGS[int(sys.argv[2])]
        run(c.experiment, int(sys.argv[3]) if len(sys.argv) > 3 else c.graphs_per_gpu,
            c.num_stations, c.k, c.gnn_layers)
    else:
        run(*(sys.argv[1:2] or ["120h_normal_mixed"]),
            *([int(sys.argv[2])] if len(sys.argv) > 2 else []))
