"""Diagnostic (GPU box): where does gradient error vs an fp64 oracle come from?

For one training step of a GNN config it prints, per parameter and per GINE-layer
input gradient, the max-norm relative error of the HIP path and of the fp32 CPU oracle
against the fp64 oracle.  Not a test: a measuring tool for DESIGN.md.
    python tools/diag_grads.py [experiment] [graphs]
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from helpers import rel_err  # noqa: E402
from oracle import gine_cpu as O  # noqa: E402
from raincast_gnn.data import synthetic_batch  # noqa: E402
from raincast_gnn.models import GNN  # noqa: E402
from raincast_gnn.params import EXPERIMENTS  # noqa: E402


def run(experiment="120h_normal_mixed", graphs=2):
    p = dict(EXPERIMENTS[experiment])
    torch.manual_seed(42)
    model = GNN(35, p["gnn_hidden"], p["gnn_hidden"], p["gnn_layers"], loss=p["loss"],
                grad_u=p["grad_u"], u=p["u"], xi=p["xi"])
    ref = O.OracleGNN(35, p["gnn_hidden"], p["gnn_layers"], p["loss"], p["grad_u"], p["u"], p["xi"])
    ref.load_state_dict(model.state_dict())
    batch = synthetic_batch(500, graphs, k=10, seed=7)
    dev = torch.device("cuda:0")

    def forward(m, b, store, gpu):
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
    for name, dt, store in (("cpu32", torch.float32, g32), ("cpu64", torch.float64, g64)):
        r = copy.deepcopy(ref).to(dt)
        b = copy.copy(batch)
        b.x, b.ensemble, b.edge_attr = (t.to(dt) for t in (batch.x, batch.ensemble, batch.edge_attr))
        lo = r.crps(forward(r, b, store, False), batch.y)
        lo.backward()
        outs[name] = r
    print(f"{experiment}: loss gpu {loss.item():.10f}")
    print("layer input-grad rel err vs fp64:  gpu | cpu32")
    for i in sorted(g64):
        print(f"  layer {i}: {rel_err(g_gpu[i], g64[i]):.2e} | {rel_err(g32[i], g64[i]):.2e}")
    p32, p64 = dict(outs["cpu32"].named_parameters()), dict(outs["cpu64"].named_parameters())
    print("param-grad rel err vs fp64:  gpu | cpu32   (only rows where gpu > 1e-6)")
    for name, prm in model.named_parameters():
        eg = rel_err(prm.grad.cpu(), p64[name].grad)
        ec = rel_err(p32[name].grad, p64[name].grad)
        if eg > 1e-6:
            print(f"  {name:45s} {eg:.2e} | {ec:.2e}")


if __name__ == "__main__":
    run(*(sys.argv[1:2] or ["120h_normal_mixed"]), *([int(sys.argv[2])] if len(sys.argv) > 2 else []))
