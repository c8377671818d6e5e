"""One GINE layer (cfg2 graph, window backward with the weight-gradient engine) forward +
backward three times; prints a digest of every output so runs and builds can be compared
bit for bit (the message-passing outputs must not depend on the engine's arithmetic).
    python tools/determinism_layer.py"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from raincast_gnn import GINEConv  # noqa: E402
from raincast_gnn import nn as rnn  # noqa: E402
from raincast_gnn.data import synthetic_batch  # noqa: E402

DEV = torch.device("cuda:0")


def digest(t):
    return hashlib.sha1(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:12]


def main():
    rnn.USE_TORCH_EXT = False
    torch.manual_seed(0)
    D = 128
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1).to(DEV).train()
    b = synthetic_batch(500, 32, k=10, seed=4).to(DEV)
    x0 = torch.randn(b.num_nodes, D, device=DEV)
    gy = torch.randn(b.num_nodes, D, device=DEV)
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    opt = None
    if "--flat" in sys.argv:  # the deferred backward: window + engine launch, batch reduction
        from raincast_gnn.optim import FlatAdamW
        opt = FlatAdamW(conv.parameters(), lr=1e-3)
    for rep in range(3):
        conv.load_state_dict(state)
        if opt is not None:
            opt.zero_grad()
        else:
            conv.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        y = conv.forward_residual_relu(x, b.edge_index, b.edge_attr)
        y.backward(gy)
        torch.cuda.synchronize()
        names = ["y", "dx"] + [n for n, _ in conv.named_parameters()]
        ts = [y, x.grad] + [p.grad for _, p in conv.named_parameters()]
        print(rep, " ".join(f"{n}={digest(t)}" for n, t in zip(names, ts)), flush=True)
        out = os.environ.get("DET_SAVE")
        if out:
            torch.save({"dx": x.grad.detach().cpu()}, f"{out}_{rep}.pt")


if __name__ == "__main__":
    main()
