"""Diagnostic: fused chain forward/backward intermediates vs fp64 torch (prints errors)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]
import torch  # noqa: E402

from raincast_gnn import chain as C  # noqa: E402

DEV = torch.device("cuda:0")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max()).item()


for N, D, F, M in [(33, 128, 35, 11), (1000, 64, 35, 51)]:
    torch.manual_seed(N)
    lins = (torch.nn.Linear(D, D).to(DEV), torch.nn.Linear(D, D).to(DEV),
            torch.nn.Linear(D, D).to(DEV), torch.nn.Linear(F + D, D).to(DEV))
    r = (torch.randn(N, D) * 3).to(DEV).requires_grad_()
    x = torch.randn(N, F).to(DEV)
    saved = {}
    orig = C._ChainFn.forward

    h0 = C.chain(r, x, lins, M)
    node = h0.grad_fn
    s_, u_, e_ = node.saved_tensors[2], node.saved_tensors[3], node.saved_tensors[4]
    p2, r0, r1, dr_ = [(m.weight.detach().double(), m.bias.detach().double()) for m in lins]
    r64 = r.detach().double()
    s64 = r64 @ p2[0].T + M * p2[1]
    u64 = torch.relu(s64 @ r0[0].T + r0[1])
    e64 = u64 @ r1[0].T + r1[1]
    h64 = torch.cat([x.double(), e64], 1) @ dr_[0].T + dr_[1]
    print(N, D, "fwd rel: s", rel(s_, s64), "u", rel(u_, u64), "e", rel(e_, e64), "h0", rel(h0, h64))
    dh = torch.randn(N, D, device=DEV)
    h0.backward(dh)
    de64 = dh.double() @ dr_[0][:, F:]
    dt64 = (de64 @ r1[0]) * (u64 > 0).double()
    ds64 = dt64 @ r0[0]
    drr = ds64 @ p2[0]
    print("  r.grad rel", rel(r.grad, drr), "dWp2", rel(lins[0].weight.grad, ds64.T @ r64),
          "dWr0", rel(lins[1].weight.grad, dt64.T @ s64), "dWr1", rel(lins[2].weight.grad, de64.T @ u64))
    print("  r.grad[0,:4]", r.grad[0, :4].tolist(), "ref", drr[0, :4].tolist())
    gw = lins[0].weight.grad.double().cpu()
    ref = (ds64.T @ r64).cpu()
    print("  dWp2 norm", gw.norm().item(), "ref", ref.norm().item(), "first", gw[0, :3].tolist(), ref[0, :3].tolist())
    print("  dWp2 vs r^T ds?", rel(gw, (r64.T @ ds64).cpu()), " vs ds^T s", rel(gw, (ds64.T @ s64).cpu()),
          " dbp2", rel(lins[0].bias.grad, M * ds64.sum(0)), "dWdr", rel(lins[3].weight.grad, dh.double().T @ torch.cat([x.double(), e64], 1)))
