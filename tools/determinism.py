"""Bit-determinism probe: each fused piece run twice on the same inputs, then one model
training step twice (fresh copies of one model), every output compared bit for bit.
    python tools/determinism.py"""
import copy
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd")]
import torch  # noqa: E402

from raincast_gnn import _lib  # noqa: E402

DEV = torch.device("cuda:0")


def same(name, a, b):
    eq = torch.equal(a, b)
    d = (a.double() - b.double()).abs().max().item() if not eq else 0.0
    print(f"{name:40s} {'same' if eq else 'DIFF'} {d:.3e}", flush=True)
    return eq


def deepset():
    N, M, F, H = 16000, 11, 35, 128
    torch.manual_seed(0)
    ens = torch.randn(N, M, F, device=DEV)
    w = torch.randn(H, F, device=DEV) / F ** 0.5
    b = torch.randn(H, device=DEV) * 0.1
    dr = torch.randn(N, H, device=DEV)
    nb = ctypes.c_size_t(0)
    _lib.call("gine_deepset_mask_bytes", N, M, H, ctypes.byref(nb))
    parts = ctypes.c_int32(0)
    _lib.call("gine_deepset_bwd_num_partials", N, H, ctypes.byref(parts))
    outs = []
    for _ in range(2):
        r = torch.full((N, H), float("nan"), device=DEV)
        mask = torch.zeros(nb.value, dtype=torch.uint8, device=DEV)
        slab = torch.full((parts.value * (H * F + H),), float("nan"), device=DEV)
        dw, db = torch.empty(H, F, device=DEV), torch.empty(H, device=DEV)
        s = _lib.stream_handle(DEV)
        P = _lib.ptr
        _lib.call("gine_deepset_fwd", P(ens), P(w), P(b), P(r), P(mask), N, M, F, H, s)
        _lib.call("gine_deepset_bwd", P(ens), P(mask), P(dr), P(slab), P(dw), P(db), N, M, F, H, s)
        torch.cuda.synchronize()
        outs.append((r, mask, slab, dw, db))
    for nm, a, b_ in zip(("ds r", "ds mask", "ds slab", "ds dw", "ds db"), *outs):
        same(nm, a, b_)
    ref = torch.relu(ens.double() @ w.double().T + b.double()).sum(1)
    print("ds r vs fp64 max rel", ((outs[0][0].double() - ref).abs().max() / ref.abs().max()).item())


def linear():
    from raincast_gnn.linear import Linear
    torch.manual_seed(1)
    lin = Linear(163, 128).to(DEV)
    x = torch.randn(16000, 163, device=DEV)
    dy = torch.randn(16000, 128, device=DEV)
    gs = []
    for _ in range(2):
        lin.weight.grad = None
        lin(x).backward(dy)
        gs.append(lin.weight.grad.clone())
    same("linear dW (engine)", *gs)


def model():
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    from raincast_gnn.optim import FlatAdamW
    torch.manual_seed(9)
    base = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    batch = synthetic_batch(500, 32, k=10, seed=4).to(DEV)
    res = []
    for _ in range(2):
        m = copy.deepcopy(base).to(DEV)
        opt = FlatAdamW(m.parameters(), lr=1e-3)
        opt.zero_grad()
        pred = m(batch)
        m.loss_fn.crps(pred, batch.y).backward()
        res.append((pred.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    same("model pred", res[0][0], res[1][0])
    for n in res[0][1]:
        same("grad " + n, res[0][1][n], res[1][1][n])


if __name__ == "__main__":
    deepset()
    linear()
    model()
