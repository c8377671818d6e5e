"""Per-parameter gradient error of one training step against the fp64 oracle, GPU and the
fp32 CPU oracle side by side (max-norm relative, as tests/helpers.assert_close_tiebreak):
    python tools/diag_param_errs.py [experiment ...]
Run under GINE_HIP_LIB=<variant .so> to compare library builds."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raincast-gnn_amd"), os.path.join(ROOT, "tests")]

from helpers import _oracle_step, rel_err  # noqa: E402
from oracle import gine_cpu as O  # noqa: E402
from raincast_gnn.data import synthetic_batch  # noqa: E402
from raincast_gnn.models import GNN  # noqa: E402
from raincast_gnn.params import EXPERIMENTS  # noqa: E402

DEV = torch.device("cuda:0")
for exp in sys.argv[1:] or ["24h_mixed"]:
    p = EXPERIMENTS[exp]
    batch = synthetic_batch(500, 2, k=10, seed=7)
    torch.manual_seed(42)
    model = GNN(35, p["gnn_hidden"], p["gnn_hidden"], p["gnn_layers"], loss=p["loss"],
                grad_u=p["grad_u"], u=p["u"], xi=p["xi"])
    ref = O.OracleGNN(35, p["gnn_hidden"], p["gnn_layers"], p["loss"], p["grad_u"], p["u"],
                      p["xi"])
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    model = model.to(DEV).train()
    outs = {"gpu": [], "cpu32": [], "cpu64": []}

    def hook(key):   # the oracle's conv output -> ResGnn's relu(conv) / x + relu(conv)
        def f(mod, args, out):
            y = torch.relu(out)
            if len(outs[key]) % len(ref.conv.convolutions):
                y = args[0] + y
            outs[key].append(y.detach().double().cpu())
        return f

    grads = {"gpu": {}, "cpu32": {}, "cpu64": {}}
    snaps = []

    def keep_grad(key, i, t):
        if t.requires_grad:
            t.register_hook(lambda g: grads[key].__setitem__(i, g.detach().double().cpu()))

    def pre(key):
        def f(mod, args):
            keep_grad(key, len(outs[key]) % len(ref.conv.convolutions), args[0])
        return f

    def wrap(fn):
        def g(*a, **k):
            keep_grad("gpu", len(outs["gpu"]), a[0])
            y = fn(*a, **k)
            snaps.append((y, [t.detach().clone() if t is not None else None
                              for t in y.grad_fn.saved_tensors]))
            outs["gpu"].append(y.detach().double().cpu())
            return y
        return g

    for c in model.conv.convolutions:
        c.forward_relu = wrap(c.forward_relu)
        c.forward_residual_relu = wrap(c.forward_residual_relu)
    loss = model.loss_fn.crps(model(batch.to(DEV)), batch.y.to(DEV))
    for i, (y, saved) in enumerate(snaps):
        now = y.grad_fn.saved_tensors
        same = [a is None or torch.equal(a, b) for a, b in zip(saved, now)]
        x, z, a1 = now[0], now[1], now[2]
        conv = model.conv.convolutions[i]
        lin1 = conv.nn[0]
        ref_a1 = z.double() @ lin1.weight.detach().double().t() + lin1.bias.detach().double()
        bn_save = now[5]
        v32 = a1 * bn_save[2] + bn_save[3]
        bnm = conv.nn[1]
        mu = ref_a1.mean(0)
        var = ref_a1.var(0, unbiased=False)
        alpha = bnm.weight.detach().double() / torch.sqrt(var + bnm.eps)
        v64 = (ref_a1 - mu) * alpha + bnm.bias.detach().double()
        flip = (v32 > 0) != (v64 > 0)
        print(f"layer {i}: saved unchanged {all(same)}; a1 vs z W1^T+b1 "
              f"{rel_err(a1, ref_a1):.3e}; mean/invstd vs fp64 "
              f"{rel_err(bn_save[0], mu):.2e}/{rel_err(bn_save[1], 1 / torch.sqrt(var + bnm.eps)):.2e};"
              f" BN-ReLU flips vs fp64 {int(flip.sum())}"
              + (f" (largest |v64| {v64[flip].abs().max().item():.2e})" if flip.any() else ""))
        lin2 = conv.nn[3]
        o64 = torch.relu(v64) @ lin2.weight.detach().double().t() + lin2.bias.detach().double()
        if now[4] is not None:
            m = now[4].bool()
            fl = m != (o64 > 0)
            print(f"   residual mask flips vs fp64 {int(fl.sum())}"
                  + (f" (largest |o64| {o64[fl].abs().max().item():.2e})" if fl.any() else ""))
        ei = batch.edge_index.to(DEV)
        ea = batch.edge_attr.to(DEV).view(-1, 1)
        lw, lb = conv.lin.weight.detach().view(1, -1), conv.lin.bias.detach().view(1, -1)
        pre32 = x[ei[0]] + (ea * lw + lb)
        pre64 = x.double()[ei[0]] + (ea.double() * lw.double() + lb.double())
        fl = (pre32 > 0) != (pre64 > 0)
        print(f"   message flips fp32 vs fp64 on the same x {int(fl.sum())}; exact zeros in x "
              f"{int((x == 0).sum())}")
    before = [[t.clone() if t is not None else None for t in y.grad_fn.saved_tensors]
              for y, _ in snaps]
    loss.backward(retain_graph=True)
    for i, (y, _) in enumerate(snaps):
        after = y.grad_fn.saved_tensors
        bad = [j for j, (a, b) in enumerate(zip(before[i], after))
               if a is not None and not torch.equal(a, b)]
        print(f"layer {i}: saved tensors changed by the backward: {bad}")
        for j in bad:
            d = (before[i][j] != after[j])
            idx = d.nonzero()
            print(f"   tensor {j} shape {tuple(after[j].shape)} {after[j].dtype}: {int(d.sum())} "
                  f"entries, first {idx[:3].tolist()} last {idx[-3:].tolist()}")
    def layer64(i, x):
        conv = model.conv.convolutions[i]
        l1, bnm, _, l2 = conv.nn
        d = lambda t: t.detach().double()
        ei = batch.edge_index.to(DEV)
        ea = batch.edge_attr.to(DEV).double().view(-1, 1)
        msg = torch.relu(x[ei[0]] + ea * d(conv.lin.weight).view(1, -1) + d(conv.lin.bias))
        agg = torch.zeros_like(x).index_add_(0, ei[1], msg)
        z = (1 + d(conv.eps)) * x + agg
        a1 = z @ d(l1.weight).t() + d(l1.bias)
        mu, var = a1.mean(0), a1.var(0, unbiased=False)
        h = torch.relu((a1 - mu) / torch.sqrt(var + bnm.eps) * d(bnm.weight) + d(bnm.bias))
        o = h @ d(l2.weight).t() + d(l2.bias)
        masks.clear()
        pre = x[ei[0]] + ea * d(conv.lin.weight).view(1, -1) + d(conv.lin.bias)
        masks.extend([(pre > 0, pre), (h > 0, (a1 - mu) / torch.sqrt(var + bnm.eps)), (o > 0, o)])
        return torch.relu(o) if i == 0 else x + torch.relu(o)

    masks = []

    for i in range(1, len(snaps)):
        x = snaps[i][0].grad_fn.saved_tensors[0].detach().double().requires_grad_(True)
        y = layer64(i, x)
        dy = grads["gpu"][i + 1].to(DEV) if i + 1 < len(snaps) else None
        if dy is None:
            continue
        (gx,) = torch.autograd.grad(y, x, dy)
        print(f"layer {i} input grad: gpu vs fp64 restatement on the gpu's x and dy "
              f"{rel_err(grads['gpu'][i], gx):.3e}")
    for c in ref.conv.convolutions:
        c.register_forward_hook(hook("cpu32"))
        c.register_forward_pre_hook(pre("cpu32"))
    r32 = dict(_oracle_step(ref, batch, torch.float32)[0].named_parameters())
    ref2 = ref
    for c in ref.conv.convolutions:
        c._forward_hooks.clear()
        c._forward_pre_hooks.clear()
        c.register_forward_hook(hook("cpu64"))
        c.register_forward_pre_hook(pre("cpu64"))
    r64 = dict(_oracle_step(ref2, batch, torch.float64)[0].named_parameters())
    for i in range(1, len(snaps)):
        with torch.no_grad():
            layer64(i, snaps[i][0].grad_fn.saved_tensors[0].detach().double())
            mg = [m for m, _ in masks]
            layer64(i, outs["cpu64"][i - 1].to(DEV))
            for name, a, (b, v) in zip(("message", "bn-relu", "residual"), mg, masks):
                fl = a != b
                print(f"layer {i} {name} decisions, gpu x vs oracle x: {int(fl.sum())} differ"
                      + (f" (|pre-activation| up to {v[fl].abs().max().item():.2e})"
                         if fl.any() else ""))
    print(f"== {exp}  lib={os.environ.get('GINE_HIP_LIB', 'main')}")
    for i, (g, c32, c64) in enumerate(zip(outs["gpu"], outs["cpu32"], outs["cpu64"])):
        print(f"layer {i} output: gpu {rel_err(g, c64):.3e}  cpu32 {rel_err(c32, c64):.3e}")
    for i in sorted(grads["cpu64"]):
        if i in grads["gpu"]:
            print(f"layer {i} input grad: gpu {rel_err(grads['gpu'][i], grads['cpu64'][i]):.3e}"
                  f"  cpu32 {rel_err(grads['cpu32'][i], grads['cpu64'][i]):.3e}")
    for name, q in model.named_parameters():
        print(f"{name:34s} gpu {rel_err(q.grad, r64[name].grad):.3e}   "
              f"cpu32 {rel_err(r32[name].grad, r64[name].grad):.3e}")
