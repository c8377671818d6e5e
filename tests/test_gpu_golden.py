"""GPU: the HIP path against the committed GINE golden vectors (tests/golden/gine_golden.npz).

Message passing: z and dx bit-identical to the fixture of the SAME edge-Linear rounding
(both roundings are run explicitly, whatever the host CPU is), through both the gather and
the window-staged kernels; dlin_w, dlin_b, deps against the fp64 fixture at 1e-5 max-norm
relative.  Full GINE layer (GINEConv + node MLP with train-mode BatchNorm): output, input
gradient, parameter gradients and BN running statistics against fp64 at 1e-5.
"""
import os

import numpy as np
import pytest
import torch

from raincast_gnn import options

from conftest import GOLDEN
from helpers import rel_err
from raincast_gnn import GINEConv, _lib, functional as Fn
from raincast_gnn.graph import GineGraph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5
FIX = np.load(os.path.join(GOLDEN, "gine_golden.npz"))
CASES = sorted({k.split("/")[1] for k in FIX.files if k.startswith("mp/")})
FLAGS = {"fma": 0, "muladd": _lib.GINE_MP_LIN_MULADD}


def t(key):
    return torch.from_numpy(FIX[key])


@pytest.mark.parametrize("window", ["0", "all"])
@pytest.mark.parametrize("name", CASES)
def test_mp_matches_golden(name, window, monkeypatch):
    monkeypatch.setattr(options, "MP_WINDOW", window)
    p = f"mp/{name}/"
    x = t(p + "x").to(DEV)
    ei, ea = t(p + "edge_index"), t(p + "edge_attr")
    g = GineGraph(ei.to(DEV), ea.to(DEV), x.size(0))
    w, b, eps = t(p + "lin_w").reshape(-1).to(DEV), t(p + "lin_b").to(DEV), t(p + "eps").to(DEV)
    dz = t(p + "dz").to(DEV)
    for rounding, flag in FLAGS.items():
        z = Fn.mp_forward(x, g, w, b, eps, lin_flag=flag)
        assert torch.equal(z.cpu(), t(p + f"z_{rounding}")), rounding
        dx, dlw, dlb, deps = Fn.mp_backward(dz, x, g, w, b, eps, lin_flag=flag)
        assert torch.equal(dx.cpu(), t(p + f"dx_{rounding}")), rounding
        for key, got in (("dlin_w64", dlw), ("dlin_b64", dlb)):
            ref = t(p + key)
            if ref.abs().max() == 0:
                assert got.abs().max().item() == 0
            else:
                assert rel_err(got, ref) <= TOL, (rounding, key, rel_err(got, ref))
        # d eps = sum(dz * x) cancels: condition-scaled bound
        scale = (t(p + "dz").double() * t(p + "x").double()).abs().sum().item()
        err = abs(deps.item() - t(p + "deps64").item())
        assert err <= TOL * max(scale, 1e-30), (rounding, err, scale)


def test_layer_matches_golden():
    p = "layer/"
    D = FIX[p + "x"].shape[1]
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    state = {k[len(p + "param/"):]: t(k) for k in FIX.files if k.startswith(p + "param/")}
    state["nn.1.num_batches_tracked"] = torch.tensor(0)
    conv.load_state_dict(state)
    conv = conv.to(DEV).train()
    x = t(p + "x").to(DEV).requires_grad_(True)
    y = conv(x, t(p + "edge_index").to(DEV), t(p + "edge_attr").to(DEV))
    y.backward(t(p + "dy").to(DEV))
    assert rel_err(y, t(p + "y64")) <= TOL
    assert rel_err(x.grad, t(p + "dx64")) <= TOL
    for k, prm in conv.named_parameters():
        if k == "nn.0.bias":
            # a bias in front of train-mode BatchNorm has an exactly zero gradient (BN removes
            # the batch mean); fp32 leaves rounding noise, bounded against dW1's scale
            scale = t(p + "grad64/nn.0.weight").abs().max().item()
            assert prm.grad.abs().max().item() <= TOL * scale
            continue
        assert rel_err(prm.grad, t(p + "grad64/" + k)) <= TOL, k
    bn = conv.nn[1]
    assert rel_err(bn.running_mean, t(p + "running_mean64")) <= TOL
    assert rel_err(bn.running_var, t(p + "running_var64")) <= TOL
    assert int(bn.num_batches_tracked) == 1
