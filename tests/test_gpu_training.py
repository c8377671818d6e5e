"""GPU: the training-step pieces around the GINE stack (flat AdamW, DeepSet restructure,
captured step) against their reference formulations."""
import copy

import pytest
import torch

from helpers import rel_err
from oracle import gine_cpu as O
from raincast_gnn.models import DeepSetEncoder
from raincast_gnn.optim import FlatAdamW

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_flat_adamw_matches_torch_adamw():
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(35, 64), torch.nn.ReLU(),
                              torch.nn.Linear(64, 5)).to(DEV)
    ref = copy.deepcopy(net)
    opt = FlatAdamW(net.parameters(), lr=3e-3, weight_decay=0.01)
    opt_ref = torch.optim.AdamW(ref.parameters(), lr=3e-3, weight_decay=0.01, foreach=False)
    x = torch.randn(256, 35, device=DEV)
    for _ in range(6):
        # identical gradients on both sides: only the optimizer arithmetic is compared
        opt_ref.zero_grad()
        ref(x).square().mean().backward()
        opt.zero_grad()
        for p, q in zip(net.parameters(), ref.parameters()):
            p.grad.copy_(q.grad)
        opt.step()
        opt_ref.step()
    assert opt.views_intact()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert rel_err(p.detach(), q.detach()) <= 2e-6
    st = opt_ref.state[next(ref.parameters())]
    assert opt.step_count.item() == st["step"].item() == 6


def test_deepset_restructure_matches_reference_form():
    torch.manual_seed(1)
    enc = DeepSetEncoder(35, 128, 128)
    ref = O.OracleDeepSet(35, 128, 128)
    ref.load_state_dict(enc.state_dict())
    ens = torch.randn(3000, 11, 35)
    out = enc.to(DEV)(ens.to(DEV))
    exp = ref(ens)
    exp64 = copy.deepcopy(ref).double()(ens.double())
    assert rel_err(out.detach().cpu(), exp64) <= 2 * rel_err(exp.detach(), exp64) + 1e-6
    assert rel_err(out.detach().cpu(), exp.detach()) <= 1e-5


def test_bench_trainer_graph_step_runs():
    import bench
    from raincast_gnn.params import BENCH_CONFIGS
    tr = bench.Trainer(BENCH_CONFIGS[1], DEV, 0, 1, 2)
    losses = [tr.eager_step().item() for _ in range(3)]
    tr.capture()
    for _ in range(3):
        losses.append(tr.step().item())
    assert all(map(lambda v: v == v, losses))  # finite / not NaN
    assert losses[-1] < losses[0]              # training makes progress (lr 1e-4, 6 steps)
