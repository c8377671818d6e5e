"""CPU: the drop-in module's interface (constructor, attributes, state_dict, errors)."""
import pytest
import torch

from oracle import gine_cpu as O
from raincast_gnn import GINEConv, _lib
from raincast_gnn.models import GNN, ResGnn


def _mlp(D=16):
    return torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                               torch.nn.Linear(D, D))


def test_constructor_semantics():
    conv = GINEConv(nn=_mlp(), train_eps=True, edge_dim=1)
    assert isinstance(conv.eps, torch.nn.Parameter) and conv.eps.item() == 0.0
    assert tuple(conv.lin.weight.shape) == (16, 1) and tuple(conv.lin.bias.shape) == (16,)
    conv2 = GINEConv(nn=_mlp(), eps=0.5, train_eps=False, edge_dim=None)
    assert "eps" in dict(conv2.named_buffers()) and conv2.lin is None
    assert conv2.eps.item() == 0.5
    with torch.no_grad():
        conv.eps.fill_(3.0)
    conv.reset_parameters()
    assert conv.eps.item() == 0.0
    with pytest.raises(ValueError, match="infer input channels"):
        GINEConv(nn=torch.nn.ReLU(), edge_dim=1)
    with pytest.raises(NotImplementedError):
        GINEConv(nn=_mlp(), edge_dim=1, aggr="mean")


def test_state_dict_keys_match_reference_layout():
    conv = GINEConv(nn=_mlp(), train_eps=True, edge_dim=1)
    ref = O.OracleGINEConv(_mlp(), train_eps=True, edge_dim=1)
    assert list(conv.state_dict()) == list(ref.state_dict())
    expected = {"eps", "nn.0.weight", "nn.0.bias", "nn.1.weight", "nn.1.bias",
                "nn.1.running_mean", "nn.1.running_var", "nn.1.num_batches_tracked",
                "nn.3.weight", "nn.3.bias", "lin.weight", "lin.bias"}
    assert set(conv.state_dict()) == expected


def test_gnn_state_dict_matches_oracle():
    m = GNN(35, 128, 128, 4, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5)
    r = O.OracleGNN(35, 128, 4, "MixedLoss", "False", 1.71, 0.5)
    assert set(m.state_dict()) == set(r.state_dict())
    r.load_state_dict(m.state_dict())
    n_params = sum(p.numel() for p in m.parameters())
    # 209,800 parameters for 24h_mixed
    assert n_params == 209800
    assert isinstance(m.conv, ResGnn) and len(m.conv.convolutions) == 4


def test_no_cpu_fallback():
    conv = GINEConv(nn=_mlp(), train_eps=True, edge_dim=1)
    x = torch.randn(5, 16)
    ei = torch.tensor([[0, 1], [1, 2]])
    with pytest.raises(_lib.GineError, match="no CPU fallback"):
        conv(x, ei, torch.ones(2, 1))


def test_edge_dim_none_and_mismatch_errors():
    conv = GINEConv(nn=_mlp(), train_eps=True, edge_dim=None)
    with pytest.raises((ValueError, _lib.GineError, NotImplementedError)):
        conv(torch.randn(3, 16), torch.tensor([[0], [1]]), torch.ones(1, 4))
