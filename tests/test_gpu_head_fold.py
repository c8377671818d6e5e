"""GPU: the output head folded into the last GINE layer's launch (gine_layer_head,
csrc/gine_mpmlp.hip k_mp_fwd_layer's epilogue) against the head's own launch
(gine_head_fwd_count, csrc/gine_head.hip) on the same layer output.

The epilogue threads hold each output row as the head kernel lays it out (one half-wave per
node, lane t = float4 t), and run the same fma order, butterfly, bias add and PostProcess, so
raw, pred and the loss's valid-target partial counts must be the same bits -- for every loss
kind, both ResGnn epilogues, with and without targets (NaN targets included), with the layer
window staging on and off, at sizes where one workgroup counts one part and where it counts
several.  Reference: models/gnn.py:138-141 (conv -> aggr -> PostProcess).
"""
import pytest
import torch

from raincast_gnn import GINEConv, _lib, head as fused_head, options
from raincast_gnn.data import relabel_edges, station_order

from helpers import knn_batch_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

KINDS = [("NormalCRPS", "False"), ("MixedNormalCRPS", "False"), ("MixedLoss", "False"),
         ("MixedLoss", "True")]


@pytest.fixture(autouse=True)
def _python_binding(monkeypatch):
    from raincast_gnn import nn as rnn
    monkeypatch.setattr(rnn, "USE_TORCH_EXT", False)
    monkeypatch.setattr(options, "LAYER_FWD", True)


def _conv(seed):
    torch.manual_seed(seed)
    D = 128
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1)
    with torch.no_grad():
        mlp[1].weight.uniform_(0.5, 1.5)
        mlp[1].bias.uniform_(-0.2, 0.2)
    return conv.to(DEV).train()


def _graph(nodes, k, graphs, seed):
    ei, ea, n = knn_batch_graph(nodes, k, graphs, seed=seed)
    ei = relabel_edges(ei, station_order(ei[:, :ei.size(1) // graphs], nodes))
    return ei.to(DEV), ea.to(DEV), n


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t


_REAL_CALL = _lib.call


def _counting_calls(monkeypatch):
    names = []
    real = _REAL_CALL

    def call(name, *args):
        names.append(name)
        return real(name, *args)
    monkeypatch.setattr(_lib, "call", call)
    return names


@pytest.mark.parametrize("loss,grad_u", KINDS)
@pytest.mark.parametrize("epilogue", ["relu", "residual"])
@pytest.mark.parametrize("nodes,k,graphs", [(500, 10, 32), (120, 6, 3), (97, 5, 1)],
                         ids=["cfg2", "small", "odd-N"])
@pytest.mark.parametrize("targets", ["y", "y-nan", "none"])
@pytest.mark.parametrize("win", [False, True], ids=["l2", "win"])
def test_folded_head_same_bits_as_head_launch(loss, grad_u, epilogue, nodes, k, graphs, targets,
                                              win, monkeypatch):
    monkeypatch.setattr(options, "LAYER_WIN", win)
    ei, ea, n = _graph(nodes, k, graphs, seed=nodes + k)
    conv = _conv(seed=k)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    kind = fused_head.loss_kind(loss, grad_u)
    K = fused_head.K_OF[kind]
    torch.manual_seed(nodes)
    lin = torch.nn.Linear(128, K).to(DEV)
    with torch.no_grad():  # pre-activations on both sides of softplus' threshold
        lin.bias.copy_(torch.tensor([0.5, 21.0, -2.0, 0.3, 1.0][:K]))
    x = torch.randn(n, 128, device=DEV) * 1.5 + 0.2
    y = None
    if targets != "none":
        y = torch.randn(n, device=DEV)
        if targets == "y-nan":
            y[torch.rand(n, device=DEV) < 0.3] = float("nan")
    fn = conv.forward_relu if epilogue == "relu" else conv.forward_residual_relu

    conv.load_state_dict(state)
    h_ref = fn(x, ei, ea)
    pred_ref = fused_head.head(h_ref, lin, kind, y)
    rec_ref = fused_head.record_of(pred_ref)

    conv.load_state_dict(state)
    plan = fused_head.plan(x, lin, kind, y)
    names = _counting_calls(monkeypatch)
    h = fn(x, ei, ea, head=plan)
    assert plan.done is not None, "the layer launch did not take the head"
    pred = fused_head.head(h, lin, kind, y, plan)
    assert not [c for c in names if c.startswith("gine_head_fwd")], names
    rec = fused_head.record_of(pred)
    torch.cuda.synchronize()

    assert torch.equal(_bits(h), _bits(h_ref))
    assert torch.equal(_bits(rec.raw), _bits(rec_ref.raw))
    assert torch.equal(_bits(pred), _bits(pred_ref))
    if y is None:
        assert rec.count_parts is None
    else:
        assert torch.equal(rec.count_parts, rec_ref.count_parts)
        assert int(rec.count_parts.sum()) == int((~torch.isnan(y)).sum())


def test_folded_head_backward_same_bits(monkeypatch):
    """The head's backward reads the raw output the fold wrote: gradients of a loss through
    layer + head are the same bits as with the head's own launch."""
    ei, ea, n = _graph(500, 10, 8, seed=3)
    conv = _conv(seed=2)
    state = {kk: v.clone() for kk, v in conv.state_dict().items()}
    kind = _lib.LOSS_MIXED
    lin = torch.nn.Linear(128, 4).to(DEV)
    x = torch.randn(n, 128, device=DEV)
    gp = torch.randn(n, 4, device=DEV)

    def run(fold):
        conv.load_state_dict(state)
        xi = x.clone().requires_grad_(True)
        plan = fused_head.plan(xi, lin, kind) if fold else None
        h = conv.forward_residual_relu(xi, ei, ea, head=plan)
        pred = fused_head.head(h, lin, kind, None, plan)
        (pred * gp).sum().backward()
        out = [pred.detach().clone(), xi.grad.clone(), lin.weight.grad.clone(),
               lin.bias.grad.clone()] + [p.grad.clone() for p in conv.parameters()]
        conv.zero_grad(set_to_none=True)
        lin.zero_grad(set_to_none=True)
        return out

    ref, got = run(False), run(True)
    for a, b in zip(got, ref):
        assert torch.equal(_bits(a), _bits(b))


def test_plan_not_taken_for_another_tensor():
    """A plan whose launch wrote a different tensor (or none) is not used: the head launches
    as usual."""
    ei, ea, n = _graph(120, 6, 3, seed=9)
    conv = _conv(seed=1)
    lin = torch.nn.Linear(128, 2).to(DEV)
    x = torch.randn(n, 128, device=DEV)
    plan = fused_head.plan(x, lin, _lib.LOSS_NORMAL)
    h = conv.forward_residual_relu(x, ei, ea, head=plan)
    other = h.clone()
    pred = fused_head.head(other, lin, _lib.LOSS_NORMAL, None, plan)
    ref = fused_head.head(other, lin, _lib.LOSS_NORMAL)
    assert plan.done is None  # consumed (one use)
    assert torch.equal(_bits(pred), _bits(ref))


@pytest.mark.parametrize("loss,grad_u", KINDS)
def test_model_step_same_bits_with_and_without_fold(loss, grad_u, monkeypatch):
    """The benchmark's training step (cfg2 shape, locality order) with the head folded into the
    last layer's launch or launched on its own: predictions, loss, every gradient and buffer
    the same bits over two steps, and no head launch of its own in the folded step."""
    import copy
    from helpers import engine_order_batch
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import gnn_from_params
    from raincast_gnn.params import BENCH_CONFIGS
    c = BENCH_CONFIGS[2]
    batch = engine_order_batch(synthetic_batch(c.num_stations, c.graphs_per_gpu, k=c.k,
                                               seed=13)).to(DEV)
    torch.manual_seed(6)
    params = dict(c.params(), loss=loss, grad_u=grad_u)
    base = gnn_from_params(params).to(DEV).train()

    def run(fold):
        monkeypatch.setattr(options, "HEAD_FOLD", fold)
        m = copy.deepcopy(base)
        names = _counting_calls(monkeypatch)
        out = []
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            pred = m(batch)
            loss_v = m.loss_fn.crps(pred, batch.y)
            loss_v.backward()
            out.append([pred.detach().clone(), loss_v.detach().clone()]
                       + [p.grad.clone() for p in m.parameters()]
                       + [b.clone() for b in m.buffers()])
        torch.cuda.synchronize()
        return out, names

    ref, names_ref = run(False)
    got, names = run(True)
    assert "gine_head_fwd_count" in names_ref
    assert not [c for c in names if c.startswith("gine_head_fwd")], names
    for a_step, b_step in zip(got, ref):
        for a, b in zip(a_step, b_step):
            assert torch.equal(a, b)
