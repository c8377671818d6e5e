"""Fused output head (csrc/gine_head.hip): ``PostProcess(aggr(h))`` of models/gnn.py:140-141
and models/model_utils.py:70-113, forward and backward, against the unfused torch modules
in fp64 (the composition is elementwise after one K-wide GEMV, so the fp32 kernel must sit
within fp32 rounding of the exact result: relative 1e-5 normwise per output)."""
import pytest
import torch

from raincast_gnn import head as fused_head
from raincast_gnn.postprocess import PostProcess

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL = 1e-5

CASES = [("NormalCRPS", "False"), ("MixedNormalCRPS", "False"), ("MixedLoss", "False"),
         ("MixedLoss", "True")]


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


@pytest.mark.parametrize("loss,grad_u", CASES)
@pytest.mark.parametrize("N,D", [(1, 128), (7, 64), (16000, 128), (333, 256), (50, 4)])
def test_head_matches_postprocess_of_linear(loss, grad_u, N, D):
    kind = fused_head.loss_kind(loss, grad_u)
    K = fused_head.K_OF[kind]
    g = torch.Generator().manual_seed(N * 7 + D + K)
    h = (torch.randn(N, D, generator=g) * 3).to(DEV).requires_grad_()
    lin = torch.nn.Linear(D, K).to(DEV)
    with torch.no_grad():  # push some pre-activations past softplus' threshold (20)
        lin.bias.copy_(torch.tensor([0.5, 21.0, -2.0, 0.3, 1.0][:K]))
    assert fused_head.fusable(h, lin, kind)
    pred = fused_head.head(h, lin, kind)

    h64 = h.detach().double().requires_grad_()
    w64 = lin.weight.detach().double().requires_grad_()
    b64 = lin.bias.detach().double().requires_grad_()
    ref = PostProcess(loss, grad_u)(torch.nn.functional.linear(h64, w64, b64))
    for k in range(K):
        assert _rel(pred[:, k], ref[:, k]) <= TOL, (k, _rel(pred[:, k], ref[:, k]))

    gp = torch.randn(N, K, generator=g).to(DEV)
    pred.backward(gp)
    ref.backward(gp.double())
    assert _rel(h.grad, h64.grad) <= TOL
    assert _rel(lin.weight.grad, w64.grad) <= TOL
    assert _rel(lin.bias.grad, b64.grad) <= TOL


def test_head_deterministic_and_model_uses_it():
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN

    torch.manual_seed(0)
    model = GNN(35, 128, 128, 2, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5).to(DEV)
    batch = synthetic_batch(60, 2, k=5, seed=1).to(DEV)
    grads = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        loss = model.loss_fn.crps(model(batch), batch.y)
        loss.backward()
        grads.append(torch.cat([model.aggr.weight.grad.reshape(-1), model.aggr.bias.grad]))
    assert torch.equal(grads[0], grads[1])


def test_captured_step_recounts_valid_targets():
    """The whole-network capture pattern: eager warm-up on ``static_y``, capture with the same
    tensor, then ``static_y.copy_(new)`` with a different number of NaN targets before the
    replay.  The replayed gradient must divide by the NEW count (the count is recomputed
    inside the graph), i.e. equal the eager gradient on the new targets bit for bit."""
    from raincast_gnn import gradbuf
    from raincast_gnn.data import synthetic_batch
    from raincast_gnn.models import GNN
    from raincast_gnn.optim import FlatAdamW

    torch.manual_seed(0)
    model = GNN(35, 128, 128, 2, loss="MixedLoss", grad_u="False", u=1.71, xi=0.5).to(DEV)
    model.train()
    opt = FlatAdamW(model.parameters(), lr=1e-4)
    batch = synthetic_batch(60, 2, k=5, seed=1).to(DEV)
    static_y = batch.y.clone()

    def fwd_bwd():
        opt.zero_grad()
        loss = model.loss_fn.crps(model(batch), static_y)
        gradbuf.loss_backward(loss)
        opt.gather_grads()
        return loss

    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        for _ in range(2):
            fwd_bwd()
    torch.cuda.current_stream(DEV).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        loss_g = fwd_bwd()
    new_y = batch.y.clone()
    new_y[::3] = float("nan")
    assert int(torch.isnan(new_y).sum()) != int(torch.isnan(batch.y).sum())
    static_y.copy_(new_y)
    graph.replay()
    torch.cuda.synchronize()
    g_graph, l_graph = opt.flat_grad.clone(), loss_g.clone()
    l_eager = fwd_bwd()
    torch.cuda.synchronize()
    assert torch.equal(l_graph, l_eager)
    assert torch.equal(g_graph, opt.flat_grad), (g_graph - opt.flat_grad).abs().max()


def test_sum_32_same_bits_as_shfl_xor_butterfly():
    """csrc/gine_headrow.hpp sum_32 (permlane16_swap + DPP lane exchanges) gives, at every
    lane, the bits of the __shfl_xor butterfly it replaces: same partners, same order, same
    rounding -- on values spread over many binades, with ties, signed zeros, inf and NaN."""
    from raincast_gnn import _lib
    g = torch.Generator().manual_seed(5)
    waves = 4096
    x = torch.randn(waves * 64, generator=g) * torch.exp2(torch.randint(-30, 30, (waves * 64,),
                                                                         generator=g).float())
    x[::97] = 0.0
    x[1::101] = -0.0
    x[5::1009] = float("inf")
    x[7::1013] = float("-inf")
    x[3::2003] = float("nan")
    x = x.to(DEV)
    outs = []
    for mode in (0, 1):
        o = torch.empty_like(x)
        _lib.call("gine_testing_sum_32", _lib.ptr(x), _lib.ptr(o), waves, mode,
                  _lib.stream_handle(DEV))
        outs.append(o)
    torch.cuda.synchronize()
    num = ~torch.isnan(outs[0])
    assert torch.equal(outs[0][num].view(torch.int32), outs[1][num].view(torch.int32))
    assert torch.equal(torch.isnan(outs[0]), torch.isnan(outs[1]))
