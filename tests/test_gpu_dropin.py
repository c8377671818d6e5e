"""GPU: the drop-in path -- the reference's model structure in torch with only GINEConv
swapped (raincast_gnn.dropin), driven like train.py:61-71 with ``batch.to(device)`` every
step -- and the graph cache's content check that keeps that path from rebuilding the CSRs
and window plans each step (raincast_gnn/graph.py, gine_graph_same_edges)."""
import pytest
import torch

from oracle import gine_cpu as O
from raincast_gnn import functional as Fn
from raincast_gnn.data import collate, synthetic_samples
from raincast_gnn.dropin import ReferenceStructGNN
from raincast_gnn.graph import _GraphCache, GineGraph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph_arrays(g):
    return [t.cpu() for t in (g.in_rowptr, g.in_src, g.in_attr, g.out_rowptr, g.out_dst,
                              g.out_attr)]


def test_content_hit_reuses_graph_and_miss_rebuilds():
    cache = _GraphCache()
    s = synthetic_samples(120, 3, k=6, seed=2)
    b = collate(s)
    n = b.num_nodes
    g0 = cache.get(b.edge_index.to(DEV), b.edge_attr.to(DEV), n)
    assert cache.stats == {"identity_hits": 0, "content_hits": 0, "builds": 1}
    # a fresh device copy of the same edge list (batch.to(device) each step): same graph
    g1 = cache.get(b.edge_index.to(DEV), b.edge_attr.to(DEV), n)
    assert g1 is g0 and cache.stats["content_hits"] == 1 and cache.stats["builds"] == 1
    # the same tensor again: identity hit
    ei = b.edge_index.to(DEV)
    ea = b.edge_attr.to(DEV)
    assert cache.get(ei, ea, n) is g0 and cache.get(ei, ea, n) is g0
    assert cache.stats["identity_hits"] >= 1
    # same sizes, one destination moved: a new graph, identical to a fresh build
    ei2 = b.edge_index.clone()
    ei2[1, 7] = (ei2[1, 7] + 1) % n
    g2 = cache.get(ei2.to(DEV), b.edge_attr.to(DEV), n)
    assert g2 is not g0 and cache.stats["builds"] == 2
    ref = GineGraph(ei2.to(DEV), b.edge_attr.to(DEV), n)
    assert all(torch.equal(a, c) for a, c in zip(_graph_arrays(g2), _graph_arrays(ref)))
    # same edges, one attribute changed (last bit): a new graph too
    ea3 = b.edge_attr.clone()
    ea3[3, 0] = torch.nextafter(ea3[3, 0], torch.tensor(10.0))
    g3 = cache.get(b.edge_index.to(DEV), ea3.to(DEV), n)
    assert g3 is not g0 and cache.stats["builds"] == 3
    # in-place change of a tensor the cache has seen: identity miss, content miss
    ei[0, 0] = (ei[0, 0] + 1) % n
    g4 = cache.get(ei, ea, n)
    assert g4 is not g0 and cache.stats["builds"] == 4


def test_content_cache_alternating_graphs_of_one_size():
    """Two distinct edge lists of the same size (two station sets) used alternately, each
    step a fresh device copy: after one build each, every step is a content hit."""
    cache = _GraphCache()
    ba = collate(synthetic_samples(120, 3, k=6, seed=2))
    bb = collate(synthetic_samples(120, 3, k=6, seed=9))
    assert ba.edge_index.shape == bb.edge_index.shape and not torch.equal(ba.edge_index,
                                                                           bb.edge_index)
    n = ba.num_nodes
    ga = cache.get(ba.edge_index.to(DEV), ba.edge_attr.to(DEV), n)
    gb = cache.get(bb.edge_index.to(DEV), bb.edge_attr.to(DEV), n)
    assert ga is not gb and cache.stats["builds"] == 2
    for step in range(6):
        b, g = (ba, ga) if step % 2 == 0 else (bb, gb)
        assert cache.get(b.edge_index.to(DEV), b.edge_attr.to(DEV), n) is g
    assert cache.stats["builds"] == 2 and cache.stats["content_hits"] == 6


def test_content_check_odd_sizes():
    """Edge counts whose int64 list is not a whole number of 16-byte vectors, unaligned
    views, and E = 0."""
    cache = _GraphCache()
    for E in (0, 1, 3, 5):
        ei = torch.randint(0, 9, (2, E))
        ea = torch.rand(E, 1)
        g = cache.get(ei.to(DEV), ea.to(DEV), 9)
        assert cache.get(ei.to(DEV), ea.to(DEV), 9) is g
    big = torch.randint(0, 50, (2, 101))
    view = big.to(DEV)[:, 1:]          # 8-byte offset view
    g = cache.get(view, None, 50)
    assert cache.get(big[:, 1:].contiguous().to(DEV), None, 50) is g


def _struct_model(loss, grad_u):
    torch.manual_seed(5)
    model = ReferenceStructGNN(35, 128, 128, 2, loss=loss, grad_u=grad_u, u=1.71, xi=0.5)
    ref = O.OracleGNN(35, 128, 2, loss, grad_u, 1.71, 0.5)
    ref.load_state_dict(model.state_dict())
    return model, ref


@pytest.mark.parametrize("loss,grad_u", [("MixedLoss", "False"), ("MixedNormalCRPS", "False")])
def test_dropin_model_matches_oracle(loss, grad_u):
    model, ref = _struct_model(loss, grad_u)
    batch = collate(synthetic_samples(100, 3, k=8, seed=4))
    model = model.to(DEV).train()
    out = model.loss_fn.crps(model(batch.to(DEV)), batch.y.to(DEV))
    out.backward()
    want = ref.crps(ref(batch), batch.y)
    want.backward()
    assert abs(out.item() - want.item()) <= 1e-5 * abs(want.item())
    g = torch.cat([p.grad.reshape(-1).cpu() for p in model.parameters()])
    r = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    assert ((g - r).abs().max() / r.abs().max()).item() <= 1e-5


def test_dropin_training_loop_builds_the_graph_once():
    from raincast_gnn.graph import graph_cache
    model, _ = _struct_model("MixedLoss", "False")
    model = model.to(DEV).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4)
    samples = synthetic_samples(150, 8, k=10, seed=6)
    host = [collate(samples[:4]), collate(samples[4:])]
    graph_cache.clear()
    before = dict(graph_cache.stats)
    losses = []
    for i in range(6):                      # train.py:61-71
        batch = host[i % 2].to(DEV)
        loss = model.loss_fn.crps(model(batch), batch.y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    d = {k: graph_cache.stats[k] - before[k] for k in before}
    assert d["builds"] == 1 and d["content_hits"] == 5, d
    assert all(v == v for v in losses)
    # the fused layer form was used (D = 128, Linear-BN-ReLU-Linear nn)
    assert Fn.fused_forward_ok(graph_cache.get(batch.edge_index, batch.edge_attr.float(),
                                               batch.num_nodes), batch.num_nodes, 128)


@pytest.mark.parametrize("order", ["dataset", "locality"])
def test_dropin_cpp_binding_same_bits_as_python_function(order, monkeypatch):
    """The C++ autograd binding of the layer (raincast_gnn.torch_ext, csrc/torch/
    gine_torch.cpp) issues the Python Function's launches: the drop-in model's predictions,
    loss, every gradient and the BatchNorm buffers are the same bits over three training
    steps, with the graph in the dataset order (gather backward) and in the locality order
    (window backward)."""
    import copy
    from raincast_gnn import nn as rnn, torch_ext
    from raincast_gnn.dropin import reference_struct_from_params
    from raincast_gnn.params import EXPERIMENTS
    from helpers import engine_order_batch
    assert torch_ext.get() is not None, "the C++ binding was not built / did not load"
    batch = collate(synthetic_samples(500, 8, k=10, seed=6))
    if order == "locality":
        batch = engine_order_batch(batch)
    batch = batch.to(DEV)
    torch.manual_seed(3)
    base = reference_struct_from_params(EXPERIMENTS["24h_mixed"]).to(DEV).train()

    def run(use_ext):
        monkeypatch.setattr(rnn, "USE_TORCH_EXT", use_ext)
        m = copy.deepcopy(base)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
        out = []
        for _ in range(3):
            pred = m(batch)
            loss = m.loss_fn.crps(pred, batch.y)
            opt.zero_grad()
            loss.backward()
            out.append([pred.detach().clone(), loss.detach().clone()]
                       + [p.grad.clone() for p in m.parameters()]
                       + [b.clone() for b in m.buffers()])
            opt.step()
        torch.cuda.synchronize()
        return out

    py, cpp = run(False), run(True)
    for a_step, b_step in zip(cpp, py):
        for a, b in zip(a_step, b_step):
            assert torch.equal(a, b)


def test_cpp_binding_backward_after_graph_eviction():
    """the C++ autograd node must hold the window plan it ran the forward with.
    Forward through the C++ binding, evict every graph from the cache and collect it, fill
    the caching allocator's freed blocks with garbage, then backward: the gradients are the
    same bits as with the graph alive."""
    import gc
    from raincast_gnn import GINEConv, torch_ext
    from raincast_gnn.graph import graph_cache
    from helpers import engine_order_batch
    assert torch_ext.get() is not None, "the C++ binding was not built / did not load"
    # cfg2's batch (32 x 500 stations, locality order): the window backward applies
    batch = engine_order_batch(collate(synthetic_samples(500, 32, k=10, seed=6))).to(DEV)
    D = 128
    torch.manual_seed(8)
    mlp = torch.nn.Sequential(torch.nn.Linear(D, D), torch.nn.BatchNorm1d(D), torch.nn.ReLU(),
                              torch.nn.Linear(D, D))
    conv = GINEConv(nn=mlp, train_eps=True, edge_dim=1).to(DEV).train()
    state = {k: v.clone() for k, v in conv.state_dict().items()}
    x0 = torch.randn(batch.num_nodes, D, device=DEV)
    gy = torch.randn(batch.num_nodes, D, device=DEV)

    def run(evict):
        conv.load_state_dict(state)
        conv.zero_grad(set_to_none=True)
        graph_cache.clear()
        x = x0.clone().requires_grad_()
        ei, ea = batch.edge_index.clone(), batch.edge_attr.clone()
        g = graph_cache.get(ei, ea.float(), batch.num_nodes)
        assert g.window_plan("out", D) is not None, "the window backward must apply"
        y = conv.forward_residual_relu(x, ei, ea)
        assert type(y.grad_fn).__name__ != "GineLayerBackward", "C++ binding expected"
        if evict:
            del g, ei, ea
            graph_cache.clear()
            gc.collect()
            junk = [torch.full((1 << 20,), float("nan"), device=DEV) for _ in range(64)]
            del junk
        y.backward(gy)
        torch.cuda.synchronize()
        return [x.grad.clone()] + [p.grad.clone() for p in conv.parameters()]

    ref = run(False)
    got = run(True)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
