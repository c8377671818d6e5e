"""CPU: the fp64 branch oracle of tests/helpers.check_training_step, exercised with the fp32
CPU oracle standing in for the engine.

At the benchmark's full size (cfg2: 32 x 500 stations, k=10) the fp32 restatement's own
gradients differ from the plain fp64 oracle's by up to 1e-4..5e-3 -- a handful of ReLU
decisions within fp32 rounding of zero go the other way and each moves one gradient entry
by the whole upstream gradient.  Against the fp64 oracle that follows the fp32 run's
decisions (each one that differs checked against its per-decision forward error bound,
EngineTies) every gradient is within 1e-5, which is the bar the GPU tests hold the engine
to (tests/test_gpu_configs.py).
"""
import numpy as np
import pytest
import torch

from helpers import branch_grad_table, oracle32_ties, _oracle_step
from raincast_gnn.data import synthetic_batch
from raincast_gnn.params import BENCH_CONFIGS, EXPERIMENTS

TOL = 1e-5


def _ref(params, seed=42):
    from oracle import gine_cpu as O
    torch.manual_seed(seed)
    return O.OracleGNN(35, params["gnn_hidden"], params["gnn_layers"], params["loss"],
                       params["grad_u"], params["u"], params["xi"])


@pytest.mark.parametrize("graphs", [2, 32], ids=["b2", "cfg2-full"])
def test_fp32_oracle_within_tol_of_its_branch_oracle(graphs):
    params = dict(EXPERIMENTS["24h_mixed"])
    c = BENCH_CONFIGS[2]
    batch = synthetic_batch(c.num_stations, graphs, k=c.k, seed=102)
    ref = _ref(params)
    ties, r32 = oracle32_ties(ref, batch)
    r64 = _oracle_step(ref, batch, torch.float64)[0]
    rb = _oracle_step(ref, batch, torch.float64, record=True, hooks=ties.hooks)[0]
    grads = {n: p.grad for n, p in r32.named_parameters()}
    # (the plain bound is the HIP engine's; this "engine" is the fp32 CPU oracle itself)
    worst, table, fails = branch_grad_table(grads, rb, r32, r64, TOL, plain_tol=None)
    print(table)
    print(ties.table())
    assert not fails, table
    # every layer input of the fp32 run within tol of the branch oracle's
    assert max(e for _, e in ties.input_err) <= TOL
    n_dec = sum(n for _, n, _, _ in ties.log)
    assert n_dec > 0 and sum(k for _, _, k, _ in ties.log) <= 1e-5 * n_dec


def test_branch_oracle_rejects_a_decision_outside_the_bound():
    """A decision flipped far from zero (not a rounding tie) fails the bound check."""
    params = dict(EXPERIMENTS["24h_mixed"])
    batch = synthetic_batch(120, 2, k=10, seed=5)
    ref = _ref(params)
    ties, _ = oracle32_ties(ref, batch)
    E = ties.layers[1]
    x = E["x"]
    # the message with the largest |pre| of edge 0, flipped
    src = batch.edge_index[0]
    pre = x[src[0]]
    c = int(pre.abs().argmax())
    E["msg_on"] = E["msg_on"].clone()
    E["msg_on"][0, c] = ~E["msg_on"][0, c]
    with pytest.raises(AssertionError, match="forward rounding bound"):
        _oracle_step(ref, batch, torch.float64, record=True, hooks=ties.hooks)


def test_deepset_mask_layout_decoding():
    """The decoding of gine_deepset_fwd's ReLU bit mask (EngineTies.read) inverts the layout
    include/gine_hip.h documents for gine_deepset_mask_layout."""
    from raincast_gnn import _lib
    from helpers import ctypes_int, decode_deepset_mask
    for N, M, H in ((500, 11, 128), (16000, 11, 128), (37, 5, 64)):
        G = ctypes_int(lambda out: _lib.call("gine_deepset_mask_layout", N, H, out))
        assert G in (4, 8, 16)
        tpg = (G * M + 15) // 16
        groups = -(-N // (2 * G))
        rng = np.random.default_rng(N)
        on = rng.random((N, M, H)) < 0.5
        # encode by the documented layout
        words = np.zeros((groups, tpg, 2 * H), dtype=np.uint16)
        n, m, c = np.nonzero(on)
        g, rem = n // (2 * G), n % (2 * G)
        h, jn = rem // G, rem % G
        j = jn * M + m
        t, q = j // 16, j % 16
        thread = (c // 32) * 64 + 32 * h + c % 32
        np.bitwise_or.at(words, (g, t, thread), (1 << q).astype(np.uint16))
        bits = decode_deepset_mask(words.reshape(-1), N, M, H, G)
        assert np.array_equal(bits, on)
