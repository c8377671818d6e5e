"""CPU: the training driver (raincast_gnn/train.py, the counterpart of train.py:55-208) on
the CPU oracle model -- epoch loop, split, loader determinism, sanity forward, checkpoint on
improvement, rank sharding.  The same driver on the HIP engine: tests/test_gpu_train.py."""
import os

import torch

from raincast_gnn import train as T
from raincast_gnn.batching import DeviceDataset, DeviceLoader
from raincast_gnn.data import synthetic_samples


class _OracleModel(torch.nn.Module):
    """The oracle GNN with the engine model's ``loss_fn.crps`` attribute."""

    def __init__(self, **kw):
        super().__init__()
        from oracle import gine_cpu as O
        self.net = O.OracleGNN(35, 32, 2, "MixedLoss", "False", 1.71, 0.5)
        self.loss_fn = type("L", (), {"crps": staticmethod(self.net.crps)})()

    def forward(self, data):
        return self.net(data)


def test_split_and_loader_are_deterministic_and_shard():
    ds = DeviceDataset(synthetic_samples(20, 23, k=4, seed=0), "cpu")
    tr, va = T.split_train_val(ds, generator=torch.Generator().manual_seed(1))
    assert (len(tr), len(va)) == (21, 2)          # n_val = int(0.1 * 23)
    a = [b.x.clone() for b in DeviceLoader(tr, 4, seed=5)]
    b = [b.x.clone() for b in DeviceLoader(tr, 4, seed=5)]
    assert len(a) == 6 and all(torch.equal(u, v) for u, v in zip(a, b))
    # two ranks: the same global batches, contiguous shards; the 1-graph tail is skipped
    full = list(DeviceLoader(tr, 4, seed=5))
    r0 = list(DeviceLoader(tr, 4, seed=5, rank=0, world=2))
    r1 = list(DeviceLoader(tr, 4, seed=5, rank=1, world=2))
    assert len(r0) == len(r1) == 5
    for f, p, q in zip(full, r0, r1):
        assert torch.equal(torch.cat([p.x, q.x]), f.x)


def test_fit_checkpoints_best_and_sanity_forward_bumps_bn(tmp_path):
    torch.manual_seed(0)
    ds = DeviceDataset(synthetic_samples(30, 12, k=5, seed=2), "cpu")
    tr, va = T.split_train_val(ds, generator=torch.Generator().manual_seed(0))
    model = _OracleModel()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    bn = model.net.conv.convolutions[0].nn[1]
    out = T.fit(model, opt, DeviceLoader(tr, 4, seed=1), DeviceLoader(va, 4, shuffle=False),
                "cpu", 3, ckpt_dir=str(tmp_path), run_id="t", example=tr.batch(torch.tensor([0])))
    steps = 3 * len(DeviceLoader(tr, 4))
    assert int(bn.num_batches_tracked) == 1 + steps   # the train-mode sanity forward + steps
    h = out["history"]
    assert len(h["train"]) == len(h["val"]) == 3
    assert out["best_val_loss"] == min(h["val"])
    path = out["best_ckpt_path"]
    assert path == os.path.join(str(tmp_path), "run_t-best.ckpt") and os.path.exists(path)
    state = torch.load(path, weights_only=True)
    assert set(state) == set(model.state_dict())


def test_train_one_epoch_mean_matches_reference_loop():
    torch.manual_seed(3)
    ds = DeviceDataset(synthetic_samples(25, 7, k=4, seed=4), "cpu")
    m1, m2 = _OracleModel(), _OracleModel()
    m2.load_state_dict(m1.state_dict())
    o1 = torch.optim.AdamW(m1.parameters(), lr=1e-3)
    o2 = torch.optim.AdamW(m2.parameters(), lr=1e-3)
    got = T.train_one_epoch(m1, DeviceLoader(ds, 3, seed=9), o1, "cpu")
    # train.py:55-74 verbatim (loss.item() per step)
    m2.train()
    total, n = 0.0, 0
    for batch in DeviceLoader(ds, 3, seed=9):
        loss = m2.loss_fn.crps(m2(batch), batch.y)
        o2.zero_grad()
        loss.backward()
        o2.step()
        total += loss.item()
        n += 1
    assert got == total / n


def test_data_parallel_loader_needs_equal_shards_and_a_batch():
    import pytest
    ds = DeviceDataset(synthetic_samples(20, 5, k=4, seed=0), "cpu")
    with pytest.raises(ValueError, match="multiple"):
        DeviceLoader(ds, 4, rank=0, world=3)        # 4 graphs over 3 ranks: 2/1/1 every step
    # 8 ranks, batches of 8, 5 samples: the only batch has fewer graphs than ranks
    loader = DeviceLoader(ds, 8, rank=0, world=8)
    assert list(loader) == []
    with pytest.raises(ValueError, match="no batch"):
        T.train_one_epoch(_OracleModel(), loader, None, "cpu")


def test_cli_rejects_a_world_size_that_does_not_divide_the_batch(tmp_path, monkeypatch):
    """24h_mixed's batch_size 8 over 3 ranks: the train CLI stops before any process group
    or device is set up, naming the constraint."""
    import json
    import pytest
    from raincast_gnn.params import EXPERIMENTS
    (tmp_path / "params.json").write_text(json.dumps(EXPERIMENTS["24h_mixed"]))
    monkeypatch.setenv("WORLD_SIZE", "3")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    with pytest.raises(SystemExit, match="not a multiple of the 3"):
        T.main(["--dir", str(tmp_path), "--run_id", "x"])


def test_step_runner_allreduce_choice():
    """The data-parallel all-reduce form is chosen up front, as bench.py's --allreduce:
    split by default, graph on request, anything else rejected."""
    import pytest
    m = torch.nn.Linear(2, 2)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    assert T.StepRunner(m, opt).allreduce == "split"
    assert T.StepRunner(m, opt, allreduce="graph").allreduce == "graph"
    with pytest.raises(ValueError):
        T.StepRunner(m, opt, allreduce="sometimes")
