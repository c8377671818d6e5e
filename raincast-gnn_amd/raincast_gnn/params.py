"""Experiment configurations.

``load_params`` reads a reference ``params.json`` as-is (train.py:127-134); the twelve
shipped configurations (trained_models/{24,72,120}h_{normal,normal_mixed,mixed,mixed_u}/
params.json) share every key except ``loss``, ``grad_u`` and ``max_dist``, which
:data:`EXPERIMENTS` records.  :data:`BENCH_CONFIGS` are the benchmark shapes of
BASELINE.json / SURVEY.md section 8.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, replace

_COMMON = {"batch_size": 8, "gnn_hidden": 128, "gnn_layers": 4, "heads": 8, "lr": 0.0001,
           "max_dist": 100, "max_epochs": 20, "u": 1.71, "xi": 0.5}

_VARIANTS = {
    "normal": {"loss": "NormalCRPS", "grad_u": "False"},
    "normal_mixed": {"loss": "MixedNormalCRPS", "grad_u": "False"},
    "mixed": {"loss": "MixedLoss", "grad_u": "False"},
    "mixed_u": {"loss": "MixedLoss", "grad_u": "True"},
}

EXPERIMENTS: dict[str, dict] = {}
for _lt in ("24h", "72h", "120h"):
    for _name, _v in _VARIANTS.items():
        cfg = dict(_COMMON, **_v)
        if _lt == "24h" and _name == "normal_mixed":
            cfg["max_dist"] = 1  # trained_models/24h_normal_mixed/params.json:6
        EXPERIMENTS[f"{_lt}_{_name}"] = cfg


def load_params(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


@dataclass(frozen=True)
class BenchConfig:
    name: str
    experiment: str
    num_stations: int
    k: int
    graphs_per_gpu: int
    gnn_layers: int | None = None   # override of params.json
    note: str = ""
    gnn_hidden: int | None = None   # override of params.json (the D=64 sweep, BASELINE.md:47)

    def params(self) -> dict:
        p = dict(EXPERIMENTS[self.experiment])
        if self.gnn_layers is not None:
            p["gnn_layers"] = self.gnn_layers
        if self.gnn_hidden is not None:
            p["gnn_hidden"] = self.gnn_hidden
        return p

    def with_hidden(self, hidden: int | None) -> "BenchConfig":
        """This configuration at hidden size ``hidden`` (None or params.json's own value:
        unchanged); the name records the sweep point, e.g. ``cfg2-D64``."""
        if hidden is None or hidden == EXPERIMENTS[self.experiment]["gnn_hidden"]:
            return self
        return replace(self, gnn_hidden=int(hidden), name=f"{self.name}-D{int(hidden)}")


BENCH_CONFIGS = {
    1: BenchConfig("cfg1", "24h_mixed", 500, 10, 1, note="CPU-runnable reference case"),
    2: BenchConfig("cfg2", "24h_mixed", 500, 10, 32, note="headline single-GPU workload"),
    3: BenchConfig("cfg3", "72h_mixed_u", 2000, 16, 64, note="HBM-bound roofline run"),
    4: BenchConfig("cfg4", "24h_mixed", 500, 10, 256, note="global batch 256, strong scaling"),
    5: BenchConfig("cfg5", "120h_normal_mixed", 10000, 32, 8, gnn_layers=3,
                   note="10k-station dense graph, 3 GINE layers"),
}
