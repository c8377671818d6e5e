"""CPU: ``bench.py --gpus N`` starts N ranks itself (one child process per GPU), the ranks
agree on the world size, and rank 0's JSON line carries ``n_gpus == --gpus``.  ``--dry-run``
replaces the GPU step by the gradient all-reduce over gloo, so the launcher, rank / world /
shard plumbing and the max-over-ranks aggregation run here without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("gpus", [1, 2])
def test_dry_run_reports_requested_ranks(gpus):
    p = _run(["--gpus", str(gpus), "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["n_gpus"] == gpus
    assert d["config"]["parallelism"] == f"dp{gpus}"
    assert d["config"]["global_batch"] == 32 * gpus          # weak scaling: 32 graphs per rank
    assert d["config"]["nodes_global"] == 500 * 32 * gpus
    assert d["config"]["allreduce_floats"] == d["config"]["parameters"] == 209800
    assert d["backend"] == ("gloo" if gpus > 1 else None)
    assert d["launcher"] is (gpus > 1)
    assert d["value"] > 0
    # the N > 1 decomposition: the all-reduce time and every rank's p50
    assert d["allreduce_ms_p50"] is not None and d["allreduce_ms_p50"] >= 0
    if gpus > 1:
        assert [r["rank"] for r in d["per_rank"]] == list(range(gpus))
        assert all(r["allreduce_ms_p50"] >= 0 for r in d["per_rank"])
    else:
        assert d["per_rank"] is None


@pytest.mark.timeout(300)
def test_dry_run_strong_scaling_splits_global_batch():
    p = _run(["--gpus", "2", "--dry-run", "--config", "4", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 256 and d["config"]["graphs_per_gpu"] == 128


@pytest.mark.timeout(300)
def test_failed_rank_fails_the_launch():
    p = _run(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"],
             {"RAINCAST_BENCH_DRY_FAIL_RANK": "1"}, timeout=200)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "must agree" in p.stderr


def test_stalled_steps_decomposition():
    """A stalled step is reported with its fwd+bwd stream time, the host wait for it (gloo)
    and the collective's own times; steps within 10x the median are not."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    steps = [2.0, 2.1, 600.0, 2.05, 1.9]
    ar = [(0.7, 0.8, 1.0, 1.2), (0.7, 0.9, 1.1, 1.3), (0.8, 1.0, 598.0, 1.25),
          (0.7, 0.8, 1.0, 1.2), (0.7, 0.8, 1.0, 1.2)]
    out = bench.stalled_steps(steps, ar)
    assert out["count"] == 1 and out["steps"][0]["step"] == 2
    rec = out["steps"][0]
    assert rec["fwd_bwd_host_wait_ms"] == 598.0 and rec["fwd_bwd_stream_ms"] == 1.25
    assert rec["allreduce_stream_ms"] == 0.8 and rec["allreduce_host_ms"] == 1.0
    assert bench.stalled_steps([2.0, 2.1, 1.9], ar[:3]) is None
