#!/usr/bin/env bash
# N>1 readiness on one GPU box: the exact N>1 code path as a forced
# world-1 RCCL group in both all-reduce forms (split / graph: same final-loss bits?), and two
# gloo ranks sharing the GPU (host threads split over the ranks, cgroup throttle counters).
#   tools/gpu_dist_check.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-dist}
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -eq 0 ] || { echo "step failed rc=$rc"; exit $rc; }; }
for f in split graph; do
  timeout -k 10 300 python bench.py --no-cpu --no-strong --steps 50 --force-allreduce \
    --allreduce $f > $O/rccl1_$f.json 2> $O/rccl1_$f.err; st $?
done
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --no-cpu --no-strong --steps 50 \
  > $O/gloo2.json 2> $O/gloo2.err; st $?
python - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for n in ("rccl1_split", "rccl1_graph", "gloo2"):
    d = json.loads(open(f"{o}/{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["step_ms_p10_p50_p90"], "loss", repr(d["final_loss"]),
          "ar", d["allreduce_ms_p50"], "thr", d.get("host_threads_per_rank"), d.get("cpu_share"),
          "throttle", d.get("cpu_throttle_timed"), "stalls", (d["stalled_steps"] or {}).get("count"))
PY
