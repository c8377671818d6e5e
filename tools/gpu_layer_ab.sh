#!/usr/bin/env bash
# Step A/B of the one-launch layer kernels (options.LAYER_FWD / LAYER_BWD) on one box, each
# variant twice interleaved, then a rocprofv3 kernel trace of the default step.
#   tools/gpu_layer_ab.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-layer_ab}; shift || true
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  for v in "LAYER_FWD=1 LAYER_BWD=1" "LAYER_FWD=0 LAYER_BWD=0" "LAYER_FWD=1 LAYER_BWD=0" "LAYER_FWD=0 LAYER_BWD=1"; do
    timeout -k 10 200 python tools/bench_with.py $v -- --no-cpu --no-strong --steps 50 "$@" > $O/b.json 2>$O/b.err || { echo "bench failed: $v"; tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['step_ms_p10_p50_p90'])" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong "$@" > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
