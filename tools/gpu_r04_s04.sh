#!/usr/bin/env bash
# Round-4 session 4: the doubly folded chain -- its GPU tests and the model parity tables,
# a step A/B against the single fold, a kernel trace of the default step, the drop-in line.
#   tools/gpu_r04_s04.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04_s04}
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > $O/pytest_chain.log 2>&1; rc=$?; tail -3 $O/pytest_chain.log; st $rc chain
[ $rc -eq 0 ] || exit 1
GINE_PARITY_REPORT=$O timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > $O/pytest_cfg.log 2>&1; rc=$?; tail -3 $O/pytest_cfg.log; st $rc configs
for rep in 1 2; do
  for v in "chain.FOLD2=1" "chain.FOLD2=0"; do
    timeout -k 10 200 python tools/bench_with.py $v -- --no-cpu --no-strong --steps 50 > $O/b.json 2>$O/b.err || { echo "bench failed: $v"; tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['step_ms_p10_p50_p90'])" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
timeout -k 10 300 python bench.py --dropin --steps 30 --warmup 5 > $O/bench_dropin.json 2> $O/bench_dropin.err; st $? bench_dropin
cat $O/bench_dropin.json
