#!/usr/bin/env bash
# Round-2 closing check: GPU parity suite, smoke, default bench (with the CPU leg), cfg3 and
# cfg5 benches, and the cfg2 kernel trace + step breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r02_final}
O=gpurun_out/$T; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; st $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; st $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; st $?
for c in 3 5; do timeout -k 10 300 python bench.py --no-cpu --config $c --steps 20 > $O/bench$c.json 2> $O/bench$c.err; st $?; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err; st $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step.txt
head -1 $O/step.txt
for f in $O/bench.json $O/bench3.json $O/bench5.json; do python -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"; done
