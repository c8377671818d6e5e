#!/usr/bin/env bash
# Full GPU check of the current tree: parity suite, smoke, cfg2 bench (no CPU leg).
#   tools/gpu_check.sh <tag> [extra bench configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-check}; shift || true
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; st $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; st $rc
timeout -k 10 300 python bench.py --no-cpu > $O/bench2.json 2> $O/bench2.err; st $?
for c in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu --config $c --steps 20 > $O/bench$c.json 2> $O/bench$c.err; st $?
done
for f in $O/bench*.json; do python -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"; done
