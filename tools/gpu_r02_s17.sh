#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s17; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; st $rc
timeout -k 10 300 python tools/mp_micro.py --configs 2,3,5 --tiles 128 --rcm > $O/mp_rcm.jsonl 2> $O/mp_rcm.err; st $?
cat $O/mp_rcm.jsonl
timeout -k 10 300 python bench.py --no-cpu > $O/bench2.json 2> $O/bench2.err; st $?
timeout -k 10 300 python bench.py --no-cpu --config 3 --steps 20 > $O/bench3.json 2> $O/bench3.err; st $?
timeout -k 10 300 python bench.py --no-cpu --config 5 --steps 20 > $O/bench5.json 2> $O/bench5.err; st $?
echo done
