#!/usr/bin/env bash
# r02_s72: chain weight-gradient engine on a side stream (parallel graph branch beside the
# DeepSet backward) -- bit-identity test, A/B RAINCAST_CHAIN_SIDE_STREAM=1 vs 0, trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s72; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k side_stream > $O/pytest_side.log 2>&1; rc=$?
tail -2 $O/pytest_side.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s72_ab "RAINCAST_CHAIN_SIDE_STREAM=1" "RAINCAST_CHAIN_SIDE_STREAM=0" || exit $?
RAINCAST_CHAIN_SIDE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step.txt
head -3 $O/step.txt
