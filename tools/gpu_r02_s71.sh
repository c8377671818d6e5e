#!/usr/bin/env bash
# r02_s71: DeepSet folding launch deals its fold workgroups first and aliases their LDS with
# the walk's -- GPU suite, A/B RAINCAST_CHAIN_F3=1 vs 0, cfg2 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s71; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s71_ab "RAINCAST_CHAIN_F3=1" "RAINCAST_CHAIN_F3=0" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step.txt
head -12 $O/step.txt
