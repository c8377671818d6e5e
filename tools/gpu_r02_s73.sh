#!/usr/bin/env bash
# r02_s73: head backward run by the CRPS pass for the unit seed (gine_crps_head_fwd_grad) --
# new tests, full GPU suite, A/B RAINCAST_CRPS_HEAD=1 vs 0, cfg2 trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s73; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "crps_pass or crps or head" > $O/pytest_head.log 2>&1; rc=$?
tail -2 $O/pytest_head.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/gpu_ab.sh r02_s73_ab "RAINCAST_CRPS_HEAD=1" "RAINCAST_CRPS_HEAD=0" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_prof.json 2> $O/bench_prof.err || exit $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step.txt
head -1 $O/step.txt; grep -E "crps|head" $O/step.txt
