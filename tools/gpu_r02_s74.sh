#!/usr/bin/env bash
# r02_s74: kernel traces of the cfg2 step with the head backward in the CRPS pass and apart
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s74; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -m gpu -x -q --timeout 120 --timeout-method thread -k "crps or head" > $O/pytest_head.log 2>&1 || { tail -20 $O/pytest_head.log; exit 1; }
tail -1 $O/pytest_head.log
for v in 1 0; do
RAINCAST_CRPS_HEAD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_prof$v.json 2> $O/bench_prof$v.err || exit $?
python tools/step_breakdown.py $O/prof$v/run_kernel_trace.csv > $O/step$v.txt
head -1 $O/step$v.txt; grep -E "crps|head" $O/step$v.txt
done
