#!/usr/bin/env bash
# r02_s32: folded dense chain -- chain + training parity tests, fold on/off A/B at cfg2
# (and cfg3 with S32_CFG3=1), cfg2 kernel trace with the fold on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${S32_TAG:-r02_s32}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_training.py -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh ${T}_ab2 "RAINCAST_CHAIN_FOLD=1" "RAINCAST_CHAIN_FOLD=0" || exit $?
if [ "${S32_CFG3:-0}" = 1 ]; then
  BENCH_ARGS="--config 3 --steps 30" bash tools/gpu_ab.sh ${T}_ab3 "RAINCAST_CHAIN_FOLD=1" "RAINCAST_CHAIN_FOLD=0" || exit $?
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench.json 2> $O/bench.err || exit $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step.txt || exit $?
grep -i "chain\|median" $O/step.txt
