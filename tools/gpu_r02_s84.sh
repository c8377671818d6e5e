#!/usr/bin/env bash
# r02_s84: AdamW two-level ticket vs one ticket word: optimizer / training tests, kernel
# stats of the cfg2 step under each, then the cfg2 step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s84; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_train.py -m gpu -q -rf -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for t in two flat; do
  GINE_ADAMW_TICKET=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
  echo "$t: $(grep -E 'k_adamw' $O/prof_$t/run_kernel_stats.csv | cut -d, -f2-7)"
done
bash tools/gpu_ab.sh r02_s84_ab2 "GINE_ADAMW_TICKET=two" "GINE_ADAMW_TICKET=flat"
