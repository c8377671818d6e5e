#!/usr/bin/env bash
# r02_s33: cfg2 step kernel trace with the folded chain (where do the extra us go?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s33; mkdir -p $O
for v in 1 0; do
  RAINCAST_CHAIN_FOLD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/bench$v.json 2> $O/bench$v.err || exit $?
  python tools/step_breakdown.py $O/prof$v/run_kernel_trace.csv > $O/step$v.txt || exit $?
done
echo done
