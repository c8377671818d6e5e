#!/usr/bin/env bash
# r02_s44: is the window message-passing backward occupancy-bound?  Extra dynamic LDS per
# workgroup (GINE_WIN_EXTRA_LDS) lowers the workgroups per CU; standalone MP timing + the
# bench's per-kernel table (combined backward).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s44; mkdir -p $O
for E in 0 40960 81920; do
  GINE_WIN_EXTRA_LDS=$E timeout -k 10 200 python tools/mp_micro.py --configs 2 --tiles 128 --rcm > $O/mp_$E.jsonl 2> $O/mp_$E.err || exit $?
  GINE_WIN_EXTRA_LDS=$E timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 30 > $O/bench_$E.json 2> $O/bench_$E.err || exit $?
done
echo done
