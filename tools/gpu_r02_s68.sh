#!/usr/bin/env bash
# r02_s68: CRPS forward writes the unit-seed gradient (no crps_bwd launch) -- GPU suite, A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s68; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/gpu_ab.sh r02_s68_ab "RAINCAST_CRPS_UNIT_GRAD=1" "RAINCAST_CRPS_UNIT_GRAD=0"
