#!/usr/bin/env bash
# r02_s67: folded chain forward in one launch (W' folded by the DeepSet launch) -- GPU suite,
# A/B RAINCAST_CHAIN_F3=1 vs 0, cfg3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s67; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s67_ab "RAINCAST_CHAIN_F3=1" "RAINCAST_CHAIN_F3=0" || exit $?
BENCH_ARGS="--config 3 --steps 20" bash tools/gpu_ab.sh r02_s67_ab3 "RAINCAST_CHAIN_F3=1" "RAINCAST_CHAIN_F3=0"
