#!/usr/bin/env bash
# r02_s52: degree-balanced work order in the window backward -- GPU suite, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s52; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s52_ab "GINE_MP_WINDOW_SLOTS=1" "GINE_MP_WINDOW_SLOTS=0"
