#!/usr/bin/env bash
# r02_s43: three-stage folded chain backward (one launch) -- parity + A/B vs two launches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s43; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_training.py -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
GINE_CHAIN_B3=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > $O/pytest_b2.log 2>&1; rc=$?
tail -1 $O/pytest_b2.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s43_ab "GINE_CHAIN_B3=1" "GINE_CHAIN_B3=0"
