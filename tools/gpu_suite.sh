#!/usr/bin/env bash
# The whole GPU test suite in one process (parity tables into gpurun_out/<tag>/).
#   tools/gpu_suite.sh <tag> [pytest args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-suite}; shift || true
O=gpurun_out/$TAG; mkdir -p $O
GINE_PARITY_REPORT=$O timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc
