#!/usr/bin/env bash
# r02_s76: CRPS pass with the head backward at cfg3 / cfg5 (many 64-node workgroups): A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
BENCH_ARGS="--config 3 --steps 20" bash tools/gpu_ab.sh r02_s76_ab3 "RAINCAST_CRPS_HEAD=1 RAINCAST_CRPS_HEAD_MAX_NODES=1000000000" "RAINCAST_CRPS_HEAD=0" || exit $?
BENCH_ARGS="--config 5 --steps 20" bash tools/gpu_ab.sh r02_s76_ab5 "RAINCAST_CRPS_HEAD=1 RAINCAST_CRPS_HEAD_MAX_NODES=1000000000" "RAINCAST_CRPS_HEAD=0"
