#!/usr/bin/env bash
# r02_s61: grid-size knobs re-checked on the current tree (row GEMMs, chain kernels)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_ab.sh r02_s61_ab "RAINCAST_X=0" "GINE_ROWGEMM_BLOCKS=512" "GINE_CHAIN_BLOCKS=512"
