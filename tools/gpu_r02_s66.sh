#!/usr/bin/env bash
# r02_s66: BN accumulator replicas and engine workgroup target re-checked on the current tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
bash tools/gpu_ab.sh r02_s66_ab "RAINCAST_X=0" "GINE_HIP_LIB=$V/rep2/libgine_hip.so" "GINE_HIP_LIB=$V/wg384/libgine_hip.so" "GINE_HIP_LIB=$V/wg320/libgine_hip.so"
