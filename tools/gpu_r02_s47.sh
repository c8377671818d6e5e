#!/usr/bin/env bash
# r02_s47: issue priority in the combined backward (engine waves first / message-passing
# waves first), A/B against the library build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
bash tools/gpu_ab.sh r02_s47_ab "RAINCAST_X=0" "GINE_HIP_LIB=$V/prio1/libgine_hip.so" "GINE_HIP_LIB=$V/prio2/libgine_hip.so"
