#!/usr/bin/env bash
# r02_s40: does the combined backward overlap its engine with the message passing when 3
# workgroups fit per CU?  (occupancy-6 variant + window plans within 53 KB of LDS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SMALL="GINE_MP_WINDOW_ROW_BYTES=36864 GINE_MP_WINDOW_LDS_BYTES=53000"
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var/occ6/libgine_hip.so
bash tools/gpu_ab.sh r02_s40_ab "RAINCAST_X=0" "$SMALL" "$SMALL GINE_HIP_LIB=$V"
