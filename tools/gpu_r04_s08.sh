#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s08}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
for v in x3 wgf32; do
  if [ $v != x3 ]; then export GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
  echo "--- $v"; timeout -k 10 120 python tools/determinism_layer.py 2>&1 | grep -v amdgpu.ids | tee $O/layer_$v.txt; st ${PIPESTATUS[0]} $v
  echo "--- $v flat"; timeout -k 10 120 python tools/determinism_layer.py --flat 2>&1 | grep -v amdgpu.ids | tee $O/layer_flat_$v.txt; st ${PIPESTATUS[0]} $v
done
