#!/usr/bin/env bash
# Is the run-to-run difference of the combined window backward tied to two workgroups per CU
# each holding more than 64 KiB of LDS?  fp32 engine, LDS floor 72 KiB / 64 KiB vs default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s23}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
V=raincast-gnn_amd/raincast_gnn/_native/var
for v in default lds64 lds72; do
  if [ $v != default ]; then export GINE_HIP_LIB=$V/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
  echo "--- $v"; timeout -k 10 120 python tools/determinism_layer.py --flat 2>&1 | grep -v amdgpu.ids | cut -c1-60 | tee $O/layer_flat_$v.txt; st ${PIPESTATUS[0]} $v
done
