#!/usr/bin/env bash
# Determinism probe of the split-bf16 build and its two fp32 variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s07}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 150 python tools/determinism.py > $O/det_x3.txt 2>&1; st $? det_x3
grep -v amdgpu.ids $O/det_x3.txt | grep -v " same" 
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsf32/libgine_hip.so timeout -k 10 150 python tools/determinism.py > $O/det_dsf32.txt 2>&1; st $? det_ds
echo "--- dsf32"; grep -v amdgpu.ids $O/det_dsf32.txt | grep -v " same"
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/wgf32/libgine_hip.so timeout -k 10 150 python tools/determinism.py > $O/det_wgf32.txt 2>&1; st $? det_wg
echo "--- wgf32"; grep -v amdgpu.ids $O/det_wgf32.txt | grep -v " same"
exit 0
