#!/usr/bin/env bash
# Determinism probes of the combined window backward: for each library
# variant under raincast_gnn/_native/var (plus the default build), three forward+backward runs
# of one cfg2 GINE layer with dx dumps; det_compare lists the rows / columns that differ from
# the default build's first run.
#   tools/gpu_det_probe.sh <tag> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
V=raincast-gnn_amd/raincast_gnn/_native/var
unset GINE_HIP_LIB
DET_SAVE=$O/ref timeout -k 10 120 python tools/determinism_layer.py --flat > $O/default.txt 2>&1; st $? default
grep -v amdgpu.ids $O/default.txt | cut -c1-400
for v in "$@"; do
  echo "--- $v"
  GINE_HIP_LIB=$V/$v/libgine_hip.so DET_SAVE=$O/$v timeout -k 10 120 python tools/determinism_layer.py --flat > $O/$v.txt 2>&1; st $? $v
  grep -v amdgpu.ids $O/$v.txt | cut -c1-400
  python tools/det_compare.py $O/ref_0.pt $O/${v}_0.pt $O/${v}_1.pt $O/${v}_2.pt 2>&1 | tee $O/${v}_cmp.txt
  rm -f $O/${v}_*.pt
done
rm -f $O/ref_*.pt
