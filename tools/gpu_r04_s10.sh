#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s10}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/occ2/libgine_hip.so DET_SAVE=$O/ref timeout -k 10 120 python tools/determinism_layer.py --flat > $O/ref.txt 2>&1; st $? ref
DET_SAVE=$O/x3 timeout -k 10 120 python tools/determinism_layer.py --flat > $O/x3.txt 2>&1; st $? x3
python tools/det_compare.py $O/ref_0.pt $O/x3_0.pt $O/x3_1.pt $O/x3_2.pt 2>&1 | tee $O/compare.txt
rm -f $O/*.pt
