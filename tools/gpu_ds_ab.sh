#!/usr/bin/env bash
# DeepSet kernel micro A/B of library builds (in-tree default vs _native/var/<name>):
#   tools/gpu_ds_ab.sh <tag> <variant>...   (variant: main | name), interleaved twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = main ]; then L=raincast-gnn_amd/raincast_gnn/_native/libgine_hip.so; else L=raincast-gnn_amd/raincast_gnn/_native/var/$v/libgine_hip.so; fi
    echo "== $v rep $rep"
    GINE_HIP_LIB=$L timeout -k 10 120 python tools/ds_micro.py --nodes ${DS_NODES:-4000,16000,128000} || exit $?
  done
done 2>&1 | tee $O/ds_ab.txt
