#!/usr/bin/env bash
# A/B of message-passing kernel builds (tools/mp_micro.py, gather kernels, engine order):
#   tools/gpu_mp_ab.sh <tag> <variant>...   (variant: main or _native/var/<name>)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
for v in "$@"; do
  if [ $v = main ]; then L=raincast-gnn_amd/raincast_gnn/_native/libgine_hip.so; else L=raincast-gnn_amd/raincast_gnn/_native/var/$v/libgine_hip.so; fi
  for D in ${DS:-128}; do
    GINE_HIP_LIB=$L timeout -k 10 200 python tools/mp_micro.py --configs ${CFGS:-2,3,5} --tiles "" --rcm --D $D > $O/mp_${v}_D$D.jsonl 2> $O/mp_${v}_D$D.err || exit $?
  done
done
for f in $O/mp_*.jsonl; do echo $f; cat $f; done
