#!/usr/bin/env bash
# r02_s57: the combined backward launch with only its engine half (MP role returns) and with
# an empty engine (GINE_WG_VARIANT=7: no MFMA, no loads, no slab stores) -- kernel table times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_s57; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for v in base nomp noeng; do
  L=""; [ $v = base ] || L="GINE_HIP_LIB=$V/$v/libgine_hip.so"
  env $L timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 20 > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?; [ $rc -le 1 ] || exit $rc
done
echo done
