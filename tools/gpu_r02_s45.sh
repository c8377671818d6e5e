#!/usr/bin/env bash
# r02_s45: what the weight-gradient engine contends on inside the combined backward --
# engine diagnostic variants (no MFMA chain / zero operand loads / no slab stores), per-kernel
# standalone times from bench.py's kernel table (results are not meaningful, only times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s45; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 20 > $O/bench_base.json 2> $O/bench_base.err || exit $?
for v in 1 2 4; do
  GINE_HIP_LIB=$V/wg$v/libgine_hip.so timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 20 > $O/bench_wg$v.json 2> $O/bench_wg$v.err
  rc=$?; [ $rc -le 1 ] || exit $rc
done
echo done
