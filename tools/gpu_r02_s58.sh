#!/usr/bin/env bash
# r02_s58: slab reduction loads in flight (unroll 8 vs 4), A/B + gradient-batch kernel time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s58; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
bash tools/gpu_ab.sh r02_s58_ab "RAINCAST_X=0" "GINE_HIP_LIB=$V/u8/libgine_hip.so" || exit $?
for v in base u8; do
  L=""; [ $v = base ] || L="GINE_HIP_LIB=$V/$v/libgine_hip.so"
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --no-cpu --no-strong --steps 20 > $O/b_$v.json 2> $O/b_$v.err || exit $?
  grep -i "grad_batch" $O/prof_$v/run_kernel_stats.csv | cut -c1-200
done
