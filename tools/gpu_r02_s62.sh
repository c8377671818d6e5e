#!/usr/bin/env bash
# r02_s62: double-buffered staging in the standalone weight-gradient engine -- GPU suite,
# A/B against GINE_WG_DB=0, cfg3/cfg5 benches both ways
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s62; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r02_s62_ab "RAINCAST_X=0" "GINE_HIP_LIB=$V/nodb/libgine_hip.so" || exit $?
for c in 3 5; do
  timeout -k 10 300 python bench.py --no-cpu --no-strong --config $c --steps 20 > $O/b${c}_db.json 2>/dev/null || exit $?
  GINE_HIP_LIB=$V/nodb/libgine_hip.so timeout -k 10 300 python bench.py --no-cpu --no-strong --config $c --steps 20 > $O/b${c}_nodb.json 2>/dev/null || exit $?
  python -c "
import json
for v in ('db','nodb'):
    d=json.loads(open('$O/b${c}_'+v+'.json').read().strip().splitlines()[-1]); print('cfg$c', v, d['ms_per_step'])"
done
