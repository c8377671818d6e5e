#!/usr/bin/env bash
# r02_s55: window backward block reduction with DPP / permlane swaps (no ds_bpermute)
# -- GPU suite, phase profile, A/B against the previous build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s55; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
GINE_HIP_LIB=$V/winprof/libgine_hip.so timeout -k 10 200 python tools/win_prof.py --config 2 > $O/winprof.txt 2>&1 || exit 1
cat $O/winprof.txt
bash tools/gpu_ab.sh r02_s55_ab "RAINCAST_X=new" "GINE_HIP_LIB=$V/prev/libgine_hip.so"
