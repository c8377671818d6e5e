#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s25; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bnacc.py tests/test_gpu_configs.py -q -x -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; st $rc
bash tools/gpu_ab.sh r02_s25_ab "PIPE=1" "GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/nopipe/libgine_hip.so"
