#!/usr/bin/env bash
# Round-4 session 3: the layer-kernel backward timing (with phase stamps), the C++ binding
# bit-equality test, the drop-in host profile and the drop-in bench line.
#   tools/gpu_r04_s03.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04_s03}
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 120 python tools/layer_prof.py > $O/layer_prof.txt 2>&1; st $? layer_prof
tail -20 $O/layer_prof.txt
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/rgprof/libgine_hip.so \
  timeout -k 10 120 python tools/layer_prof.py --stamps > $O/layer_stamps.txt 2>&1; st $? stamps
tail -30 $O/layer_stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dropin.log 2>&1; rc=$?; tail -3 $O/pytest_dropin.log; st $rc dropin_tests
timeout -k 10 200 python tools/dropin_prof.py > $O/dropin_prof.txt 2>&1; st $? dropin_prof
head -2 $O/dropin_prof.txt
timeout -k 10 300 python bench.py --dropin --steps 30 --warmup 5 > $O/bench_dropin.json 2> $O/bench_dropin.err; st $? bench_dropin
cat $O/bench_dropin.json
