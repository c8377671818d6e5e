#!/usr/bin/env bash
# Round-4 working session on one box: the layer-kernel tests, the layer A/B with a kernel
# trace, the drop-in host profile and the gather-kernel counters at cfg5.  Every GPU step
# has its own time limit; a crash-class exit stops the session.
#   tools/gpu_r04_batch.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04_batch}
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_bnacc.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > $O/pytest_layer.log 2>&1; rc=$?; tail -2 $O/pytest_layer.log; st $rc tests
[ $rc -eq 0 ] || exit 1
bash tools/gpu_layer_ab.sh $TAG/ab || exit 1
timeout -k 10 200 python tools/dropin_prof.py > $O/dropin_prof.txt 2>&1; st $? dropin
timeout -k 10 200 python tools/dropin_prof.py --same-edges > $O/dropin_prof_same.txt 2>&1; st $? dropin_same
head -1 $O/dropin_prof.txt; head -1 $O/dropin_prof_same.txt
bash tools/gpu_mp_counters.sh $TAG/mpctr5 5 > $O/mpctr5.log 2>&1; st $? counters
tail -12 $O/mpctr5.log
