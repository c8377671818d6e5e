#!/usr/bin/env bash
# determinism of the column-major split engine in the combined launch (reference digests:
# dx=c080e6a8e730 lin.weight=31f17cf6aae7 from the fp32-engine build), then the GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s11}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 120 python tools/determinism_layer.py --flat 2>&1 | grep -v amdgpu.ids | cut -c1-140 | tee $O/layer_flat.txt; st ${PIPESTATUS[0]} layer
timeout -k 10 150 python tools/determinism.py > $O/det.txt 2>&1; st $? det
grep -c DIFF $O/det.txt; grep -v amdgpu $O/det.txt | head -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_deepset.py tests/test_gpu_training.py tests/test_gpu_chain.py tests/test_gpu_layer.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; st $rc tests
