# the gradient mean as one RCCL AVG collective: forced world-1 RCCL split / graph bits and
# times against the single-process step, the distributed GPU tests
export TMPDIR=/tmp; O=gpurun_out/r06_s26; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > $O/pytest_train.log 2>&1; rc=$?; tail -2 $O/pytest_train.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_dist_check.sh r06_s26/dist
