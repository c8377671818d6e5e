# full-size oracle parity at cfg3 (64 x 2,000 stations) in the locality order
export TMPDIR=/tmp; O=gpurun_out/r06_s23; mkdir -p $O
GINE_FULL_PARITY=1 GINE_PARITY_REPORT=$O/parity timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -k "full_config and cfg3" -x -v -s --timeout 1800 --timeout-method thread > $O/pytest_full_cfg3.log 2>&1; rc=$?; tail -6 $O/pytest_full_cfg3.log; exit $rc
