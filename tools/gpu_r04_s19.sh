#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s19}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_configs.py tests/test_gpu_training.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; st $rc tests
[ $rc -eq 0 ] || exit 1
for cfg in 3 5; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 > $O/bench_cfg$cfg.json 2> $O/bench_cfg$cfg.err; st $? bench$cfg
  python -c "import json;d=json.loads(open('$O/bench_cfg$cfg.json').read().strip().splitlines()[-1]);print('cfg$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}) and d['cpu_baseline'].get('value'))"
done
