export TMPDIR=/tmp; O=gpurun_out/r06_s09; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_head_fold.py tests/test_gpu_head.py tests/test_gpu_layer.py tests/test_gpu_layer_win.py -x -q --timeout 120 --timeout-method thread > $O/pytest_fold.log 2>&1; rc=$?; tail -5 $O/pytest_fold.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench2_$i.json 2> $O/bench2.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench2_$i.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'], d.get('step_trace'))
"
done
