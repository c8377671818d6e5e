export TMPDIR=/tmp; O=gpurun_out/r06_s08; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer_win.py tests/test_gpu_layer.py tests/test_gpu_golden.py tests/test_gpu_fuzz.py -q --timeout 120 --timeout-method thread > $O/pytest_layer.log 2>&1; rc=$?; tail -3 $O/pytest_layer.log; [ $rc -le 1 ] || exit $rc
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
GINE_HIP_LIB=$V/layerprof/libgine_hip.so timeout -k 10 200 python tools/layer_prof.py --config 2 --no-win > $O/stamps_l2.txt 2>&1 || exit $?
sed -n '/matrix role/,$p' $O/stamps_l2.txt
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench2_$i.json 2> $O/bench2.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench2_$i.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'], {k: v['us'] for k,v in d['kernels'].items() if v.get('in_step')})
"
done
