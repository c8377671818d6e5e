export TMPDIR=/tmp; O=gpurun_out/r06_s05; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer_win.py tests/test_gpu_layer.py tests/test_gpu_golden.py tests/test_gpu_layer_bwd.py tests/test_gpu_dropin.py -q --timeout 120 --timeout-method thread > $O/pytest_layer.log 2>&1; rc=$?; tail -5 $O/pytest_layer.log; [ $rc -le 1 ] || exit $rc
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for lib in layerprof layerprof_nogather; do
  GINE_HIP_LIB=$V/$lib/libgine_hip.so timeout -k 10 200 python tools/layer_prof.py --config 2 > $O/stamps_$lib.txt 2>&1 || exit $?
  echo "== $lib"; sed -n '/phase A detail/,$p' $O/stamps_$lib.txt
done
GINE_HIP_LIB=$V/layerprof/libgine_hip.so timeout -k 10 200 python tools/layer_prof.py --config 2 --no-win > $O/stamps_l2.txt 2>&1 || exit $?
echo "== l2"; sed -n '/phase A detail/,$p' $O/stamps_l2.txt
timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench2.json 2> $O/bench2.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])
for k,v in d['kernels'].items():
    if v.get('in_step'): print(k, v['us'])
"
