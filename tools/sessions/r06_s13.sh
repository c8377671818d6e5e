# folded head: parity tests, launch time / phase stamps with and without it, step A/B
export TMPDIR=/tmp; O=gpurun_out/r06_s13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_head_fold.py tests/test_gpu_layer.py tests/test_gpu_layer_win.py -x -q --timeout 120 --timeout-method thread > $O/pytest_fold.log 2>&1; rc=$?; tail -3 $O/pytest_fold.log; [ $rc -eq 0 ] || exit $rc
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for h in "" "--head 2"; do
  echo "== head: ${h:-none}"
  timeout -k 10 200 python tools/layer_prof.py --config 2 --no-win --no-stamps $h > "$O/time_${h// /}.txt" 2>&1 || exit $?
  tail -1 "$O/time_${h// /}.txt"
  GINE_HIP_LIB=$V/layerprof/libgine_hip.so timeout -k 10 200 python tools/layer_prof.py --config 2 --no-win $h > "$O/stamps_${h// /}.txt" 2>&1 || exit $?
  sed -n '/span entry/,/Linear2 chains/p' "$O/stamps_${h// /}.txt"
done
for i in 1 2; do
for f in "" "--no-head-fold"; do
timeout -k 10 200 python bench.py --no-cpu --no-strong $f > $O/bench_$i$f.json 2> $O/bench.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_$i$f.json').read().strip().splitlines()[-1])
print('$f' or 'fold', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])
"
done
done
