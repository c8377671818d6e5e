# split-bf16 doubly folded chain (k_chain2_x3): parity tests, then interleaved step A/B against
# the fp32-MFMA chain (variant library), then kernel traces of both
export TMPDIR=/tmp; O=gpurun_out/r06_s21; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_training.py tests/test_gpu_head_fold.py -x -q --timeout 200 --timeout-method thread > $O/pytest_chain.log 2>&1; rc=$?; tail -4 $O/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for lib in x3 fp32; do
  if [ $lib = fp32 ]; then export GINE_HIP_LIB=$V/chainfp32/libgine_hip.so; else unset GINE_HIP_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench_$i$lib.json 2> $O/bench.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$i$lib.json').read().strip().splitlines()[-1])
print('$lib', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])
"
done
done
unset GINE_HIP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_x3 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-strong > $O/prof_x3.log 2>&1 || exit $?
python tools/step_breakdown.py $O/prof_x3/run_kernel_trace.csv --steps 20 > $O/step_x3.txt && cat $O/step_x3.txt | head -24
