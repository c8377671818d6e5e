#!/usr/bin/env bash
# split engine: determinism (default = one workgroup per CU; e1 = 128-register cap with one
# workgroup per CU forced by LDS), the GPU tests, step A/B against the fp32-engine build,
# kernel traces of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s12}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
V=raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 120 python tools/determinism_layer.py --flat 2>&1 | grep -v amdgpu.ids | cut -c1-100 | tee $O/layer_flat.txt; st ${PIPESTATUS[0]} layer
GINE_HIP_LIB=$V/e1/libgine_hip.so timeout -k 10 120 python tools/determinism_layer.py --flat 2>&1 | grep -v amdgpu.ids | cut -c1-100 | tee $O/layer_flat_e1.txt; st ${PIPESTATUS[0]} layer_e1
timeout -k 10 150 python tools/determinism.py > $O/det.txt 2>&1; st $? det
echo "DIFF lines: $(grep -c DIFF $O/det.txt)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_deepset.py tests/test_gpu_training.py tests/test_gpu_chain.py tests/test_gpu_layer.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; st $rc tests
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in x3 wgf32; do
    if [ $v != x3 ]; then export GINE_HIP_LIB=$V/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 50 > $O/b.json 2>$O/b.err || { echo "bench failed: $v"; tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['step_ms_p10_p50_p90'], d['roofline']['avg_us'])" | tee -a $O/ab.txt
  done
done
unset GINE_HIP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
export GINE_HIP_LIB=$V/wgf32/libgine_hip.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f32 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong > $O/prof_f32.log 2>&1 || { echo "rocprof f32 failed"; exit 1; }
python tools/step_breakdown.py $O/prof_f32/run_kernel_trace.csv > $O/step_breakdown_f32.txt 2>&1
head -12 $O/step_breakdown_f32.txt
