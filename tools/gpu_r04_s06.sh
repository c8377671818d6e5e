#!/usr/bin/env bash
# Round-4 session 6: the split-bf16 weight-gradient engine and DeepSet forward -- the rest of the GPU suite from
# test_gpu_layer on, then step A/B against the fp32-engine / fp32-DeepSet builds and a kernel trace.
#   tools/gpu_r04_s06.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04_s06}
O=gpurun_out/$TAG; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_deepset.py tests/test_gpu_training.py tests/test_gpu_chain.py tests/test_gpu_layer.py tests/test_gpu_train.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; st $rc tests
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/ds_micro.py --nodes 4000,16000 > $O/ds_micro_x3.txt 2>&1; st $? ds_micro
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsf32/libgine_hip.so timeout -k 10 120 python tools/ds_micro.py --nodes 4000,16000 > $O/ds_micro_f32.txt 2>&1; st $? ds_micro_f32
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsprof/libgine_hip.so timeout -k 10 120 python tools/ds_micro.py --nodes 16000 --prof > $O/ds_prof_fwd.txt 2>&1; st $? ds_prof
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsprof/libgine_hip.so timeout -k 10 120 python tools/ds_micro.py --nodes 16000 --prof --bwd > $O/ds_prof_bwd.txt 2>&1; st $? ds_prof_bwd
grep -v amdgpu.ids $O/ds_micro_x3.txt $O/ds_micro_f32.txt $O/ds_prof_fwd.txt $O/ds_prof_bwd.txt
GINE_PARITY_REPORT=$O timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest_cfg.log 2>&1; rc=$?; tail -2 $O/pytest_cfg.log; st $rc configs
for rep in 1 2; do
  for v in x3 wgf32 dsf32; do
    if [ $v != x3 ]; then export GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 50 > $O/b.json 2>$O/b.err || { echo "bench failed: $v"; tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['step_ms_p10_p50_p90'], d['roofline']['avg_us'])" | tee -a $O/ab.txt
  done
  unset GINE_HIP_LIB
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
