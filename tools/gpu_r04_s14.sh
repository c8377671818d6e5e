#!/usr/bin/env bash
# DeepSet kernels: timings at two sizes and the phase stamps of the forward and backward
# (workgroup 0, tools/ds_micro.py --prof on the GINE_DS_PROFILE build); then the default step
# once more (bench + kernel trace) on the combined-kernel-fp32 / split-elsewhere build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s14}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
timeout -k 10 120 python tools/ds_micro.py --nodes 4000,16000 > $O/ds_micro.txt 2>&1; st $? ds_micro
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsprof/libgine_hip.so timeout -k 10 120 python tools/ds_micro.py --nodes 16000 --prof > $O/ds_prof_fwd.txt 2>&1; st $? ds_prof
GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/dsprof/libgine_hip.so timeout -k 10 120 python tools/ds_micro.py --nodes 16000 --prof --bwd > $O/ds_prof_bwd.txt 2>&1; st $? ds_prof_bwd
grep -v amdgpu.ids $O/ds_micro.txt $O/ds_prof_fwd.txt $O/ds_prof_bwd.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 50 > $O/b.json 2>$O/b.err || { echo "bench failed"; tail -5 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['step_ms_p10_p50_p90'], d['roofline']['avg_us'])" | tee -a $O/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
