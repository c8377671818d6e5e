#!/usr/bin/env bash
# DeepSet: split vs fp32 chains, 16- vs 8-node groups at 16,000 nodes (HIP events), then the
# step with 8-node groups against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s15}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc in $2"; exit $rc; }; }
V=raincast-gnn_amd/raincast_gnn/_native/var
for v in x3 g8 dsf32 dsf32g8; do
  if [ $v != x3 ]; then export GINE_HIP_LIB=$V/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
  echo "--- $v"; timeout -k 10 120 python tools/ds_micro.py --nodes 4000,16000,32000 2>&1 | grep -v amdgpu.ids | tee $O/ds_$v.txt; st ${PIPESTATUS[0]} $v
done
for rep in 1 2; do
  for v in x3 g8; do
    if [ $v != x3 ]; then export GINE_HIP_LIB=$V/$v/libgine_hip.so; else unset GINE_HIP_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu --no-strong --steps 50 > $O/b.json 2>$O/b.err || { echo "bench failed: $v"; tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$v', d['ms_per_step'], d['step_ms_p10_p50_p90'])" | tee -a $O/ab.txt
  done
done
unset GINE_HIP_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dropin.log 2>&1; rc=$?; tail -2 $O/pytest_dropin.log; st $rc dropin_tests
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/dropin_prof.py > $O/dropin_prof.txt 2>&1; st $? dropin_prof
head -2 $O/dropin_prof.txt
timeout -k 10 300 python bench.py --dropin --steps 30 --warmup 5 > $O/bench_dropin.json 2> $O/bench_dropin.err; st $? bench_dropin
python -c "import json;d=json.loads(open('$O/bench_dropin.json').read().strip().splitlines()[-1]);print('dropin', d['value'], d['ms_per_step'], d['gine_stack_ms_fwd_bwd'])"
