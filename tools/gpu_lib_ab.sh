#!/usr/bin/env bash
# Step-time A/B of library builds (in-tree default vs _native/var/<name>/libgine_hip.so),
# interleaved on one box:  tools/gpu_lib_ab.sh <tag> <config> <variant>...  (variant: main | name)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; C=$2; shift 2; mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = main ]; then L=raincast-gnn_amd/raincast_gnn/_native/libgine_hip.so; else L=raincast-gnn_amd/raincast_gnn/_native/var/$v/libgine_hip.so; fi
    GINE_HIP_LIB=$L timeout -k 10 300 python bench.py --config $C --no-cpu --no-strong --steps ${STEPS:-50} --kernel-reps ${KREPS:-20} ${BENCH_ARGS:-} > $O/c${C}_${v}_$rep.json 2> $O/c${C}_${v}_$rep.err
    rc=$?; [ $rc -le 1 ] || { echo "crash-class $rc ($v)"; exit $rc; }
    python - "$O/c${C}_${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(f"{sys.argv[2]:14s} {d['config']['workload'][:6]} {d['ms_per_step']:.4f} ms  p50 {d['step_ms_p10_p50_p90'][1]:.4f}  {d['value']:.0f} graphs/s  "
      + "  ".join(f"{n} {k[n]['us']}" for n in ("gine_mp_bwd_mlp_wgrad", "gine_mp_fwd_layer", "gine_mp_fwd", "gine_mp_bwd") if n in k))
PY
  done
done | tee $O/ab_c$C.txt
