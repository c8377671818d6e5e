#!/usr/bin/env bash
# A/B of environment switches on the cfg2 training step, alternated on one box:
#   tools/gpu_ab.sh <tag> "ENV=1 ENV2=0" "ENV=0" ...   (each variant run twice, interleaved)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python bench.py --no-cpu --no-strong --steps 100 ${BENCH_ARGS:-} > $O/v${i}_r$rep.json 2> $O/v${i}_r$rep.err
    rc=$?; [ $rc -le 1 ] || { echo "crash-class $rc ($v)"; exit $rc; }
    python - "$O/v${i}_r$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms  p50 {d['step_ms_p10_p50_p90'][1]:.4f}  {d['value']:.0f} graphs/s")
PY
  done
done | tee $O/ab.txt
