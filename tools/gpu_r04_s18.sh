#!/usr/bin/env bash
# cfg3 / cfg5: the doubly folded one-launch chain (DeepSet-launch fold) above 32,768 nodes
# against the two-launch singly folded chain (chain.F3_MAX_NODES).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s18}; mkdir -p $O
for cfg in 3 5; do
  for rep in 1 2; do
    for v in "chain.F3_MAX_NODES=32768" "chain.F3_MAX_NODES=1000000000"; do
      timeout -k 10 200 python tools/bench_with.py $v -- --config $cfg --no-cpu --no-strong --steps 20 > $O/b.json 2>$O/b.err || { echo "bench failed: $cfg $v"; tail -5 $O/b.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('cfg$cfg', '$v', d['ms_per_step'], d['step_ms_p10_p50_p90'])" | tee -a $O/ab.txt
    done
  done
done
