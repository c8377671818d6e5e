#!/usr/bin/env bash
# window tile size (options.WINDOW_NODES) at cfg2 / cfg3 and the window plans everywhere
# (options.MP_WINDOW = "all") at cfg5: step A/Bs, each variant twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_s22}; mkdir -p $O
ab() {  # ab <cfg> <variant...>
  local cfg=$1; shift
  for rep in 1 2; do
    for v in "$@"; do
      timeout -k 10 200 python tools/bench_with.py $v -- --config $cfg --no-cpu --no-strong --steps 30 > $O/b.json 2>$O/b.err || { echo "bench failed: $cfg $v"; tail -5 $O/b.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('cfg$cfg', '$v', d['ms_per_step'], d['step_ms_p10_p50_p90'])" | tee -a $O/ab.txt
    done
  done
}

ab 3 WINDOW_NODES=128 WINDOW_NODES=64
ab 5 MP_WINDOW=auto MP_WINDOW=all
