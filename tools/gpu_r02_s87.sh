#!/usr/bin/env bash
# r02_s87: HBM traffic per kernel launch (PMC FETCH_SIZE / WRITE_SIZE, separate passes) at
# cfg2, cfg3 and cfg5 for the bench's roofline "traffic" field.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s87; mkdir -p $O
for c in 2 3 5; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$c -o run -- python3 bench.py --config $c --steps 3 --warmup 2 --no-cpu --no-graph --no-strong --kernel-reps 3 > $O/fetch$c.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write$c -o run -- python3 bench.py --config $c --steps 3 --warmup 2 --no-cpu --no-graph --no-strong --kernel-reps 3 > $O/write$c.log 2>&1 || exit $?
  python tools/pmc_summary.py $O/fetch$c/run_counter_collection.csv $O/write$c/run_counter_collection.csv --config cfg$c --traffic-json $O/r02_s87_cfg${c}_pmc_traffic.json > $O/r02_s87_cfg${c}_pmc_summary.txt 2>&1 || exit $?
done
echo done
