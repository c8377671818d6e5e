set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_s11; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-strong > $O/bench_loc.json 2> $O/bench_loc.err && \
timeout -k 10 300 python bench.py --no-cpu --no-strong --station-order dataset > $O/bench_ds.json 2> $O/bench_ds.err && \
timeout -k 10 300 python bench.py --no-cpu --no-strong > $O/bench_loc2.json 2> $O/bench_loc2.err && \
timeout -k 10 300 python bench.py --no-cpu --config 3 --steps 20 > $O/bench3_loc.json 2> $O/bench3_loc.err && \
timeout -k 10 300 python bench.py --no-cpu --config 3 --steps 20 --station-order dataset > $O/bench3_ds.json 2> $O/bench3_ds.err && \
timeout -k 10 300 python bench.py --no-cpu --config 5 --steps 20 > $O/bench5_loc.json 2> $O/bench5_loc.err && \
timeout -k 10 300 python bench.py --no-cpu --config 5 --steps 20 --station-order dataset > $O/bench5_ds.json 2> $O/bench5_ds.err
rc=$?; echo "bench rc=$rc"; exit $rc
