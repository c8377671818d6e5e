# confirmation of the final tree's rebuilt library (same source hash as r06_s33): GPU suite,
# smoke, bench with the driver's command
export TMPDIR=/tmp
bash tools/gpu_session.sh r06_s44 tests smoke bench || exit $?
O=gpurun_out/r06_s44
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit $?
