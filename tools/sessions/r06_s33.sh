# closing measurements of the round-6 tree: GPU suite, smoke, bench (default and the driver's
# command), rocprof step trace, PMC traffic
export TMPDIR=/tmp
bash tools/gpu_session.sh r06_s33 tests smoke bench prof pmc || exit $?
O=gpurun_out/r06_s33
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || exit $?
python tools/step_breakdown.py $O/prof/run_kernel_trace.csv --steps 20 > $O/step_breakdown.txt
head -3 $O/step_breakdown.txt
python -c "
import json
for f in ('$O/bench.log', '$O/bench_driver_cmd.json'):
    d = json.loads([l for l in open(f) if l.startswith('{')][-1])
    print(f, d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'], d['roofline'].get('frac'), d['roofline'].get('traffic'), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)
"
