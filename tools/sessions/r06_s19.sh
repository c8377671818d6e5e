# the driver's command with the clock settle (default) and without it, interleaved
export TMPDIR=/tmp; O=gpurun_out/r06_s19; mkdir -p $O
for i in 1 2; do
for a in "" "--settle-steps 0"; do
t=$(echo "x$a" | tr -d ' -')
s0=$(date +%s.%N)
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $a > $O/bench_$i$t.json 2> $O/bench.err || exit $?
s1=$(date +%s.%N)
python -c "
import json; d=json.loads(open('$O/bench_$i$t.json').read().strip().splitlines()[-1])
print('${a:-settle 100}', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'], d.get('settle_steps'), 'run_s', round($s1-$s0,1), 'cpu', d['cpu_baseline']['value'])
"
done
done
