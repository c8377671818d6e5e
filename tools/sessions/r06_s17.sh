# the driver's short run (20 steps, 5 warmup) against a long one on the same box, interleaved
export TMPDIR=/tmp; O=gpurun_out/r06_s17; mkdir -p $O
for i in 1 2; do
for a in "--steps 20 --warmup 5" "--steps 400 --warmup 100"; do
t=$(echo $a | tr -d ' -')
timeout -k 10 200 python bench.py --no-cpu --no-strong $a > $O/bench_$i$t.json 2> $O/bench.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_$i$t.json').read().strip().splitlines()[-1])
print('$a', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])
"
done
done
