# settle length: the driver's 20-step line after 100 / 400 settle replays against a long run
export TMPDIR=/tmp; O=gpurun_out/r06_s20; mkdir -p $O
for i in 1 2; do
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --settle-steps 400" "--steps 400 --warmup 100"; do
t=$(echo "x$a" | tr -d ' -')
timeout -k 10 300 python3 bench.py --no-cpu --no-strong $a > $O/bench_$i$t.json 2> $O/bench.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_$i$t.json').read().strip().splitlines()[-1])
print('$a', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'], d.get('settle_steps'))
"
done
done
