# A/B on one box: the output head folded into the last layer's launch vs its own launch
export TMPDIR=/tmp; O=gpurun_out/r06_s10; mkdir -p $O
for i in 1 2 3; do
for f in "" "--no-head-fold"; do
timeout -k 10 200 python bench.py --no-cpu --no-strong $f > $O/bench_$i$f.json 2> $O/bench.err || exit $?
python -c "
import json; d=json.loads(open('$O/bench_$i$f.json').read().strip().splitlines()[-1])
print('$f' or 'fold', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])
"
done
done
