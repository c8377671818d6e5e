# kernel traces of the cfg2 step with the head folded and with its own launch
export TMPDIR=/tmp; O=gpurun_out/r06_s16; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fold -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-strong > $O/prof_fold.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nofold -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-strong --no-head-fold > $O/prof_nofold.log 2>&1 || exit $?
for v in fold nofold; do
  f=$(ls $O/prof_$v/*/run_kernel_trace.csv 2>/dev/null || ls $O/prof_$v/run_kernel_trace.csv)
  python tools/step_breakdown.py $f --steps 20 > $O/step_$v.txt && head -12 $O/step_$v.txt
done
python - <<'PY'
import csv,re
for v in ("fold","nofold"):
    rows=list(csv.DictReader(open(f"gpurun_out/r06_s16/prof_{v}/run_kernel_trace.csv")))
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    idx=[i for i,r in enumerate(rows) if 'k_adamw' in r['Kernel_Name']]
    print("==", v)
    for a,b in zip(idx[-4:-1], idx[-3:]):
        ks=[(re.search(r'k_\w+', r['Kernel_Name']).group(0), (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000) for r in rows[a+1:b+1]]
        print(" ".join(f"{n[2:10]}:{d:.1f}" for n,d in ks), f"sum {sum(d for _,d in ks):.1f}")
PY
