# kernel traces of the cfg2 step with the head folded and with its own launch
export TMPDIR=/tmp; O=gpurun_out/r06_s11; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fold -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-strong > $O/prof_fold.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nofold -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu --no-strong --no-head-fold > $O/prof_nofold.log 2>&1 || exit $?
for v in fold nofold; do
  f=$(ls $O/prof_$v/*/run_kernel_trace.csv 2>/dev/null || ls $O/prof_$v/run_kernel_trace.csv)
  python tools/step_breakdown.py $f --steps 20 > $O/step_$v.txt && head -12 $O/step_$v.txt
done
