export TMPDIR=/tmp; O=gpurun_out/r06_s18; mkdir -p $O
timeout -k 10 120 python tools/clock_ramp.py --seconds 2 > $O/ramp.txt 2>&1 || exit $?
timeout -k 10 120 python tools/clock_ramp.py --seconds 1 --idle-ms 2000 > $O/ramp_idle2s.txt 2>&1 || exit $?
cat $O/ramp.txt; tail -25 $O/ramp_idle2s.txt
