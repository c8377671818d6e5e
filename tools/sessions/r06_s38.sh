# gradient batch: slab workgroup shape by chunk count (job times, tests touching slab sums, bench)
export TMPDIR=/tmp; O=gpurun_out/r06_s38; mkdir -p $O
timeout -k 10 200 python tools/gradbatch_jobs.py > $O/jobs.txt 2>&1 || exit $?
KTESTS="grad or slab or wgrad or head or deepset or linear or chain or mlp" bash tools/gpu_session.sh r06_s38 ktests benchnc || exit $?
