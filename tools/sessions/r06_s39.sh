# gradient batch: jobs ordered longest first; + slab unroll 16 variant
export TMPDIR=/tmp; O=gpurun_out/r06_s39; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 200 python tools/gradbatch_jobs.py > $O/jobs_ordered.txt 2>&1 || exit $?
GINE_HIP_LIB=$V/su16/libgine_hip.so timeout -k 10 200 python tools/gradbatch_jobs.py > $O/jobs_ordered_unroll16.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench.json 2>&1 || exit $?
GINE_HIP_LIB=$V/su16/libgine_hip.so timeout -k 10 200 python bench.py --no-cpu --no-strong > $O/bench_unroll16.json 2>&1 || exit $?
