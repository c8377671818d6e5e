# chain backward with the ReLU mask issued before the next tile's prefetch (shipped) against
# the mask behind it (variant); chain tests; step A/B
export TMPDIR=/tmp; O=gpurun_out/r06_s32; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $O/pytest_chain.log 2>&1; rc=$?; tail -2 $O/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep backward | sed 's/^/early /' || exit $?
GINE_HIP_LIB=$V/chainepl/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep backward | sed 's/^/late /' || exit $?
done
GINE_HIP_LIB=$V/chainprof/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py > $O/stamps.txt 2>&1 || exit $?
grep -A12 "^backward" $O/stamps.txt
