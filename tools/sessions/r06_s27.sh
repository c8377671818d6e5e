# chain kernels: launch times and phase stamps at cfg2's shape
export TMPDIR=/tmp; O=gpurun_out/r06_s27; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 200 python tools/chain_prof.py --no-stamps > $O/times.txt 2>&1 || exit $?
cat $O/times.txt | grep -v amdgpu.ids
GINE_HIP_LIB=$V/chainprof/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt | grep -v amdgpu.ids
