# chain forward with W'^T staged through LDS (shipped library) against the library before it
export TMPDIR=/tmp; O=gpurun_out/r06_s31; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for i in 1 2 3; do
timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/wlds /' || exit $?
GINE_HIP_LIB=$V/chainold/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/old /' || exit $?
done
GINE_HIP_LIB=$V/chainprof/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py > $O/stamps_wlds.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/stamps_wlds.txt | head -14
