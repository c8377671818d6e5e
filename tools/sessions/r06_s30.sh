# chain kernels after the pre-loop wait fix (fp32 chains, the shipped library) against the
# library before it and the split-bf16 chains with the same fix; stamps of the fixed fp32 form
export TMPDIR=/tmp; O=gpurun_out/r06_s30; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for i in 1 2; do
timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/fixed /' || exit $?
GINE_HIP_LIB=$V/chainold/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/old /' || exit $?
GINE_HIP_LIB=$V/chainx3/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/x3fixed /' || exit $?
done
GINE_HIP_LIB=$V/chainprof/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py > $O/stamps_fixed.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/stamps_fixed.txt
