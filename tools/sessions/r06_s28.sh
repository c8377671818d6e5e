# chain kernels, fp32 chains against split-bf16 chains with the weights split in the loop:
# launch times and phase stamps at cfg2's shape
export TMPDIR=/tmp; O=gpurun_out/r06_s28; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for i in 1 2; do
timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/fp32 /' || exit $?
GINE_HIP_LIB=$V/chainx3/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py --no-stamps 2>&1 | grep -v amdgpu.ids | sed 's/^/x3 /' || exit $?
done
GINE_HIP_LIB=$V/chainx3prof/libgine_hip.so timeout -k 10 200 python tools/chain_prof.py > $O/stamps_x3.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/stamps_x3.txt
