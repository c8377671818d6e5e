# DeepSet kernels at cfg2's 16,000 nodes: launch times and block 0's per-tile phases
export TMPDIR=/tmp; O=gpurun_out/r06_s35; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
timeout -k 10 200 python tools/ds_micro.py --nodes 16000 --reps 50 2>&1 | grep -v amdgpu.ids || exit $?
GINE_HIP_LIB=$V/dsprof/libgine_hip.so timeout -k 10 200 python tools/ds_micro.py --nodes 16000 --prof 2>&1 | grep -v amdgpu.ids || exit $?
GINE_HIP_LIB=$V/dsprof/libgine_hip.so timeout -k 10 200 python tools/ds_micro.py --nodes 16000 --prof --bwd 2>&1 | grep -v amdgpu.ids || exit $?
