# CRPS + head-backward pass with 32 nodes per workgroup (500 workgroups at cfg2) vs 64:
# pass times x2 interleaved, the loss / head / training GPU tests on the variant, step A/B
export TMPDIR=/tmp; O=gpurun_out/r06_s45; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for r in 1 2; do
  echo "== 64"; timeout -k 10 200 python tools/crps_micro.py --head --nodes 1000,4000,16000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== 32"; GINE_HIP_LIB=$V/hn32/libgine_hip.so timeout -k 10 200 python tools/crps_micro.py --head --nodes 1000,4000,16000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
done > $O/crps_ab.txt 2>&1 || exit 1
GINE_HIP_LIB=$V/hn32/libgine_hip.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -k "crps or head or loss or training or golden" --timeout 120 --timeout-method thread > $O/pytest_hn32.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
STEPS=200 bash tools/gpu_lib_ab.sh r06_s45 2 main hn32 || exit $?
