# DeepSet forward: mask words kept in LDS and stored per group (MDEF) vs per tile: kernel
# times x2 interleaved, the DeepSet / training / golden GPU tests, step A/B
export TMPDIR=/tmp; O=gpurun_out/r06_s43; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for r in 1 2; do
  echo "== defer"; timeout -k 10 200 python tools/ds_micro.py --nodes 4000,16000,32000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== per-tile"; GINE_HIP_LIB=$V/mdef0/libgine_hip.so timeout -k 10 200 python tools/ds_micro.py --nodes 4000,16000,32000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
done > $O/ds_ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -k "deepset or golden or parity or training or chain" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
STEPS=200 bash tools/gpu_lib_ab.sh r06_s43 2 main mdef0 || exit $?
