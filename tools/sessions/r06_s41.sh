# DeepSet start-up loads behind the first tiles' loads (LATE) vs before the walk: kernel
# times (x2 interleaved), the DeepSet GPU tests, step A/B
export TMPDIR=/tmp; O=gpurun_out/r06_s41; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for r in 1 2; do
  echo "== late"; timeout -k 10 200 python tools/ds_micro.py --nodes 4000,16000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== before"; GINE_HIP_LIB=$V/prelate0/libgine_hip.so timeout -k 10 200 python tools/ds_micro.py --nodes 4000,16000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
done > $O/ds_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -q -rf -k "deepset or golden or parity" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
STEPS=200 bash tools/gpu_lib_ab.sh r06_s41 2 main prelate0 || exit $?
