# DeepSet: the split chain at 8-node groups (A/B at 8,000 / 16,000 / 32,000 nodes)
export TMPDIR=/tmp; O=gpurun_out/r06_s36; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for v in base g8 g8x3 base; do
  if [ $v = base ]; then L=; else L=$V/$v/libgine_hip.so; fi
  echo "== $v"
  GINE_HIP_LIB=$L timeout -k 10 200 python tools/ds_micro.py --nodes 8000,16000,32000 --reps 100 2>&1 | grep -v amdgpu.ids || exit $?
done 2>&1 | tee $O/ab.txt
