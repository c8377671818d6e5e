# DeepSet forward diagnostic builds: which part of the per-tile time is on the critical path
export TMPDIR=/tmp; O=gpurun_out/r06_s42; mkdir -p $O
V=$PWD/raincast-gnn_amd/raincast_gnn/_native/var
for r in 1 2; do
  for v in main dsdiag1 dsdiag2 dsdiag3 dsdiag4 dsdiag8; do
    if [ $v = main ]; then L=$PWD/raincast-gnn_amd/raincast_gnn/_native/libgine_hip.so; else L=$V/$v/libgine_hip.so; fi
    echo "== $v"; GINE_HIP_LIB=$L timeout -k 10 200 python tools/ds_micro.py --nodes 16000 --reps 100 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/diag.txt 2>&1
