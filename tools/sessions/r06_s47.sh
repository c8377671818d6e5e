# S training steps per captured graph (1, 2, 4, 1): per-step GPU time and the final loss
export TMPDIR=/tmp; O=gpurun_out/r06_s47; mkdir -p $O
timeout -k 10 400 python tools/multistep_graph.py > $O/multistep.txt 2>&1
