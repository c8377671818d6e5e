# the gap between graph replays: host replay-call time vs GPU time; HIP runtime graph switches
export TMPDIR=/tmp; O=gpurun_out/r06_s46; mkdir -p $O
for v in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"; do
  echo "== [$v]"
  env $v timeout -k 10 200 python tools/replay_gap.py 2>&1 | grep -v amdgpu.ids || exit 1
done > $O/replay_gap.txt 2>&1
