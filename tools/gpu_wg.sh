#!/usr/bin/env bash
# Weight-gradient engine diagnostic variants on the GPU box (built there: tools/bin is not shipped)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-wg}; mkdir -p $O
bash tools/wg_variants.sh > $O/build.log 2>&1 || exit 1
for v in 0 1 2 3 4 16 18 8; do
  for n in 16000 128000; do
    timeout -k 5 60 tools/bin/wg_v$v $n >> $O/wg.log 2>&1 || { echo "rc $? v$v"; exit 1; }
  done
done
cat $O/wg.log
