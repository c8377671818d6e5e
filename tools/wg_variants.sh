#!/usr/bin/env bash
# Build the weight-gradient engine microbenchmark in its diagnostic variants (CPU side).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
for v in 0 1 2 3 4 16 18 8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
    -I raincast-gnn_amd/csrc -DGINE_WG_VARIANT=$v tools/wg_micro.hip -o tools/bin/wg_v$v &
done
wait
