#!/usr/bin/env bash
# Register / LDS / occupancy summary of the kernels in one HIP source (device compile only):
#   tools/kres.sh gine_deepset.hip [grep-pattern] [extra hipcc flags...]
set -eu
SRC=$1; PAT=${2:-.}; shift; [ $# -gt 0 ] && shift
CS=$(cd "$(dirname "$0")/../raincast-gnn_amd/csrc" && pwd)
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I"$CS/../../include" \
  -I"$CS" --cuda-device-only -c "$CS/$SRC" -o /tmp/kres_dev.o "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys, subprocess
pat = re.compile(sys.argv[1])
cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+([A-Za-z ]+?): (\S+)", line)
    if m and cur: rows[cur][m.group(1).strip()] = m.group(2)
names = list(rows)
dem = subprocess.run(["c++filt"], input="\n".join(names),
                     capture_output=True, text=True).stdout.splitlines()
for n, d in zip(names, dem):
    if not pat.search(d): continue
    g = rows[n].get
    print("%-90s v%s a%s spill%s/%s lds%s occ%s" % (d[:90], g("VGPRs"), g("AGPRs"), g("VGPRs Spill"),
          g("ScratchSize [bytes/lane]"), g("LDS Size [bytes/block]"), g("Occupancy [waves/SIMD]")))
' "$PAT"
