#!/usr/bin/env bash
# Hardware counters of the gather message-passing kernels (k_mp_fwd / k_mp_bwd) at a
# configuration (default cfg5, the bench's locality order), one rocprofv3 --pmc pass per
# counter group within the per-block limits (8 SQ, 4 TCP, 2 TA, 2 TD, 2 GRBM, 4 TCC); names
# missing from this device's `rocprofv3 -L` list are dropped before a pass runs.
#   tools/gpu_mp_counters.sh <tag> [config]
#   LAYER=1 FILTER=gine::k_mp_fwd_layer tools/gpu_mp_counters.sh <tag> 2   (the layer forward)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-mpctr}; CFG=${2:-5}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
have() {  # the names of "$@" this device lists
  python - "$O/counters_list.txt" "$@" <<'PY'
import re, sys
text = open(sys.argv[1]).read()
print(" ".join(n for n in sys.argv[2:] if re.search(r"\b" + re.escape(n) + r"\b", text)))
PY
}
pass_run() {  # pass_run <name> counters...
  local name=$1; shift
  local c; c=$(have "$@")
  [ -n "$c" ] || { echo "pass $name: no listed counters"; return 0; }
  echo "pass $name: $c"
  if [ "${LAYER:-0}" = 1 ]; then  # the one-launch layer forward (tools/layer_prof.py)
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/$name -o run -- \
      python3 tools/layer_prof.py --config $CFG --reps 5 --no-stamps > $O/$name.log 2>&1
  else
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/$name -o run -- \
      python3 tools/mp_micro.py --configs $CFG --tiles "" --rcm --eager --reps 5 > $O/$name.log 2>&1
  fi
  local rc=$?
  [ $rc -eq 0 ] || { echo "pass $name rc=$rc"; tail -3 $O/$name.log; exit $rc; }
}
pass_run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU
pass_run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_IFETCH
pass_run ta TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum
pass_run ta2 TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
pass_run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
pass_run tcp2 TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_GATE_EN1_sum TCP_GATE_EN2_sum
pass_run td TD_BUSY_avr TD_TC_STALL_sum
pass_run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
pass_run grbm GRBM_GUI_ACTIVE GRBM_COUNT
for f in $O/*/run_counter_collection.csv; do echo "$f"; done > $O/passes.txt
python tools/pmc_summary.py $O/*/run_counter_collection.csv --filter "${FILTER:-gine::k_mp_}" > $O/summary.txt 2>&1
cat $O/summary.txt
