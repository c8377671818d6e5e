#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s16; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; st $?
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD" \
           "SQ_INST_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  n=$(echo $set | tr ' ' '\n' | head -1)
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$n -o run -- python3 tools/mp_micro.py --configs 3 --tiles 128 --rcm --eager --reps 3 > $O/pmc_$n.log 2>&1; st $?
done
echo ok
