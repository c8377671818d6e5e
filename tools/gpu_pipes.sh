#!/usr/bin/env bash
# Per-kernel pipe utilisation of the training step (eager launches, 2 PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pipes}; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
A="SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
C="GRBM_GUI_ACTIVE SQ_CYCLES TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
for P in A B; do
  timeout -s KILL 120 rocprofv3 --pmc ${!P} --output-format csv -d $O/pmc_$P -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu --no-graph --kernel-reps 3 --no-strong > $O/pmc_$P.log 2>&1; st $?
done
echo ok
