#!/usr/bin/env bash
# r02_s13: message-passing kernels under the locality (RCM) station order + per-config bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s13; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 300 python tools/mp_micro.py --configs 2,3,5 --tiles 128,64,32 > $O/mp_ds.jsonl 2> $O/mp_ds.err; st $?
timeout -k 10 300 python tools/mp_micro.py --configs 2,3,5 --tiles 128,64,32 --rcm > $O/mp_rcm.jsonl 2> $O/mp_rcm.err; st $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/sq1 -o run -- python3 tools/mp_micro.py --configs 2 --tiles 128 --rcm --eager --reps 5 > $O/sq1.log 2>&1; st $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/sq2 -o run -- python3 tools/mp_micro.py --configs 2 --tiles 128 --rcm --eager --reps 5 > $O/sq2.log 2>&1; st $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/l2 -o run -- python3 tools/mp_micro.py --configs 2 --tiles 128 --rcm --eager --reps 5 > $O/l2.log 2>&1; st $?
timeout -k 10 300 python bench.py --no-cpu --config 3 --steps 20 > $O/bench3.json 2> $O/bench3.err; st $?
timeout -k 10 300 python bench.py --no-cpu --config 5 --steps 20 > $O/bench5.json 2> $O/bench5.err; st $?
timeout -k 10 300 python bench.py --no-cpu --config 1 --steps 50 > $O/bench1.json 2> $O/bench1.err; st $?
echo done
