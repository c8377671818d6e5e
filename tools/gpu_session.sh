#!/usr/bin/env bash
# One GPU session on the gpurun box: each GPU step has its own time limit; a crash-class exit
# (fault/abort/segv/timeout) ends the session, ordinary test failures do not.
#   tools/gpu_session.sh <tag> [steps...]   steps: tests smoke bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS=${*:-tests smoke bench prof}

run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log" | tee -a "$OUT/session.log"
  case $rc in
    0|1) return 0 ;;   # pass / test failures: keep going
    *) echo "crash-class exit $rc: stopping session" | tee -a "$OUT/session.log"; exit $rc ;;
  esac
}

for s in $STEPS; do
  case $s in
    tests) GINE_PARITY_REPORT=$OUT/parity run pytest_gpu 660 python -u -m pytest tests -m gpu -q -rf --durations=15 --timeout 200 --timeout-method thread ;;
    det)   run determinism_layer 200 python tools/determinism_layer.py --flat ;;
    copy)  run copy_probe 200 python tools/copy_probe.py ;;
    ntests) run pytest_new 300 python -u -m pytest ${NTESTS:-tests/test_gpu_dropin.py} -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    btests) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/bounds/libgine_hip.so \
            run pytest_bounds 300 python -u -m pytest tests/test_gpu_bnacc.py tests/test_gpu_deepset.py -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    ktests) run pytest_k 600 python -u -m pytest tests -m gpu -q -rf -k "${KTESTS:-window}" --timeout 120 --timeout-method thread ;;
    layerprof) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/layerprof/libgine_hip.so \
            run layer_prof 200 python tools/layer_prof.py --config ${LPCFG:-2} ;;
    lbprof) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/layerbwdprof/libgine_hip.so \
            run layer_bwd_prof 200 python tools/layer_bwd_prof.py ;;
    chain) run chain_micro 200 python tools/chain_micro.py ;;
    dsab)  run ds_ab 900 bash tools/gpu_ds_ab.sh $TAG/dsab ${DSVARS:-main} ;;
    kvtests) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/${LIBVAR}/libgine_hip.so \
            run pytest_k_${LIBVAR} 600 python -u -m pytest tests -m gpu -q -rf -k "${KTESTS:-deepset}" --timeout 120 --timeout-method thread ;;
    smoke) run smoke 150 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchnc) run bench_nocpu 600 python bench.py --no-cpu ;;
    bench1) run bench_cfg1 600 python bench.py --config 1 ;;
    bench64) run bench_cfg2_d64 600 python bench.py --hidden 64 ;;
    dropin) run bench_dropin 600 python bench.py --dropin --steps 30 ;;
    dropinprof) run rocprof_dropin 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
               -d "$OUT/prof_dropin" -o run -- python3 bench.py --dropin --steps 20 --warmup 5 ;;
    prof64) run rocprof_d64 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof64" -o run -- \
               python3 bench.py --hidden 64 --steps 20 --warmup 5 --no-cpu --no-strong ;;
    bench3) run bench_cfg3 600 python bench.py --config 3 --steps 20 ;;
    bench5) run bench_cfg5 600 python bench.py --config 5 --steps 20 ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
               python3 bench.py --steps 20 --warmup 5 --no-cpu --no-strong ;;
    pmc)   # PMC_ARGS: bench options of the configuration (e.g. "--config 3"); PMC_NAME: its name
           P=${PMC_NAME:-cfg2}
           run pmc_fetch_$P 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$P" -o run -- \
               python3 bench.py --steps 5 --warmup 2 --no-cpu --no-strong --no-graph --kernel-reps 5 ${PMC_ARGS:-}
           run pmc_write_$P 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$P" -o run -- \
               python3 bench.py --steps 5 --warmup 2 --no-cpu --no-strong --no-graph --kernel-reps 5 ${PMC_ARGS:-}
           python tools/pmc_summary.py "$OUT"/pmc_fetch_$P/run_counter_collection.csv \
               "$OUT"/pmc_write_$P/run_counter_collection.csv --config $P \
               --tree-hash "$(python -c 'import bench; print(bench.source_tree_hash())')" \
               --traffic-json "$OUT/${P}_pmc_traffic.json" > "$OUT/${P}_pmc_summary.txt" 2>&1 ;;
    libtests) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/${LIBVAR}/libgine_hip.so \
            run pytest_${LIBVAR} 660 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread ;;
    overlap1)  # world-1 RCCL rehearsal: the captured step with the overlapped tail all-reduce
           # against the split form -- the same final loss bits (an all-reduce over one rank
           # is exact) and both lines' timings
           for m in graph split; do
             run rccl1_$m 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 1 \
                 --force-allreduce --allreduce $m --no-cpu --no-strong --steps 30 --kernel-reps 5
           done
           python - "$OUT" <<'PY' | tee -a "$OUT/session.log"
import json, sys
o = sys.argv[1]
d = {m: json.loads([l for l in open(f"{o}/rccl1_{m}.log") if l.startswith("{")][-1]) for m in ("graph", "split")}
for m, v in d.items():
    print(m, v["ms_per_step"], v["config"].get("allreduce_in_graph"), v["config"].get("allreduce_overlap"), v["final_loss"])
print("same final loss bits:", d["graph"]["final_loss"] == d["split"]["final_loss"])
PY
           ;;
    dist2) run bench_dist2_gloo 600 python bench.py --gpus 2 --dist-backend gloo --steps 10 \
               --warmup 3 --no-cpu ;;
    rgprof) GINE_HIP_LIB=raincast-gnn_amd/raincast_gnn/_native/var/rgprof/libgine_hip.so run rg_prof 300 python tools/rg_prof.py ;;
    var)   for v in raincast-gnn_amd/csrc/build/var/*/; do n=$(basename "$v")
             GINE_HIP_LIB=${v}libgine_hip.so run var_${n}_base 300 python bench.py --no-cpu --steps 30 ${VARARGS:-}
           done ;;
    varbase) run var_base 300 python bench.py --no-cpu --steps 30 ${VARARGS:-} ;;
    mpmicro) run mp_micro 300 python tools/mp_micro.py ${MPARGS:-} ;;
    mpvar) for v in raincast-gnn_amd/csrc/build/var/*/; do n=$(basename "$v")
             GINE_HIP_LIB=${v}libgine_hip.so run mp_micro_${n} 300 python tools/mp_micro.py ${MPARGS:-}
           done ;;
    mpnvar) for v in raincast-gnn_amd/raincast_gnn/_native/var/mp_*/; do n=$(basename "$v")
             GINE_HIP_LIB=${v}libgine_hip.so run mp_micro_${n} 300 python tools/mp_micro.py ${MPARGS:-}
           done ;;
    mpsq)  run mp_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/mp_sq1" -o run -- \
               python3 tools/mp_micro.py --eager --reps 5 ${MPARGS:-}
           run mp_sq2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/mp_sq2" -o run -- \
               python3 tools/mp_micro.py --eager --reps 5 ${MPARGS:-}
           run mp_l2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d "$OUT/mp_l2" -o run -- \
               python3 tools/mp_micro.py --eager --reps 5 ${MPARGS:-} ;;
    floor) run launch_floor 300 python tools/launch_floor.py ;;
    counters) run list_counters 300 rocprofv3 -L ;;
    dsmicro) run ds_micro 300 python tools/ds_micro.py ;;
    dssq)  run ds_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$OUT/ds_sq1" -o run -- \
               python3 tools/ds_micro.py --reps 5 --nodes 16000
           run ds_sq2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/ds_sq2" -o run -- \
               python3 tools/ds_micro.py --reps 5 --nodes 16000 ;;
    sq)    run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$OUT/pmc_sq" -o run -- \
               python3 bench.py --steps 5 --warmup 2 --no-cpu --no-graph --kernel-reps 5 ;;
  esac
done
echo "session done" | tee -a "$OUT/session.log"
