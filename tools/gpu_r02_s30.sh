#!/usr/bin/env bash
# Distributed rehearsals on one GPU: RCCL all-reduce captured in the step graph (world 1,
# forced collective) and two gloo ranks sharing the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_s30; mkdir -p $O
st() { local rc=$1; [ $rc -le 1 ] || { echo "crash-class $rc"; exit $rc; }; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --force-allreduce --no-cpu --steps 30 --warmup 5 > $O/rccl1.json 2> $O/rccl1.err; st $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 10 --warmup 3 > $O/gloo2.json 2> $O/gloo2.err; st $?
for f in rccl1 gloo2; do python - $O/$f.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['n_gpus'], d['value'], d['ms_per_step'], d['config']['allreduce_in_graph'], d.get('strong_scaling_cfg4',{}) and d['strong_scaling_cfg4']['value'])
PY
done
