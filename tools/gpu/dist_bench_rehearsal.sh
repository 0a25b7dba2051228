#!/bin/bash
# bench.py's N > 1 leg at its real size (R-MAT s26) with N ranks sharing the box's one GPU over gloo
# (RCCL needs a GPU per rank): the torch.distributed loop, the MSF gather, the edge-for-edge check
# against a one-GPU solve. Each N under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-distbench}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
port=29611
for N in ${NS:-2}; do
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --backend gloo --steps ${STEPS:-2} --warmup 1 $BARGS > "$OUT/bench_n$N.json" 2> "$OUT/bench_n$N.err" || { echo "N=$N failed"; tail -30 "$OUT/bench_n$N.err"; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_n$N.json') if l.startswith('{')][-1])
print('N=$N', d['config']['m'], d['ms_per_step'], d.get('ms_per_step_solve'), d['loop'], d['parity'])"
  port=$((port+1))
done
