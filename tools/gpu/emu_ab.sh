#!/bin/bash
# same-box A/B of the s26 x W per-rank emulation: one run per library in $VARIANTS ("name:path"), REPS rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-emuab}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for v in $VARIANTS; do
  name=${v%%:*}; lib=${v#*:}
  GHS_MST_LIB=$lib timeout -k 10 300 python -u tools/dist_emulate.py --scale ${SCALE:-26} --world ${W:-8} --reps 2 --no-ref > $OUT/$name.$rep.txt 2> $OUT/$name.$rep.err || { echo "$name failed"; tail -20 $OUT/$name.$rep.err; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$name.$rep.txt'):
    d=json.loads(l); print('$name', d['rep'], d['sum_max_rank_compute_ms'])"
done
done
