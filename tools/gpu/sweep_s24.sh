#!/bin/bash
# Level-plan sweep on R-MAT s24 around the default (3 levels, 0.5n, x8): speed only.
set -o pipefail
OUT=gpurun_out/${TAG:-sweeps24}
mkdir -p "$OUT"
timeout -k 10 500 python3 tools/sweep_levels.py --workload rmat --scale ${SCALE:-24} --reps 3 --levels ${LEVELS:-2,3,4} --l1 ${L1:-0.3,0.4,0.5,0.6,0.75} --growth ${GROWTH:-4,6,8,12,16} > "$OUT/rmat.jsonl" 2> "$OUT/rmat.err" || { echo "sweep failed"; tail -20 "$OUT/rmat.err"; exit 1; }
python3 -c "
import json
r=[json.loads(l) for l in open('$OUT/rmat.jsonl')]
r.sort(key=lambda d:d['ms'])
for d in r[:12]: print(d['levels'], d['l1'], d['growth'], d['ms'], d['rounds'], d['edges_per_level'])
"
