#!/bin/bash
# Level-plan sweep on the grid workloads (speed only; the MSF weight is asserted identical).
set -o pipefail
OUT=gpurun_out/${TAG:-sweepgrid}
mkdir -p "$OUT"
for w in grid grid-gradient; do
timeout -k 10 400 python3 tools/sweep_levels.py --workload $w --reps 2 --levels ${LEVELS:-1,2,3,4} --l1 ${L1:-0.25,0.5,0.75,1.0,1.25,1.5} --growth ${GROWTH:-2,4,8} > "$OUT/$w.jsonl" 2> "$OUT/$w.err" || { echo "sweep $w failed"; tail -20 "$OUT/$w.err"; exit 1; }
python3 -c "
import json
r=[json.loads(l) for l in open('$OUT/$w.jsonl')]
r.sort(key=lambda d:d['ms'])
for d in r[:8]: print('$w', d['levels'], d['l1'], d['growth'], d['ms'], d['rounds'], d['edges_per_level'])
"
done
