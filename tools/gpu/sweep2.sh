#!/bin/bash
# Level-plan sweeps on the current library: the grids over l1, R-MAT s24 over l1 / growth / levels.
set -o pipefail
OUT=gpurun_out/${TAG:-sweep2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/sweep_levels.py --workload grid --reps 3 --levels 2 --l1 1.0,1.1,1.2,1.3,1.5 --growth 2 > "$OUT/grid.jsonl" 2> "$OUT/grid.err" || { echo "grid sweep failed"; tail -20 "$OUT/grid.err"; exit 1; }
timeout -k 10 300 python3 -u tools/sweep_levels.py --workload grid-gradient --reps 3 --levels 2 --l1 1.0,1.1,1.2,1.3 --growth 2 > "$OUT/gradient.jsonl" 2> "$OUT/gradient.err" || { echo "gradient sweep failed"; tail -20 "$OUT/gradient.err"; exit 1; }
timeout -k 10 300 python3 -u tools/sweep_levels.py --workload rmat --scale 24 --reps 5 --levels 3,4 --l1 0.35,0.5,0.7 --growth 4,8,16 > "$OUT/rmat.jsonl" 2> "$OUT/rmat.err" || { echo "rmat sweep failed"; tail -20 "$OUT/rmat.err"; exit 1; }
for f in grid gradient rmat; do python3 -c "
import json
for l in open('$OUT/$f.jsonl'):
    d=json.loads(l); print('$f', d['levels'], d['l1'], d['growth'], d['ms'], d['rounds'], d['planned_levels'])
"; done
