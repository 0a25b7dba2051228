#!/bin/bash
# Finer level-plan sweep around the r03 candidates (more repeats).
set -o pipefail
OUT=gpurun_out/${TAG:-sweep3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { name=$1; shift; timeout -k 10 300 python3 -u tools/sweep_levels.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err" || { echo "$name sweep failed"; tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$name.jsonl'):
    d=json.loads(l); print('$name', d['levels'], d['l1'], d['growth'], d['ms'], d['rounds'], d['planned_levels'])
"; }
run rmat24 --workload rmat --scale 24 --reps 9 --levels 3 --l1 0.5,0.3,0.35,0.4,0.5 --growth 8
run rmat26 --workload rmat --scale 26 --reps 5 --levels 3 --l1 0.5,0.35,0.5,0.35 --growth 8
run grid --workload grid --reps 5 --levels 2 --l1 1.0,1.15,1.2,1.25,1.0 --growth 2
run gradient --workload grid-gradient --reps 5 --levels 2 --l1 1.0,1.2,1.3,1.4,1.0 --growth 2
