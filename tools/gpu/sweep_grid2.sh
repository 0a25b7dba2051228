#!/bin/bash
# Level-plan sweep on the grids (tools/sweep_levels.py), each workload under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-sweepgrid}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in ${WLS:-grid grid-gradient}; do
  timeout -k 10 400 python3 -u tools/sweep_levels.py --workload $wl --reps ${REPS:-3} --levels "${LEVELS:-2,3}" --l1 "${L1:-0.8,0.9,1.0,1.1}" --growth "${GROWTH:-1.5,2}" > "$OUT/$wl.jsonl" 2> "$OUT/$wl.err" || { echo "sweep $wl failed"; tail -20 "$OUT/$wl.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$wl.jsonl'):
    d=json.loads(l); print('$wl', d['levels'], d['l1'], d['growth'], d['ms'], d['rounds'], d['planned_levels'])
"
done
