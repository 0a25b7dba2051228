#!/bin/bash
# Round 6: the grid lines (uniform and gradient weights) and their per-round profiles.
set -o pipefail
OUT=gpurun_out/${TAG:-r06grid}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in ${WORKLOADS:-grid grid-gradient}; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --no-cpu-baseline --no-scaling-base $BARGS > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "bench $wl failed"; tail -5 "$OUT/bench_$wl.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$wl.json'));print('$wl', d['ms_per_step'], d['value']/1e9, 'G edges/s')"
  if [ -z "$NOROUNDS" ]; then
    timeout -k 10 300 python3 -u tools/round_profile.py --workload $wl > "$OUT/rounds_$wl.txt" 2>&1 || { echo "rounds $wl failed"; tail -5 "$OUT/rounds_$wl.txt"; exit 1; }
    head -3 "$OUT/rounds_$wl.txt" | tail -2
  fi
done
