#!/bin/bash
# rocprofv3 kernel-trace summaries of the grid bench lines (the roofline kernel's average duration
# is checked against the line's own events), each under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-tracegrids}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in grid grid-gradient; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$wl" -o run -- python3 bench.py --workload $wl --no-cpu-baseline --no-scaling-base > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "rocprof $wl failed"; tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/prof_summary.py "$OUT/prof_$wl/run_results.db" > "$OUT/kernels_$wl.md" && head -14 "$OUT/kernels_$wl.md"
  rm -rf "$OUT/prof_$wl"
  python3 -c "
import json
d=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$wl', d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['launches'], r['frac'], r['traffic'])"
done
