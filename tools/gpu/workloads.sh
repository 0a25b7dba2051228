#!/bin/bash
# Bench lines for the BASELINE configs other than the headline: grid 16384^2 (config 5, uniform
# and gradient weights) and R-MAT s26 on one GPU (config 4's graph, the N=8 target, solved by one
# rank) — plus a kernel-trace profile of the grid run.
set -o pipefail
OUT=gpurun_out/${TAG:-workloads}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in grid grid-gradient; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 > "$OUT/$w.json" 2> "$OUT/$w.err" || { echo "bench $w failed"; tail -30 "$OUT/$w.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', 'value', round(d['value']/1e9,3), 'ms', d['ms_per_step'], 'rounds', d['breakdown']['rounds'], 'levels', d['breakdown']['levels'], 'mst', d['mst'])"
done
timeout -k 10 300 python3 bench.py --scale 26 --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/s26.json" 2> "$OUT/s26.err" || { echo "bench s26 failed"; tail -30 "$OUT/s26.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/s26.json'));print('s26', 'value', round(d['value']/1e9,3), 'ms', d['ms_per_step'], 'rounds', d['breakdown']['rounds'], 'mst', d['mst'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_grid" -o run -- python3 bench.py --workload grid --no-cpu-baseline --steps 3 --warmup 1 > "$OUT/grid_prof.json" 2> "$OUT/grid_prof.err" || { echo "rocprof grid failed"; tail -30 "$OUT/grid_prof.err"; exit 1; }
python3 tools/prof_summary.py "$OUT/prof_grid/run_results.db" > "$OUT/grid_kernels.md" && head -25 "$OUT/grid_kernels.md"
