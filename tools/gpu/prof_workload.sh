#!/bin/bash
# Kernel-trace profile of one bench workload ($WL, default grid) -> per-kernel summary + timeline.
set -o pipefail
OUT=gpurun_out/${TAG:-profwl}
mkdir -p "$OUT"
export TMPDIR=/tmp
WL=${WL:-grid}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --workload $WL --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "rocprof failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step']); print([(r['level'], r['live_arcs'], r['fragments'], r['hooks']) for r in d['breakdown']['per_round']])"
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -24 "$OUT/kernels.md"
python3 tools/prof_timeline.py "$OUT/prof/run_results.db" > "$OUT/timeline.txt"; python3 tools/timeline_agg.py "$OUT/timeline.txt" > "$OUT/timeline_agg.txt"; cat "$OUT/timeline_agg.txt"
