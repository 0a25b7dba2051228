#!/bin/bash
# One kernel-traced bench run (no tests): per-kernel summary, timeline and its aggregate.
set -o pipefail
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "rocprof bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'])"
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -25 "$OUT/kernels.md"
python3 tools/prof_timeline.py "$OUT/prof/run_results.db" "^k_select\\b(?!_)" -2 > "$OUT/timeline.txt"; python3 tools/timeline_agg.py "$OUT/timeline.txt" > "$OUT/timeline_agg.txt"; cat "$OUT/timeline_agg.txt"
rm -rf "$OUT/prof"
