#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench command (no CPU baseline leg, so the
# profile holds only the timed GPU path + warmup + generation).
set -o pipefail
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
cat "$OUT/prof_bench.json" | head -c 600; echo
find "$OUT/prof" -name '*kernel_stats.csv' | head -5
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
head -40 "$f"
