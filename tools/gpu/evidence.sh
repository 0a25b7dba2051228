#!/bin/bash
# Round evidence in one call: parity suite, smoke, the default bench line (with CPU baseline),
# a rocprofv3 kernel-trace summary of the bench, and the HBM-traffic PMC passes. Each GPU step
# has its own limit; the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${TAG:-evidence}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['kernel'],d['roofline']['frac'],'cpu',d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-scaling-base > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -16 "$OUT/kernels.md"
python3 tools/prof_timeline.py "$OUT/prof/run_results.db" > "$OUT/timeline.txt"; python3 tools/timeline_agg.py "$OUT/timeline.txt" > "$OUT/timeline_agg.txt"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
TAG=${TAG:-evidence}/pmc bash tools/gpu/pmc_traffic.sh || { echo "pmc failed"; exit 1; }
