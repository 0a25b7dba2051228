#!/bin/bash
# Development loop on the GPU box: parity tests, then one profiled bench run (kernel trace).
set -o pipefail
OUT=gpurun_out/${TAG:-dev}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/bench_plain.json" 2> "$OUT/bench_plain.err" || { echo "bench failed"; tail -30 "$OUT/bench_plain.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_plain.json'));print('UNPROFILED value',d['value'],'ms',d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "rocprof bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline'] and d['roofline']['frac'])"
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -25 "$OUT/kernels.md"
python3 tools/prof_timeline.py "$OUT/prof/run_results.db" > "$OUT/timeline.txt"; tail -1 "$OUT/timeline.txt"; python3 tools/timeline_agg.py "$OUT/timeline.txt" > "$OUT/timeline_agg.txt"
