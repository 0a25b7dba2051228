#!/bin/bash
# Parity suite (incl. the full-size tests), then bench lines for R-MAT s24 and the grids.
set -o pipefail
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --durations=12 --timeout 300 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
grep -E "passed|failed" "$OUT/pytest_gpu.log" | tail -1
grep -A14 "slowest" "$OUT/pytest_gpu.log"
for w in rmat grid grid-gradient; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$w.json" 2> "$OUT/$w.err" || { echo "bench $w failed"; tail -30 "$OUT/$w.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', 'value', round(d['value']/1e9,3), 'ms', d['ms_per_step'], 'rounds', d['breakdown']['rounds'], 'levels', d['breakdown']['levels'], 'mst', d['mst'])"
done
