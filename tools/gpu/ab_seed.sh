#!/bin/bash
# Parity suite with the a-side seed on, then A/B of GHS_SEED_RUNS on R-MAT s24 and the grid.
set -o pipefail
OUT=gpurun_out/${TAG:-abseed}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for rep in 1 2; do
for wl in rmat grid; do
for sr in 0 1; do
  GHS_SEED_RUNS=$sr timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline > "$OUT/$wl.$sr.$rep.json" 2> "$OUT/$wl.$sr.$rep.err" || { echo "bench failed"; tail -20 "$OUT/$wl.$sr.$rep.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$wl.$sr.$rep.json'));print('$wl seed=$sr', round(d['value']/1e9,3), 'ms', d['ms_per_step'], d['mst'])"
done; done; done
