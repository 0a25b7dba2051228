#!/bin/bash
# level-plan sweep on one box: bench lines at each level growth (R-MAT s24 unless BENCH_ARGS)
set -o pipefail
OUT=gpurun_out/${TAG:-sweep_growth}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
for g in ${GS:-4 8 16 100}; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-scaling-base --level-growth $g ${BENCH_ARGS} > "$OUT/g$g.$rep.json" 2> "$OUT/g$g.$rep.err" || { echo "bench $g failed"; tail -30 "$OUT/g$g.$rep.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/g$g.$rep.json'));print('$g', 'value', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3))"
done
done
