#!/bin/bash
# level-plan sweep on one box: bench lines at each level1 (edges per vertex) for one workload
set -o pipefail
OUT=gpurun_out/${TAG:-sweep_plan}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
for l1 in ${L1S:-1.0 1.2 1.4}; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-scaling-base --workload ${WL:-grid} --level1 $l1 ${BENCH_ARGS} > "$OUT/l$l1.$rep.json" 2> "$OUT/l$l1.$rep.err" || { echo "bench $l1 failed"; tail -30 "$OUT/l$l1.$rep.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/l$l1.$rep.json'));print('$l1', 'value', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3))"
done
done
