#!/bin/bash
# A/B timing on the GPU box: optional parity tests (default library), then one unprofiled bench
# run per variant. Variants are "name:VAR=val,VAR=val" words in $VARIANTS (env for that run only),
# e.g. VARIANTS="base: w1:GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/libghs_mst_w1.so".
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
for rep in $(seq 1 ${REPS:-1}); do
for v in $VARIANTS; do
  name=${v%%:*}
  envs=${v#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-scaling-base ${BENCH_ARGS} > "$OUT/$name.$rep.json" 2> "$OUT/$name.$rep.err" ) || { echo "bench $name failed"; tail -30 "$OUT/$name.$rep.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.$rep.json'));print('$name', 'value', round(d['value']/1e9,3), 'ms', round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k, v in list((d.get('kernels') or {}).items())[:${TOPK:-6}]})"
done
done
