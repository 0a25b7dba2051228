#!/bin/bash
# Quick loop: a pytest subset (PYTEST_K), then bench lines for WLS; each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$PYTEST_K" ]; then
timeout -k 10 ${LIMIT:-400} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
fi
for wl in ${WLS:-grid}; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --no-cpu-baseline --no-scaling-base ${BENCH_ARGS:-} > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
  python3 - "$OUT/bench_$wl.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "value %.4g ms %.4f" % (d["value"], d["ms_per_step"]))
s1 = d["stage1_roofline"]; print("  stage1", s1 and s1["frac"], s1 and s1["ms"])
for k, v in list(d["kernels"].items())[:12]: print("  %-22s %3d  %8.4f ms  frac %s" % (k, v["launches"], v["ms_per_step"], v["frac"]))
PY
done
if [ -n "$ROUNDS" ]; then
  for wl in $ROUNDS; do timeout -k 10 200 python3 tools/round_profile.py --workload $wl > "$OUT/rounds_$wl.txt" 2>&1 || { echo "round profile failed"; tail -20 "$OUT/rounds_$wl.txt"; exit 1; }; cat "$OUT/rounds_$wl.txt"; done
fi
