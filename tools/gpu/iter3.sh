#!/bin/bash
# Round-3 development loop: GPU parity suite, then bench lines (no CPU baselines) for the given
# workloads; each step under its own limit, the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${TAG:-iter}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$NOTEST" ]; then
timeout -k 10 ${LIMIT:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
fi
for wl in ${WLS:-rmat grid grid-gradient}; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --no-cpu-baseline --no-scaling-base ${BENCH_ARGS:-} > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
  python3 - "$OUT/bench_$wl.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "value %.4g ms %.4f" % (d["value"], d["ms_per_step"]))
s1 = d["stage1_roofline"]; print("  stage1", s1 and s1["frac"], s1 and s1["ms"])
for k, v in list(d["kernels"].items())[:12]: print("  %-22s %3d  %8.4f ms  frac %s" % (k, v["launches"], v["ms_per_step"], v["frac"]))
PY
done
