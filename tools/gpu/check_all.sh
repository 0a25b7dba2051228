#!/bin/bash
# The GPU parity suite, then one bench line (with its CPU baseline); each step under its own
# limit, the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${TAG:-check}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 ${LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4g ms %.4f" % (d["value"], d["ms_per_step"]))
r = d["roofline"]; print("roofline", r["kernel"], r["frac"], r["avg_launch_ms"], r["launches"], "traffic", r["traffic"])
print("stage1", d["stage1_roofline"] and d["stage1_roofline"]["frac"], d["stage1_roofline"] and d["stage1_roofline"]["ms"])
for k, v in d["kernels"].items(): print("  %-22s %3d  %8.4f ms  frac %s" % (k, v["launches"], v["ms_per_step"], v["frac"]))
if d.get("cpu_baseline"): print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
if d.get("scaling_base"): print("scaling_base", d["scaling_base"])
PY
