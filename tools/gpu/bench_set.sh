#!/bin/bash
# Optional pytest subset (PYTEST_K), then one bench line per spec in $SPECS ("name|bench args"
# entries separated by ';'); each step under its own limit, the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${TAG:-set}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 ${LIMIT:-500} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
IFS=';' read -ra SP <<< "$SPECS"
for spec in "${SP[@]}"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-scaling-base $args > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "bench $name failed"; tail -30 "$OUT/$name.err"; exit 1; }
  python3 - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s1 = d["stage1_roofline"]
print(sys.argv[2], "value %.4g ms %.4f" % (d["value"], d["ms_per_step"]), "stage1", s1 and s1["frac"], s1 and s1["ms"])
print("   ", {k: round(v["ms_per_step"], 3) for k, v in list(d["kernels"].items())[:int(__import__("os").environ.get("TOPK", "9"))]})
PY
done
