#!/bin/bash
# The bench lines of every BASELINE workload on one GPU (headline with CPU baselines + s26
# scaling point; both grids), each step under its own limit; lines under gpurun_out/$TAG/.
set -o pipefail
OUT=gpurun_out/${TAG:-benchall}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u bench.py ${S24_ARGS:-} > "$OUT/bench_s24.json" 2> "$OUT/bench_s24.err" || { echo "s24 failed"; tail -20 "$OUT/bench_s24.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload grid --steps 5 --no-cpu-baseline > "$OUT/bench_grid16k.json" 2> "$OUT/bench_grid16k.err" || { echo "grid failed"; tail -20 "$OUT/bench_grid16k.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload grid-gradient --steps 5 --no-cpu-baseline > "$OUT/bench_grid16k_gradient.json" 2> "$OUT/bench_grid16k_gradient.err" || { echo "gradient failed"; tail -20 "$OUT/bench_grid16k_gradient.err"; exit 1; }
for f in "$OUT"/bench_*.json; do
python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; s1 = d["stage1_roofline"] or {}
print("%-28s %.4g edges/s  %.3f ms  dominant %s frac %.3f  stage1 %.3f" % (d["config"]["workload"], d["value"], d["ms_per_step"], r["kernel"], r["frac"], s1.get("frac", 0)))
if d.get("cpu_baseline"): print("   cpu omp", d["cpu_baseline"]["value"], "cores", d["cpu_baseline"]["cores"])
if d.get("scaling_base"): print("   scaling_base", d["scaling_base"]["workload"], d["scaling_base"]["value"], d["scaling_base"]["ms_per_step"])
PY
done
