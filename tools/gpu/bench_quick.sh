#!/bin/bash
# bench.py lines for the given workloads (default: the N=1 headline with CPU baselines) + a
# rocprofv3 kernel-trace summary of the headline; each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-benchq}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4g ms %.4f" % (d["value"], d["ms_per_step"]))
r = d["roofline"]; print("roofline", r["kernel"], r["frac"], r["avg_launch_ms"], r["launches"])
print("stage1", d["stage1_roofline"])
for k, v in d["kernels"].items(): print("  %-22s %3d  %8.4f ms  frac %s" % (k, v["launches"], v["ms_per_step"], v["frac"]))
if d.get("cpu_baseline"): print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"], d["cpu_baseline"]["host_cpus"])
if d.get("scaling_base"): print("scaling_base", d["scaling_base"])
PY
if [ -n "$PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-scaling-base ${BENCH_ARGS:-} > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -24 "$OUT/kernels.md"
python3 tools/prof_timeline.py "$OUT/prof/run_results.db" > "$OUT/timeline.txt"; python3 tools/timeline_agg.py "$OUT/timeline.txt" > "$OUT/timeline_agg.txt"; cat "$OUT/timeline_agg.txt"
rm -f "$OUT/prof/run_results.db"
fi
