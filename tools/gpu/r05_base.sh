#!/bin/bash
# Round 5, first box: the shipped r04 tree measured — bench lines of every workload, per-round
# profiles (R-MAT s24, grid), a rocprofv3 kernel-trace summary of the default bench.
set -o pipefail
OUT=gpurun_out/${TAG:-r05base}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|134|137|139) echo "step '$2' ended with $1: stopping"; exit 1;; esac; }
for spec in ${BENCHES:-rmat grid grid-gradient rmat:26}; do
  w=${spec%%:*}; extra=""; tag=$w; [ "$spec" != "$w" ] && { extra="--scale ${spec#*:}"; tag=${w}${spec#*:}; }
  timeout -k 10 300 python3 -u bench.py --workload $w $extra --no-cpu-baseline --no-scaling-base > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"; rc=$?
  fatal $rc bench-$tag
  [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag','value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'rounds',d['breakdown']['rounds'],'flags',d['breakdown']['pass_flags'])" || tail -5 "$OUT/bench_$tag.err"
done
for spec in ${ROUNDS:-rmat:24 grid:0}; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$OUT/rounds_${wl}_$sc.txt" 2>&1; rc=$?
  fatal $rc rounds-$spec
  cat "$OUT/rounds_${wl}_$sc.txt"
done
if [ -z "$NOTRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-scaling-base > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"; rc=$?
fatal $rc rocprof
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -30 "$OUT/kernels.md"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
fi
