#!/bin/bash
# Round-6 evidence on the current tree: the default bench line (as the driver runs it), the other
# workloads' lines, a rocprofv3 kernel-trace summary of the default bench, HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes) of every bench workload's stage-1 and dominant kernels, the
# per-round profiles. Each GPU step under its own limit; raw profiler databases deleted after summary.
set -o pipefail
OUT=gpurun_out/${TAG:-r06final}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|134|137|139) echo "step '$2' ended with $1: stopping"; exit 1;; esac; }
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"; rc=$?; fatal $rc bench-default
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print('default value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'dom',d['roofline']['kernel'],d['roofline']['frac'],'cpu',d['cpu_baseline']['value'],'base',d.get('scaling_base',{}).get('ms_per_step'))" || tail -5 "$OUT/bench_default.err"
for w in grid grid-gradient; do
  timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline --no-scaling-base > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err"; rc=$?; fatal $rc bench-$w
  python3 -c "import json;d=json.load(open('$OUT/bench_$w.json'));print('$w value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'dom',d['roofline']['kernel'],d['roofline']['frac'])" || tail -5 "$OUT/bench_$w.err"
done
fi
if [ "${PART:-1}" = 2 ]; then
if [ -z "$NOTRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-scaling-base > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"; rc=$?; fatal $rc rocprof
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -24 "$OUT/kernels.md"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
fi
KRE="k_filter|k_select|k_minedge|k_level_pass|k_win|k_wmin|k_wstarts|k_bucket|k_bmin|k_jump_ident|k_jump|k_hook|k_seed_runs|k_tail_open|k_tail_round|k_tail_hook|k_resolve"
for spec in ${PMC_SPECS:-rmat:rmat-s24-ef16 grid:grid-16384x16384 grid-gradient:grid-gradient-16384x16384}; do
  wl=${spec%%:*}; tag=${spec#*:}
  TAG=${TAG:-r06final}/pmc_$wl KRE="$KRE" WL=$tag BENCH_ARGS="--workload $wl --no-scaling-base" bash tools/gpu/pmc_traffic.sh; rc=$?; fatal $rc pmc-$wl
done
for spec in rmat:24 rmat:26 grid:0 grid-gradient:0; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  f="$OUT/rounds_${wl}.txt"; [ "$sc" = 26 ] && f="$OUT/rounds_${wl}_s26.txt"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$f" 2>&1; rc=$?; fatal $rc rounds-$wl-$sc
done
fi
echo evidence part ${PART:-1} done
