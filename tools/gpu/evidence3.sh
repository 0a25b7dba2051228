#!/bin/bash
# Round-3 evidence on the current tree: rocprofv3 kernel-trace summary of the default bench, HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes) of every bench workload, and the s26 x8 multi-rank
# emulation. Each GPU step under its own limit; raw profiler databases are deleted after summary
# (gpurun copies back at most 64 MiB).
set -o pipefail
OUT=gpurun_out/${TAG:-ev3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$NOTRACE" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --no-cpu-baseline --no-scaling-base > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo "rocprof failed"; tail -30 "$OUT/prof_bench.err"; exit 1; }
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -24 "$OUT/kernels.md"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv"
rm -rf "$OUT/prof"
fi
KRE="k_filter|k_select|k_minedge|k_level_pass|k_win|k_wmin|k_bucket|k_bmin|k_jump_ident|k_jump|k_hook"
for spec in ${PMC_SPECS:-rmat:rmat-s24-ef16 grid:grid-16384x16384 grid-gradient:grid-gradient-16384x16384}; do
  wl=${spec%%:*}; tag=${spec#*:}
  TAG=${TAG:-ev3}/pmc_$wl KRE="$KRE" WL=$tag BENCH_ARGS="--workload $wl --no-scaling-base" bash tools/gpu/pmc_traffic.sh || { echo "pmc $wl failed"; exit 1; }
done
if [ -z "$NOEMU" ]; then
timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 > "$OUT/emu_s26_w8.jsonl" 2> "$OUT/emu_s26_w8.err" || { echo "emulate failed"; tail -5 "$OUT/emu_s26_w8.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/emu_s26_w8.jsonl'):
    d=json.loads(l); print('rep', d['rep'], 'single', d['single_gpu_ms'], 'compute', d['sum_max_rank_compute_ms'], 'wire MB/rank', round(d['wire_bytes_per_rank']/1e6,1))
"
fi
