#!/bin/bash
# HBM traffic per launch of the bench's kernels: one rocprofv3 --pmc run per counter (FETCH_SIZE
# needs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass), each under its own time limit.
set -o pipefail
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KRE=${KRE:-k_filter|k_select|k_minedge|k_level_pass|k_win}
WL=${WL:-rmat-s24-ef16}
BENCH_ARGS=${BENCH_ARGS:---no-scaling-base}  # the headline workload only (no s26 scaling leg)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d "$OUT/fetch" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 0 ${BENCH_ARGS} > "$OUT/fetch.json" 2> "$OUT/fetch.err" || { echo "fetch pass failed"; tail -5 "$OUT/fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d "$OUT/write" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 0 ${BENCH_ARGS} > "$OUT/write.json" 2> "$OUT/write.err" || { echo "write pass failed"; tail -5 "$OUT/write.err"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$WL" "$OUT/${WL}_pmc.json"
rm -rf "$OUT/fetch" "$OUT/write"
