#!/bin/bash
# Kernel-trace profile of the emulated N-rank decomposition (all ranks' kernels on one GPU:
# per-rank cost = totals / N per step).
set -o pipefail
OUT=gpurun_out/${TAG:-profemu}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/dist_emulate.py --scale ${SCALE:-26} --world ${WORLD:-8} --reps 1 --no-ref > "$OUT/emu.jsonl" 2> "$OUT/emu.err" || { echo "rocprof failed"; tail -30 "$OUT/emu.err"; exit 1; }
python3 tools/prof_summary.py "$OUT/prof/run_results.db" > "$OUT/kernels.md" && head -30 "$OUT/kernels.md"
