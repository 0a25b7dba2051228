#!/bin/bash
# generation timing (s24, s26) and a kernel-trace summary of one s24 generation (full names)
set -o pipefail
OUT=gpurun_out/${TAG:-gen}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/gen_time.py --scales ${SCALES:-24 26} --reps 3 > "$OUT/gen.jsonl" 2> "$OUT/gen.err" || { echo "gen failed"; tail -20 "$OUT/gen.err"; exit 1; }
cat "$OUT/gen.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 tools/gen_time.py --scales 24 --reps 1 > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name "*.db" | head -1)
[ -n "$f" ] && python3 tools/prof_summary.py "$f" --width 260 > "$OUT/kernel_stats.md" && cat "$OUT/kernel_stats.md"
find "$OUT/prof" -name "*.db" -delete
true
