#!/bin/bash
# the native emulated loop with lib/exp/base.so and the tree: host time + kernel-trace totals
set -o pipefail
OUT=gpurun_out/${TAG:-inplace}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base new; do
  if [ $v = base ]; then export GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so; else unset GHS_MST_LIB; fi
  timeout -k 10 200 python3 -u tools/emu_native.py 26 8 3 > "$OUT/$v.txt" 2>&1 || { echo "$v failed"; tail -20 "$OUT/$v.txt"; exit 1; }
  grep rep "$OUT/$v.txt" | sed "s/^/$v /"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run -- python3 tools/emu_native.py 26 8 1 > "$OUT/prof_$v.log" 2>&1 || { echo "rocprof $v failed"; tail -20 "$OUT/prof_$v.log"; exit 1; }
  python3 tools/prof_summary.py "$OUT/prof_$v/run_results.db" > "$OUT/kernels_$v.md"
  grep -E "pack_best|unpack_best|emu_min|total kernel" "$OUT/kernels_$v.md" | sed "s/^/$v /"
  find "$OUT/prof_$v" -name "*.db" -delete
done
