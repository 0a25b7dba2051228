#!/bin/bash
# The native emulated multi-rank loop (tools/emu_native.py) on the tree's library and on $CAND.
set -o pipefail
OUT=gpurun_out/${TAG:-emuab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base: cand:distributed_ghs_implementation_amd/lib/exp/$CAND.so base: cand:distributed_ghs_implementation_amd/lib/exp/$CAND.so; do
  name=${v%%:*}; lib=${v#*:}
  ( [ -n "$lib" ] && export GHS_MST_LIB=$lib; timeout -k 10 200 python3 -u tools/emu_native.py 26 8 ${REPS:-4} ) >> "$OUT/$name.txt" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.txt"; exit 1; }
  echo "== $name"; grep "^rep" "$OUT/$name.txt" | tail -${REPS:-4}
done
