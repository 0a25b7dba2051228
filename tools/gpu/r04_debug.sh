#!/bin/bash
set -o pipefail
OUT=gpurun_out/${TAG:-r04dbg}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in ${SPECS:-rmat:20:24 rmat:15:16}; do
  timeout -k 10 300 python3 -u tools/debug_paths.py $spec > "$OUT/dbg_$spec.txt" 2>&1 || { echo "debug $spec failed"; tail -30 "$OUT/dbg_$spec.txt"; exit 1; }
  echo "== $spec"; cat "$OUT/dbg_$spec.txt"
done
