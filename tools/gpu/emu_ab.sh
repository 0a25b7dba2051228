#!/bin/bash
# Native multi-rank loop (ghs_mst_emulated) at R-MAT s26 x8 on one GPU, per library variant
# (VARIANTS: "name:GHS_MST_LIB=path" words, "base:" = the tree's library), REPS repetitions.
set -o pipefail
OUT=gpurun_out/${TAG:-emuab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; envs=${v#*:}
  ( [ -n "$envs" ] && export "$envs"; timeout -k 10 300 python3 -u tools/emu_native.py ${SCALE:-26} ${WORLD:-8} ${REPS:-6} > "$OUT/$name.txt" 2>&1 ) || { echo "emu $name failed"; tail -20 "$OUT/$name.txt"; exit 1; }
  echo "== $name"; grep rep "$OUT/$name.txt"
done
