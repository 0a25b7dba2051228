#!/bin/bash
# Round 6: s26 x 8 per-rank emulation (tools/dist_emulate.py --profile --per-rank) over variants
# "name:extra args" in $EMUS; the kernels-only line of each printed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r06emu}
mkdir -p $OUT
for v in ${EMUS:-base:}; do
  name=${v%%:*}; args=${v#*:}; args=${args//,/ }
  timeout -k 10 400 python3 -u tools/dist_emulate.py --scale ${SCALE:-26} --world ${W:-8} --reps 2 --profile --per-rank $args > $OUT/emu_$name.txt 2> $OUT/emu_$name.err || { echo "emu $name failed"; tail -5 $OUT/emu_$name.err; exit 1; }
  echo "$name: $(grep -o '"sum_max_rank_compute_ms": [0-9.]*' $OUT/emu_$name.txt | tail -1) $(grep 'kernels only' $OUT/emu_$name.err)"
  grep "round 7 rank\|round 6 rank" $OUT/emu_$name.err | awk '{print $3, $5, $6, $8}' | tr '\n' ' '; echo
done
