#!/bin/bash
# Per-round kernel profiles (tools/round_profile.py) of the bench workloads; each under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-rounds}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in ${SPECS:-rmat:24 rmat:26 grid:0 grid-gradient:0}; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$OUT/rounds_${wl}_$sc.txt" 2>&1 || { echo "round profile $spec failed"; tail -20 "$OUT/rounds_${wl}_$sc.txt"; exit 1; }
  echo "== $spec"; cat "$OUT/rounds_${wl}_$sc.txt"
done
