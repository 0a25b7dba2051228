#!/bin/bash
# Per-round profiles of R-MAT scales ($SCALES) for each library variant ($VARIANTS "name:path" words,
# "base:" = the tree's library); each run under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-roundsab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base:}; do
  name=${v%%:*}; lib=${v#*:}
  for sc in ${SCALES:-24 26}; do
    ( [ -n "$lib" ] && export GHS_MST_LIB=$lib; timeout -k 10 240 python3 -u tools/round_profile.py --workload ${WL:-rmat} --scale $sc > "$OUT/${name}_$sc.txt" 2>&1 ) || { echo "$name s$sc failed"; tail -20 "$OUT/${name}_$sc.txt"; exit 1; }
    echo "== $name s$sc"; grep -v amdgpu.ids "$OUT/${name}_$sc.txt" | grep -E "^m=|^r ?[0-9]+ L. live.* frags +[0-9]{7}"
  done
done
