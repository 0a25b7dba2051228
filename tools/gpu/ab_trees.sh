#!/bin/bash
# Same-box A/B of two source trees: the current tree and a git worktree of another revision
# (BASE, default exp_base; built in place beforehand), bench lines alternated REPS times per
# workload. Each run under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-abtrees}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=${BASE:-exp_base}
for w in ${WLS:-rmat}; do
for rep in $(seq 1 ${REPS:-3}); do
  for side in base new; do
    dir=.; [ $side = base ] && dir=$BASE
    ( cd $dir && timeout -k 10 240 python3 -u bench.py --workload $w --no-cpu-baseline --no-scaling-base $BARGS ) > "$OUT/$w.$side.$rep.json" 2> "$OUT/$w.$side.$rep.err"; rc=$?
    case $rc in 0) ;; 124|134|137|139) echo "$side $w ended with $rc: stopping"; exit 1;; *) echo "$side $w failed"; tail -5 "$OUT/$w.$side.$rep.err"; continue;; esac
    python3 -c "import json;d=json.load(open('$OUT/$w.$side.$rep.json'));print('$w $side rep $rep', 'ms', round(d['ms_per_step'],4), 's1', d['stage1_roofline']['frac'])"
  done
done
done
