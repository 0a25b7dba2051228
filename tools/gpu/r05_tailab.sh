#!/bin/bash
# tail tests, then the same-box A/B against the r04 tree (R-MAT s24, grid), then both round profiles
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tailab
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "tail or totals or golden or random_tie" > gpurun_out/tailab/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/tailab/pytest.log | tail -8
case $rc in 0) ;; *) exit 1;; esac
WLS="${WLS:-rmat grid}" REPS=${REPS:-3} TAG=tailab bash tools/gpu/ab_trees.sh || exit 1
for side in base new; do dir=.; [ $side = base ] && dir=exp_base; (cd $dir && timeout -k 10 200 python3 -u tools/round_profile.py --workload rmat --scale 24 2>&1 | grep -E " L0 live  *[0-9]{7} frags  *[0-9]{1,5} |L1 live  *252|noop|sum") || exit 1; done
