#!/bin/bash
# Full suite + bench lines on the tree's library (full3.sh), the grid level sweep, then a candidate
# library ($CAND, lib/exp/<name>.so): its parity subset and grid A/B round profiles against the tree's.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_FULL" ]; then TAG=${TAG:-re}_full bash tools/gpu/full3.sh || exit 1; fi
if [ -z "$SKIP_SWEEP" ]; then TAG=${TAG:-re}_sweep bash tools/gpu/sweep_grid2.sh || exit 1; fi
if [ -n "$CAND" ]; then
  lib=distributed_ghs_implementation_amd/lib/exp/$CAND.so
  OUT=gpurun_out/${TAG:-re}_cand; mkdir -p $OUT
  GHS_MST_LIB=$lib timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${CAND_K:-windowed or grid or lattice or bucketed or smoke or readme or golden}" > $OUT/pytest_gpu.log 2>&1 || { echo "cand pytest failed"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -20 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  TAG=${TAG:-re}_cand VARIANTS="base: cand:$lib" WL=grid SCALES=0 bash tools/gpu/rounds_ab.sh || exit 1
  TAG=${TAG:-re}_cand VARIANTS="base: cand:$lib" WL=grid-gradient SCALES=0 bash tools/gpu/rounds_ab.sh || exit 1
fi
exit 0
