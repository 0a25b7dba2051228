#!/bin/bash
# GPU tests (PYTEST_K), then per-round profiles: the grid for each of $GVARIANTS, R-MAT s24/s26 for
# each of $RVARIANTS ("name:path", "base:" = the tree's library).
set -o pipefail
OUT=gpurun_out/${TAG:-jumpab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 ${LIMIT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
[ -n "$GVARIANTS" ] && { TAG=${TAG:-jumpab} VARIANTS="$GVARIANTS" WL=${GWL:-grid} SCALES=0 bash tools/gpu/rounds_ab.sh || exit 1; }
[ -n "$RVARIANTS" ] && { TAG=${TAG:-jumpab} VARIANTS="$RVARIANTS" WL=rmat SCALES="${RSCALES:-24 26}" bash tools/gpu/rounds_ab.sh || exit 1; }
exit 0
