#!/bin/bash
# GPU parity suite only (one process, per-test thread timeouts), log under gpurun_out/.
set -o pipefail
OUT=gpurun_out/${TAG:-pytest}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.log"
exit $rc
