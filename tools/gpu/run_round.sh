#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprof kernel-trace summary. Every GPU step has its
# own time limit and the steps are chained: the first failure ends the call.
set -o pipefail
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
