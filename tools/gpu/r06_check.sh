#!/bin/bash
# Round 6 batch: the CSR microbenchmark, the whole GPU suite, the default bench line and the s24
# per-round profile — each step under its own limit, chained so that a failure stops the call.
set -o pipefail
OUT=gpurun_out/${TAG:-r06chk}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$NOMB" ]; then
  timeout -k 10 200 python3 -u tools/csr_rows_bench.py > "$OUT/csr_rows.json" 2> "$OUT/csr_rows.err" || { echo "microbench failed"; tail -5 "$OUT/csr_rows.err"; exit 1; }
  cat "$OUT/csr_rows.json"
fi
if [ -z "$NOTESTS" ]; then
  timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; }
fi
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-scaling-base > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['ms_per_step'], d['value']/1e9, 'G edges/s, s1', d['stage1_roofline']['frac'])"
timeout -k 10 200 python3 -u tools/round_profile.py > "$OUT/rounds_rmat.txt" 2>&1 && tail -8 "$OUT/rounds_rmat.txt"
