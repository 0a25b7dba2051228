#!/bin/bash
# Full GPU suite, smoke, the default bench line (CPU baselines + s26 scaling base), the grid
# lines, and the native multi-rank loop at s26 x8 on one GPU; each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-full}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench_rmat.json" 2> "$OUT/bench_rmat.err" || { echo "bench failed"; tail -30 "$OUT/bench_rmat.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_rmat.json'));print('rmat value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['kernel'],d['roofline']['frac'],'stage1',d['stage1_roofline']['frac'],'cpu',d['cpu_baseline']['value'],'s26',d['scaling_base']['ms_per_step'])"
for wl in grid grid-gradient; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --no-scaling-base > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$wl.json'));print('$wl value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['kernel'],d['roofline']['frac'],'stage1',d['stage1_roofline']['frac'],'cpu',d['cpu_baseline'] and d['cpu_baseline']['value'])"
done
timeout -k 10 300 python3 -u tools/emu_native.py 26 8 3 > "$OUT/emu_native_s26_w8.txt" 2>&1 || { echo "emu failed"; tail -20 "$OUT/emu_native_s26_w8.txt"; exit 1; }
cat "$OUT/emu_native_s26_w8.txt"
