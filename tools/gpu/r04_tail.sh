#!/bin/bash
# Round 4: the LDS tail — its parity tests first (a fault stops the script), then the full GPU
# suite, the bench lines and the per-round profiles of R-MAT s24 and the grid.
set -o pipefail
OUT=gpurun_out/${TAG:-r04tail}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "tail" > "$OUT/pytest_tail.log" 2>&1 || { echo "tail tests failed"; grep -E "FAILED|Error|assert" "$OUT/pytest_tail.log" | head -30; tail -40 "$OUT/pytest_tail.log"; exit 1; }
tail -2 "$OUT/pytest_tail.log"
if [ -z "$QUICK" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
fi
for w in rmat grid grid-gradient; do
  timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline --no-scaling-base > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed"; tail -30 "$OUT/bench_$w.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$w.json'));print('$w','value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'rounds',d['breakdown']['rounds'],'flags',d['breakdown']['pass_flags'])"
done
for spec in rmat:24 grid:0; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$OUT/rounds_${wl}_$sc.txt" 2>&1 || { echo "round profile $spec failed"; tail -20 "$OUT/rounds_${wl}_$sc.txt"; exit 1; }
  cat "$OUT/rounds_${wl}_$sc.txt"
done
timeout -k 10 300 python3 -u tools/emu_native.py 26 8 4 > "$OUT/emu_native_s26_w8.txt" 2>&1 || { echo "emu failed"; tail -20 "$OUT/emu_native_s26_w8.txt"; exit 1; }
cat "$OUT/emu_native_s26_w8.txt"
