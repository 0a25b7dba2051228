#!/bin/bash
# Round 4: the LDS tail + the global bucket-major records — their parity tests, the full GPU suite
# (failures listed, the run goes on unless a step faults or times out), the bench lines, the
# per-round profiles of R-MAT s24 and the grid, the emulated s26 x8 calls.
set -o pipefail
OUT=gpurun_out/${TAG:-r04tail}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|134|137|139) echo "step '$2' ended with $1: stopping"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "tail" > "$OUT/pytest_tail.log" 2>&1; rc=$?
fatal $rc tail-tests
grep -E "FAILED|passed|failed" "$OUT/pytest_tail.log" | tail -15
if [ -z "$QUICK" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --durations=10 -k "not tail" > "$OUT/pytest_gpu.log" 2>&1; rc=$?
fatal $rc gpu-suite
grep -E "FAILED|passed|failed" "$OUT/pytest_gpu.log" | tail -15
fi
for spec in rmat grid grid-gradient rmat:26; do
  w=${spec%%:*}; extra=""; tag=$w; [ "$spec" != "$w" ] && { extra="--scale ${spec#*:}"; tag=${w}${spec#*:}; }
  timeout -k 10 300 python3 -u bench.py --workload $w $extra --no-cpu-baseline --no-scaling-base > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"; rc=$?
  fatal $rc bench-$tag
  [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag','value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'rounds',d['breakdown']['rounds'],'flags',d['breakdown']['pass_flags'])" || tail -5 "$OUT/bench_$tag.err"
done
for spec in rmat:24 grid:0; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$OUT/rounds_${wl}_$sc.txt" 2>&1; rc=$?
  fatal $rc rounds-$spec
  cat "$OUT/rounds_${wl}_$sc.txt"
done
timeout -k 10 300 python3 -u tools/emu_native.py 26 8 4 > "$OUT/emu_native_s26_w8.txt" 2>&1; rc=$?
fatal $rc emu
cat "$OUT/emu_native_s26_w8.txt"
