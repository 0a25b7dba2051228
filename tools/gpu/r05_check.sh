#!/bin/bash
# Round 5: a selection of the GPU suite (-k "$K"), then bench lines (BENCHES) — each step under its
# own limit; a fault, abort or timeout ends the script.
set -o pipefail
OUT=gpurun_out/${TAG:-r05chk}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|134|137|139) echo "step '$2' ended with $1: stopping"; exit 1;; esac; }
if [ -n "$K" ]; then
timeout -k 10 ${KT:-600} python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1; rc=$?
fatal $rc pytest
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -25
fi
for spec in ${BENCHES:-rmat}; do
  w=${spec%%:*}; extra=""; tag=$w; [ "$spec" != "$w" ] && { extra="--scale ${spec#*:}"; tag=${w}${spec#*:}; }
  timeout -k 10 300 python3 -u bench.py --workload $w $extra --no-cpu-baseline --no-scaling-base $BARGS > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"; rc=$?
  fatal $rc bench-$tag
  [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/bench_$tag.json'));print('$tag','value',round(d['value']/1e9,3),'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'rounds',d['breakdown']['rounds'],'flags',d['breakdown']['pass_flags'])" || tail -5 "$OUT/bench_$tag.err"
done
for spec in ${ROUNDS}; do
  wl=${spec%%:*}; sc=${spec#*:}
  args="--workload $wl"; [ "$wl" = rmat ] && args="$args --scale $sc"
  timeout -k 10 240 python3 -u tools/round_profile.py $args > "$OUT/rounds_${wl}_$sc.txt" 2>&1; rc=$?
  fatal $rc rounds-$spec
  cat "$OUT/rounds_${wl}_$sc.txt"
done
python3 -c "from distributed_ghs_implementation_amd import _native; print('slot retries', _native.slot_retries())"
