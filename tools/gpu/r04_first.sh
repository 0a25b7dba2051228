#!/bin/bash
# Round 4, first box: the GPU suite on the ABI 7 tree, the s24 bench line, the s26 x8 emulated
# calls (driver cache: reused state, host phase times). Each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-r04a}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'s1',d['stage1_roofline']['frac'],'base',d.get('scaling_base',{}).get('ms_per_step'))"
timeout -k 10 300 python3 -u tools/emu_native.py 26 8 4 > "$OUT/emu_native_s26_w8.txt" 2>&1 || { echo "emu failed"; tail -20 "$OUT/emu_native_s26_w8.txt"; exit 1; }
cat "$OUT/emu_native_s26_w8.txt"
