#!/bin/bash
# heavy-bucket passes after the edge-count guard: s25 / s26 solves with GHS_HV=1 (fall back), the
# heavy-bucket parity tests, and the s26 x8 emulation with GHS_HV=1 (ranks of 131M edges use it)
set -o pipefail
OUT=gpurun_out/${TAG:-hvguard}
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in 25 26; do GHS_HV=1 timeout -k 10 120 python3 tools/hv_check.py $s || exit 1; done
GHS_HV=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "heavy_buckets or s26 or s24_full" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
GHS_HV=1 timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 --reps 1 > "$OUT/emu.jsonl" 2> "$OUT/emu.err" || { echo "emulate failed"; tail -20 "$OUT/emu.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/emu.jsonl'):
    d=json.loads(l); print('hv1 x8', 'compute %.3f ms' % d['sum_max_rank_compute_ms'], [r['max_rank_ms'] for r in d['per_round']][:9])
"
