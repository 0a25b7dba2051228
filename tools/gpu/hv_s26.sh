#!/bin/bash
# heavy-edge buckets (GHS_HV) at s26, where the giant bitmap (8 MiB) no longer fits one XCD's L2:
# heavy-bucket parity, one-GPU bench A/B, then the N=8 emulation A/B
set -o pipefail
OUT=gpurun_out/${TAG:-hvs26}
mkdir -p "$OUT"
export TMPDIR=/tmp
GHS_HV=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "heavy_buckets or s26" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
TAG=${TAG:-hvs26} REPS=2 VARIANTS="off:GHS_HV=0 on:GHS_HV=1" TOPK=8 BENCH_ARGS="--scale 26 --steps 3 --warmup 1" bash tools/gpu/ab.sh || exit 1
for v in 0 1; do
  GHS_HV=$v timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 --reps 2 > "$OUT/emu_hv$v.jsonl" 2> "$OUT/emu_hv$v.err" || { echo "emulate failed"; tail -20 "$OUT/emu_hv$v.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/emu_hv$v.jsonl'):
    d=json.loads(l); print('hv$v', 'compute %.3f ms' % d['sum_max_rank_compute_ms'], [r['max_rank_ms'] for r in d['per_round']][:9])
"
done
