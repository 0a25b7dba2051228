#!/bin/bash
# Parity suite, the 2-rank gloo rehearsal (bench.py --gpus 2 on the one GPU), the s26 w8 emulation.
set -o pipefail
OUT=gpurun_out/${TAG:-distcheck}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
TAG=${TAG:-distcheck}/dist2 timeout -k 10 400 bash tools/gpu/dist2.sh || { echo "dist2 failed"; exit 1; }
timeout -k 10 300 python3 tools/dist_emulate.py --scale ${SCALE:-26} --world ${WORLD:-8} > "$OUT/emu.jsonl" 2> "$OUT/emu.err" || { echo "emulate failed"; tail -20 "$OUT/emu.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/emu.jsonl'):
    d=json.loads(l)
    print('rep', d['rep'], 'single %s ms  sum max-rank compute %.2f ms  rounds %d  collective MB %.1f' % (d['single_gpu_ms'], d['sum_max_rank_compute_ms'], d['rounds'], d['collective_bytes']/1e6))
    print([r['max_rank_ms'] for r in d['per_round']])
"
