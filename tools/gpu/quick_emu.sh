#!/bin/bash
# Parity suite + headline bench + the s26 w8 emulation (per-rank compute of the 8-GPU run).
set -o pipefail
OUT=gpurun_out/${TAG:-qemu}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'])"
timeout -k 10 300 python3 tools/dist_emulate.py --scale ${SCALE:-26} --world ${WORLD:-8} > "$OUT/emu.jsonl" 2> "$OUT/emu.err" || { echo "emulate failed"; tail -20 "$OUT/emu.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/emu.jsonl'):
    d=json.loads(l)
    print('rep', d['rep'], 'single %.2f ms  sum max-rank compute %.2f ms  rounds %d  collective MB %.1f' % (d['single_gpu_ms'], d['sum_max_rank_compute_ms'], d['rounds'], d['collective_bytes']/1e6))
    print([r['max_rank_ms'] for r in d['per_round']])
"
