#!/bin/bash
# multi-rank parity subset + s26 x8 emulation with the per-round kernel profile of the max rank
set -o pipefail
OUT=gpurun_out/${TAG:-emuc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q --timeout 250 --timeout-method thread -k "${PYK:-partitioned or native_loop or emulated or multi_gpu or stepwise}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world ${WORLD:-8} --reps 1 --profile > "$OUT/emu.jsonl" 2> "$OUT/emu.err" || { echo "emulate failed"; tail -20 "$OUT/emu.err"; exit 1; }
python3 -c "
import json
for l in open('$OUT/emu.jsonl'):
    d=json.loads(l)
    print('single %.2f ms  sum max-rank compute %.3f ms  rounds %d  wire MB %.1f' % (d['single_gpu_ms'], d['sum_max_rank_compute_ms'], d['rounds'], d['wire_bytes_per_rank']/1e6))
    print([r['max_rank_ms'] for r in d['per_round']])
"
grep -v "amdgpu.ids" "$OUT/emu.err" | tail -16
