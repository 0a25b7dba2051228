#!/bin/bash
# Parity suite, the 2-rank gloo rehearsal, then the per-rank cost of the N-GPU decomposition
# emulated on the one GPU (tools/dist_emulate.py) for the configs the driver's scaling run uses.
set -o pipefail
OUT=gpurun_out/${TAG:-distemu}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
TAG=${TAG:-distemu}/dist2 timeout -k 10 400 bash tools/gpu/dist2.sh || { echo "dist2 failed"; exit 1; }
for cfg in "25 2" "26 4" "26 8"; do
  set -- $cfg
  timeout -k 10 300 python3 tools/dist_emulate.py --scale $1 --world $2 > "$OUT/emu_s$1_w$2.jsonl" 2> "$OUT/emu_s$1_w$2.err" || { echo "emulate s$1 w$2 failed"; tail -20 "$OUT/emu_s$1_w$2.err"; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/emu_s$1_w$2.jsonl')][-1]
print('s%d w%d single %.2f ms  sum max-rank compute %.2f ms  rounds %d  collective MB %.1f' % (d['scale'], d['world'], d['single_gpu_ms'], d['sum_max_rank_compute_ms'], d['rounds'], d['collective_bytes']/1e6))
print([(r['max_rank_ms'], [(c[0][10:14], round(c[1]/1e6,1)) for c in r['collectives']]) for r in d['per_round']])
"
done
