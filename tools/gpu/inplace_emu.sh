#!/bin/bash
# multi-rank parity subset, then s26 x8 emulation with / without the in-place first-round MIN
set -o pipefail
OUT=gpurun_out/${TAG:-inplemu}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q --timeout 250 --timeout-method thread -k "partitioned or native_loop or emulated or multi_gpu or stepwise or separate or rccl" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
for v in pack inplace; do
  extra=""; [ $v = pack ] && extra="--no-inplace"
  timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 --reps 2 $extra > "$OUT/$v.$rep.jsonl" 2> "$OUT/$v.$rep.err" || { echo "emulate $v failed"; tail -20 "$OUT/$v.$rep.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$v.$rep.jsonl'):
    d=json.loads(l); print('$v', 'compute %.3f ms' % d['sum_max_rank_compute_ms'], [r['max_rank_ms'] for r in d['per_round']][:9])
"
done
done
