#!/bin/bash
# multi-rank parity subset, then the s26 xN emulation with lib/exp/base.so (HEAD) and the tree
set -o pipefail
OUT=gpurun_out/${TAG:-emuab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q --timeout 250 --timeout-method thread -k "${PYK:-partitioned or native_loop or emulated or multi_gpu or stepwise or heavy or separate}" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in base new; do
  if [ $v = base ]; then export GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so; else unset GHS_MST_LIB; fi
  timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world ${WORLD:-8} --reps 3 > "$OUT/$v.jsonl" 2> "$OUT/$v.err" || { echo "emulate $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/$v.jsonl'):
    d=json.loads(l)
    print('$v', 'rep', d['rep'], 'compute %.3f ms' % d['sum_max_rank_compute_ms'], [r['max_rank_ms'] for r in d['per_round']])
"
done
