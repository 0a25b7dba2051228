#!/bin/bash
# refresh the committed multi-rank emulations: s26 at N = 2, 4, 8 (3 reps) and the N = 8
# per-round kernel profile of the max rank
set -o pipefail
OUT=gpurun_out/${TAG:-emuref}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world $w --reps 3 > "$OUT/emu_w$w.jsonl" 2> "$OUT/emu_w$w.err" || { echo "emulate w$w failed"; tail -20 "$OUT/emu_w$w.err"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/emu_w$w.jsonl'):
    d=json.loads(l); print('w$w', 'compute %.3f ms' % d['sum_max_rank_compute_ms'], 'wire MB %.1f' % (d['wire_bytes_per_rank']/1e6), 'single %.2f' % d['single_gpu_ms'])
"
done
timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 --reps 1 --profile > "$OUT/emu_prof.jsonl" 2> "$OUT/emu_prof.err" || { echo "emulate profile failed"; tail -20 "$OUT/emu_prof.err"; exit 1; }
grep -v "amdgpu.ids" "$OUT/emu_prof.err" > "$OUT/profile.txt"; tail -3 "$OUT/profile.txt" | cut -c1-300
