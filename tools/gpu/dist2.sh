#!/bin/bash
# Two ranks sharing the box's one GPU (gloo): the multi-rank stepwise solve end to end, checked
# against the single-rank result of the same graph. Never the driver's 8-GPU run.
set -o pipefail
OUT=gpurun_out/${TAG:-dist2}
mkdir -p "$OUT"
S=${SCALE:-20}
timeout -k 10 200 python3 bench.py --scale $S --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/n1.json" 2> "$OUT/n1.err" || { echo "n1 failed"; tail -20 "$OUT/n1.err"; exit 1; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --backend gloo --scale $S --steps 2 --warmup 1 --no-cpu-baseline --verify-ranks > "$OUT/n2.json" 2> "$OUT/n2.err" || { echo "n2 failed"; tail -30 "$OUT/n2.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
last = lambda p: json.loads([l for l in open(p) if l.startswith("{")][-1])
a = last(o + "/n1.json"); b = last(o + "/n2.json")
print("n1", a["mst"], a["value"], "n2", b["mst"], b["value"])
assert a["mst"] == b["mst"], "N=2 MSF differs from N=1"
print("N=2 (gloo, shared GPU) == N=1")
PY
grep "ranks agree" "$OUT/n2.err"
