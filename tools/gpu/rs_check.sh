#!/bin/bash
# Multi-rank checks of the reduce-scatter protocol: the multi-rank GPU tests, then the s26 x8
# emulation with the library loop's protocol (profiled) and with the all-reduce protocol.
set -o pipefail
OUT=gpurun_out/${TAG:-rs}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-partitioned or native or distributed or emulated or rank or multi or windowed}" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 tools/dist_emulate.py --scale 26 --world 8 --profile > "$OUT/emu_s26_w8_rs.jsonl" 2> "$OUT/emu_s26_w8_rs.err" || { echo "emulate rs failed"; tail -5 "$OUT/emu_s26_w8_rs.err"; exit 1; }
timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world 8 --allreduce-hooks --no-ref > "$OUT/emu_s26_w8_ar.jsonl" 2> "$OUT/emu_s26_w8_ar.err" || { echo "emulate ar failed"; tail -5 "$OUT/emu_s26_w8_ar.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
for f in ("emu_s26_w8_rs.jsonl", "emu_s26_w8_ar.jsonl"):
    for l in open(sys.argv[1] + "/" + f):
        d = json.loads(l)
        print(f, d["rep"], "single", d["single_gpu_ms"], "compute", d["sum_max_rank_compute_ms"],
              "wire MB", round(d["wire_bytes_per_rank"] / 1e6, 1), "proj", d["projected_ms_busbw_300"])
PY
tail -1 "$OUT/emu_s26_w8_rs.err"
[ -n "$ROUNDS" ] && { SPECS="$ROUNDS" TAG=${TAG:-rs} bash tools/gpu/rounds_all.sh > /dev/null || exit 1; }
exit 0
