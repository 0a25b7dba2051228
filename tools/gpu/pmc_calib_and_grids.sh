#!/bin/bash
# (1) FETCH_SIZE / WRITE_SIZE calibration on known random-gather / atomic / scatter byte counts;
# (2) HBM-traffic PMC passes for the grid workloads' kernels; (3) the multi-rank emulation of
# config 4 (s26, N = 2 / 4 / 8). Each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-calib}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/cal_$c" -o run -- tools/microbench/fetch_calib > "$OUT/cal_$c.txt" 2>&1 || { echo "calib $c failed"; tail -5 "$OUT/cal_$c.txt"; exit 1; }
done
python3 - "$OUT" <<'PY'
import glob, os, sqlite3, sys, json
o = sys.argv[1]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for db in glob.glob(os.path.join(o, "cal_" + c, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        for name, v in con.execute("select kernel_name, sum(value) from counters_collection where counter_name = ? group by dispatch_id", (c,)):
            res.setdefault(name.split("(")[0].replace("void ", ""), {})[c] = v * 1024.0
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(o, "calib.json"), "w"), indent=1)
PY
grep expect "$OUT/cal_FETCH_SIZE.txt"
for wl in grid grid-gradient; do
  TAG=${TAG:-calib}/pmc_$wl KRE="k_filter|k_select|k_minedge|k_level_pass|k_win|k_jump_ident|k_hook|k_jump" WL=$wl-16384x16384 BENCH_ARGS="--workload $wl" bash tools/gpu/pmc_traffic.sh || { echo "pmc $wl failed"; exit 1; }
done
for w in 2 4 8; do
  timeout -k 10 300 python3 tools/dist_emulate.py --scale 26 --world $w > "$OUT/emu_s26_w$w.jsonl" 2> "$OUT/emu_s26_w$w.err" || { echo "emulate $w failed"; tail -5 "$OUT/emu_s26_w$w.err"; exit 1; }
done
python3 -c "
import json
for w in (2,4,8):
    for l in open('$OUT/emu_s26_w%d.jsonl' % w):
        d=json.loads(l)
        print(w, d['rep'], 'single', d['single_gpu_ms'], 'compute', d['sum_max_rank_compute_ms'], 'payload MB', round(d['collective_bytes']/1e6,1), 'wire MB/rank', round(d['wire_bytes_per_rank']/1e6,1), 'proj', d['projected_ms_busbw_300'])
"
