#!/bin/bash
# L2 hit/miss counts of k_filter at R-MAT s24 and s26 (one --pmc pass per scale, its own limit)
set -o pipefail
OUT=gpurun_out/${TAG:-l2hit}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sc in ${SCALES:-24 26}; do
  timeout -s KILL 240 rocprofv3 --pmc ${COUNTERS:-TCC_HIT_sum TCC_MISS_sum} --kernel-include-regex "${KRE:-k_filter}" -d "$OUT/s$sc" -o run -- python3 tools/round_profile.py --scale $sc --reps 1 ${RP_ARGS:-} > "$OUT/s$sc.txt" 2> "$OUT/s$sc.err" || { echo "pmc s$sc failed"; tail -5 "$OUT/s$sc.err"; exit 1; }
  python3 - "$OUT/s$sc" "$sc" "${COUNTERS:-TCC_HIT_sum TCC_MISS_sum}" <<'PY'
import glob, os, sqlite3, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for db in glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True):
    c = sqlite3.connect(db)
    for name, cn, disp, v in c.execute("select kernel_name, counter_name, dispatch_id, sum(value) from counters_collection "
                                       "group by kernel_name, counter_name, dispatch_id"):
        acc[name.split("(")[0][:48]][cn].append(float(v))
for k, cs in acc.items():
    parts = " ".join(f"{cn} {sum(v) / len(v):.4g}" for cn, v in sorted(cs.items()))
    h, m = cs.get("TCC_HIT_sum"), cs.get("TCC_MISS_sum")
    rate = f" rate {sum(h) / max(1.0, sum(h) + sum(m)):.3f}" if h and m else ""
    print(f"s{sys.argv[2]} {k}: per launch {parts}{rate}")
PY
  rm -rf "$OUT/s$sc"
done
