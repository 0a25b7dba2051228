"""Aggregate a prof_timeline.py listing: time and launches per kernel, total gaps."""
import re
import sys
from collections import defaultdict

rows = []
for line in open(sys.argv[1]):
    m = re.match(r"\s*([\d.]+)\s+gap\s*([\d.]+)\s+([\d.]+)us\s+(.*)", line)
    if m:
        rows.append((float(m.group(1)), float(m.group(2)), float(m.group(3)), m.group(4).strip()))
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    agg[r[3]][0] += 1
    agg[r[3]][1] += r[2]
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:40s} {v[0]:4d} {v[1]:9.1f} us")
print(f"gaps {sum(r[1] for r in rows):.1f} us over {len(rows)} dispatches")
