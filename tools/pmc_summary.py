"""Per-kernel PMC summary from rocprofv3 --pmc passes (rocpd .db files under DIR/p*/)."""
import glob
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(.*\)$", "", name).replace("void ", "").replace("ghs::", "")[:40]


def main():
    d = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    dur = defaultdict(float)
    for db in sorted(glob.glob(os.path.join(d, "p*", "*.db"))):
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        q = "select * from counters_collection"
        for row in c.execute(q):
            r = dict(zip(cols, row))
            k = short(r.get("kernel_name") or r.get("name") or "?")
            cn = r.get("counter_name")
            vals[k][cn] += float(r.get("value") or 0)
            calls[k][cn] += 1
    for k in sorted(vals):
        print(f"## {k}")
        for cn in sorted(vals[k]):
            print(f"  {cn:24s} {vals[k][cn]:16.4g}  (records {calls[k][cn]})")


if __name__ == "__main__":
    main()
