"""Per-launch HBM traffic of the bench's main kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR WORKLOAD_TAG OUT.json

FETCH_DIR / WRITE_DIR hold the rocpd .db of a `--pmc FETCH_SIZE` pass and a `--pmc WRITE_SIZE`
pass (separate runs, as the pool requires). Units: FETCH_SIZE / WRITE_SIZE are KiB. gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half of the bytes of a
wide coalesced streaming read (16 B per lane), so the fetch figure is doubled; WRITE_SIZE is exact
for 16-B streaming stores and is reported as measured (the staged compaction writes are 256-B
contiguous per wave instruction). Both raw and corrected numbers are kept.
"""
import glob
import json
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(.*\)$", "", name).replace("void ", "").replace("ghs::", "")


def per_kernel(d, counter):
    vals = defaultdict(list)
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        for name, disp, value in c.execute(
                "select kernel_name, dispatch_id, sum(value) from counters_collection where counter_name = ? "
                "group by dispatch_id", (counter,)):
            vals[short(name)].append(float(value))
    return vals


def main():
    fdir, wdir, tag, out = sys.argv[1:5]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        kernels[k] = {
            "launches_fetch_pass": len(f), "launches_write_pass": len(w),
            # one workload per profile: a kernel launched once per step must show equal launches
            # (the s26 scaling leg of bench.py is excluded by --no-scaling-base)
            "fetch_raw_min_max": [1024.0 * min(f), 1024.0 * max(f)] if f else None,
            "fetch_bytes_per_launch_raw": fb, "write_bytes_per_launch": wb,
            "fetch_bytes_per_launch": 2 * fb if fb is not None else None,
            "traffic_bytes_per_launch": (2 * fb if fb is not None else 0) + (wb or 0),
        }
    doc = {"workload": tag, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as measured; KiB -> bytes",
           "kernels": kernels}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in kernels.items():
        print(f"{k:32s} fetch {v['fetch_bytes_per_launch'] or 0:14.4g} B  write {v['write_bytes_per_launch'] or 0:14.4g} B")


if __name__ == "__main__":
    main()
