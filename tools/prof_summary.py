"""Summarise a rocprofv3 output (rocpd .db or kernel_stats.csv) into a compact per-kernel table.

    python tools/prof_summary.py gpurun_out/r01/prof/run_results.db [--steps K] > profiles/x.md
"""
import re
import sqlite3
import sys


WIDTH = 90


def short(name):
    name = re.sub(r"\(.*\)$", "", name)  # drop the argument list
    name = name.replace("void ", "").replace("ghs::", "")
    if "rocprim" in name:  # the kernel kind, not the namespace prefix
        name = re.sub(r"rocprim::ROCPRIM_\w+?_NS::", "", name)
    return name[:WIDTH]


def main():
    global WIDTH
    path = sys.argv[1]
    if "--width" in sys.argv:
        WIDTH = int(sys.argv[sys.argv.index("--width") + 1])
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"| kernel | calls | total ms | avg us | min us | max us | % |")
    print(f"|---|---|---|---|---|---|---|")
    for name, n, s, a, lo, hi in rows:
        print(f"| `{short(name)}` | {n} | {s / 1e6:.3f} | {a / 1e3:.2f} | {lo / 1e3:.2f} | {hi / 1e3:.2f} | {100 * s / tot:.1f} |")
    print(f"\ntotal kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    main()
