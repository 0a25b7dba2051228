"""Per-dispatch timeline of the last bench step from a rocprofv3 rocpd .db (gaps = host/launch time).

    python tools/prof_timeline.py run_results.db [first-kernel-of-step-regex]
"""
import re
import sqlite3
import sys


def short(n):
    n = re.sub(r"\(.*\)$", "", n).replace("void ", "").replace("ghs::", "")
    if "rocprim" in n:
        k = re.findall(r"detail::(\w+?)_(?:config|kernel|impl)", n)
        return "rocprim:" + ("/".join(dict.fromkeys(k)) if k else n[:40])
    return n[:48]


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else r"^k_select\b(?!_)"
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if re.search(pat, r[0].replace("ghs::", ""))]
    occ = int(sys.argv[3]) if len(sys.argv) > 3 else -1  # which step (-1: the last)
    s = idx[occ]
    e = idx[occ + 1] if occ + 1 < 0 else len(rows)  # up to the next step's marker
    rows = rows[:e]
    t0 = rows[s][1]
    if s > 0:
        print(f"gap before the step's first kernel: {(rows[s][1] - rows[s - 1][2]) / 1e3:.1f} us (after {short(rows[s - 1][0])})")
    prev = t0
    busy = 0
    for r in rows[s:]:
        print(f"{(r[1] - t0) / 1e3:9.1f} gap{(r[1] - prev) / 1e3:7.1f} {r[3] / 1e3:8.1f}us {short(r[0])}")
        prev = r[2]
        busy += r[3]
    print(f"step span {(rows[-1][2] - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
