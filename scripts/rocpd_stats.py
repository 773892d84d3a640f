#!/usr/bin/env python3
"""Kernel stats (the rocprofv3 --stats CSV columns) from a rocpd SQLite
results database: python scripts/rocpd_stats.py run_results.db [out.csv]."""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    rows = c.execute(f"select {name}, end - start from kernels").fetchall()
    agg = {}
    for n, d in rows:
        a = agg.setdefault(n, [0, 0, None, 0, []])
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
    total = sum(a[1] for a in agg.values()) or 1
    res = sorted(((n, a[0], a[1], a[1] / a[0], 100.0 * a[1] / total, a[2], a[3]) for n, a in agg.items()),
                 key=lambda r: -r[2])
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in res:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[4], 3), r[5], r[6]])


if __name__ == "__main__":
    main()
