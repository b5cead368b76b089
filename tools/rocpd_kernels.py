#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 rocpd database (run_results.db, the
ROCm 7 default output): for each kernel, launches, average of the last
`last` launches (the timed / calibration ones) and of all launches, in ms.
usage: rocpd_kernels.py run_results.db [last] [out.csv]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    db, last = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    q = (f"select s.kernel_name, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id order by d.start")
    runs = defaultdict(list)
    for name, s, e in con.execute(q):
        runs[name].append((e - s) / 1e6)
    rows = []
    for name, ds in sorted(runs.items(), key=lambda kv: -sum(kv[1][-last:])):
        t = ds[-last:]
        rows.append((name[:90], len(ds), round(sum(t) / len(t), 4), round(sum(ds) / len(ds), 4)))
    for r in rows:
        print(f"{r[2]:9.4f} ms (last {min(last, r[1])}) {r[3]:9.4f} ms (all {r[1]})  {r[0]}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "LastAverageMs", "AllAverageMs"])
            w.writerows(rows)


if __name__ == "__main__":
    main()
