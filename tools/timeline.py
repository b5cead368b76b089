"""Timeline of a rocprofv3 kernel trace (--kernel-trace --output-format csv):
every dispatch's start / end (us, relative to the first ladder of the window)
and queue, for the steps around ladder number `--first` .. `--first + --n`.
Shows how the front kernels of step k+1 overlap step k's ladder.
Usage: python tools/timeline.py trace.csv [--ladder k_ecmult_k6] [--first 3] [--n 4]"""
import argparse
import csv
import re


def short(name):
    m = re.search(r"gv::(\w+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--ladder", default="k_ecmult_k6")
    ap.add_argument("--first", type=int, default=3)
    ap.add_argument("--n", type=int, default=4)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    lad = [r for r in rows if a.ladder in r["Kernel_Name"]]
    if len(lad) < a.first + a.n:
        raise SystemExit(f"only {len(lad)} ladder dispatches")
    t0 = int(lad[a.first]["Start_Timestamp"])
    t1 = int(lad[a.first + a.n - 1]["End_Timestamp"])
    print(f"{'kernel':32s} {'queue':>5s} {'start':>9s} {'end':>9s} {'dur':>8s}  (us; ladder {a.first}..{a.first + a.n - 1})")
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t1:
            continue
        print(f"{short(r['Kernel_Name']):32s} {r['Queue_Id']:>5s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
    gaps = [(int(lad[i + 1]["Start_Timestamp"]) - int(lad[i]["End_Timestamp"])) / 1e3 for i in range(a.first, a.first + a.n - 1)]
    per = [(int(lad[i + 1]["Start_Timestamp"]) - int(lad[i]["Start_Timestamp"])) / 1e3 for i in range(a.first, a.first + a.n - 1)]
    print("ladder start-to-start us:", [round(x, 1) for x in per], " idle gap between ladders us:", [round(x, 1) for x in gaps])


if __name__ == "__main__":
    main()
