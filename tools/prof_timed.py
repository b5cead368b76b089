"""Per-kernel durations of the TIMED launches of a profiled bench run.

rocprofv3's kernel_stats.csv averages every launch of the process, including
the warmup and the two parity launches, which run before the GPU clock has
ramped (e.g. k_ecmult 8.2-8.4 ms for those vs 7.3-7.4 ms for the timed ones).
bench.py's `roofline.kernel_ms` is the HIP-event average over the timed steps
only; this tool takes the last `steps` launches of each kernel from
run_kernel_trace.csv so the committed profile and the bench line describe the
same launches.

usage: prof_timed.py run_kernel_trace.csv steps out.csv
"""
import collections
import csv
import sys


def main():
    src, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    runs = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"]
        runs[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TimedCalls", "TimedAverageNs", "TimedMinNs", "TimedMaxNs", "AllAverageNs"])
        for name, rs in sorted(runs.items(), key=lambda kv: -sum(d for _, d in kv[1])):
            rs.sort()
            t = [d for _, d in rs[-steps:]]
            w.writerow([name, len(rs), len(t), round(sum(t) / len(t), 1), min(t), max(t),
                        round(sum(d for _, d in rs) / len(rs), 1)])
            print(name[:40], len(rs), round(sum(t) / len(t) / 1e6, 4), "ms timed")


if __name__ == "__main__":
    main()
