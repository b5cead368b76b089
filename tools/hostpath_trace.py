"""Timeline of c2_hostpath calls (1M C2 items from host buffers, grouped keys):
run under `rocprofv3 --kernel-trace --memory-copy-trace`, then
`hostpath_trace.py --analyze <trace dir> <calls.json>` prints, per call, the
kernels and copies relative to the call's start (host steady clock, which is
rocprofv3's timestamp domain) and where the call's time goes.
usage: hostpath_trace.py [calls.json] [pinned|pageable] [steps]
       hostpath_trace.py --analyze DIR calls.json"""
import csv
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd")):
    sys.path.insert(0, p)


def run(out, mode, steps):
    import bench
    import gpuverify as gvm
    pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
    ver = gvm.Verifier([0])
    arrs = (pub, sig, dig)
    hp = None
    if mode == "pinned":
        hp = [ver.host_array(a.shape, a.dtype) for a in arrs]
        for h, a in zip(hp, arrs):
            h[...] = a
        arrs = hp
    ver.verify_batch_digests_bits(*arrs)                 # tables, staging ring
    ver.verify_batch_digests_bits(*arrs)
    calls = []
    for _ in range(steps):
        t0 = time.monotonic_ns()
        bits = ver.verify_batch_digests_bits(*arrs)
        t1 = time.monotonic_ns()
        calls.append((t0, t1))
    got = bench.unpack_bits(bits, len(exp))
    json.dump({"mode": mode, "calls": calls, "mismatches": int(np.count_nonzero(got != exp))}, open(out, "w"))
    print(mode, [round((b - a) / 1e6, 3) for a, b in calls], "ms; mismatches", int(np.count_nonzero(got != exp)))
    if hp:
        for h in hp:
            ver.host_free(h)
    ver.close()


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(r)
    return rows


def analyze(d, calls_file):
    cf = json.load(open(calls_file))
    ks = load(os.path.join(d, "**", "*kernel_trace.csv"))
    ms = load(os.path.join(d, "**", "*memory_copy_trace.csv"))
    ev = []
    for r in ks:
        ev.append(("K", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gv::", ""),
                   int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id", ""))))
    for r in ms:
        ev.append(("C", r.get("Direction", r.get("Operation", "copy")), int(r["Start_Timestamp"]),
                   int(r["End_Timestamp"]), r.get("Size", r.get("Bytes", ""))))
    ev.sort(key=lambda e: e[2])
    for t0, t1 in cf["calls"]:
        print(f"--- call {(t1 - t0) / 1e6:.3f} ms ({cf['mode']})")
        inside = [e for e in ev if e[2] >= t0 - 1000 and e[2] <= t1]
        agg = {}
        for kind, name, s, e, x in inside:
            key = (kind, name)
            a = agg.setdefault(key, [0, 0.0, None, None])
            a[0] += 1
            a[1] += (e - s) / 1e6
            a[2] = (s - t0) / 1e6 if a[2] is None else a[2]
            a[3] = (e - t0) / 1e6
        for (kind, name), (cnt, busy, first, last) in sorted(agg.items(), key=lambda kv: kv[1][2]):
            print(f"  {kind} {name[:34]:34s} x{cnt:<3d} busy {busy:7.3f}  first start {first:7.3f}  last end {last:7.3f}")
        lad = [e for e in inside if e[0] == "K" and "ecmult" in e[1]]
        if lad:
            print(f"  ladder window {(lad[0][2] - t0) / 1e6:.3f} .. {(lad[-1][3] - t0) / 1e6:.3f} ms; "
                  f"ladder busy {sum(e[3] - e[2] for e in lad) / 1e6:.3f} ms")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1] if len(sys.argv) > 1 else "calls.json", sys.argv[2] if len(sys.argv) > 2 else "pinned",
            int(sys.argv[3]) if len(sys.argv) > 3 else 3)
