#!/usr/bin/env python3
"""A/B of the 6-bit-window keyed ladder (k_ecmult_k6) against k_ecmult_k4<true>
on one context, alternated, same batch (the bench's C2 workload):

  grouped   gv_dev_verify_digests over the C2 batch (keys grouped and
            tabulated inside every call): option "k6" 0 / 1
  cached    gv_dev_verify_digests_keyed over the same batch with the 65,536
            keys loaded once (bench_extras.c2_key_cache): option "keys_k6" 0 / 1

One JSON line per measurement (stdout); --reps alternations."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import bench as B  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402


def grouped(ver, d, n, steps):
    el, st = X._timed_device_runs(ver, lambda: ver.dev_verify_digests(0, n, d[0], d[1], d[2], d[3]), steps)
    return n * steps / el, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--what", default="grouped,cached")
    a = ap.parse_args()
    pub, sig, dig, exp = B.make_digest_workload(a.n, 0xC2, 65536, 0.0, B.host_cores()["effective"])
    ver = gvm.Verifier([0])
    n = a.n
    d = [ver.dev_alloc(x.nbytes) for x in (pub, sig, dig)]
    for p, x in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, x)
    nw = (n + 63) // 64
    d.append(ver.dev_alloc(nw * 8))
    what = a.what.split(",")
    for rep in range(a.reps):
        for k6 in ((0, 1) if rep % 2 == 0 else (1, 0)):
            if "grouped" in what:
                ver.set_option("k6", k6)
                r0 = ver.route_stats()
                v, st = grouped(ver, d, n, a.steps)
                r1 = ver.route_stats()
                bits = np.zeros(nw, np.uint64)
                ver.dev_download(bits, d[3])
                mm = int(np.count_nonzero(X._unpack_bits(bits, n) != exp))
                print(json.dumps({"ab": "grouped", "k6": k6, "rep": rep, "value": round(v, 1), "mismatches": mm,
                                  "routes": {k: r1[k] - r0[k] for k in r1 if r1[k] != r0[k]}, "stages": st}),
                      flush=True)
            if "cached" in what:
                ver.set_option("k6", 0)
                ver.set_option("keys_k6", k6)
                r = X.c2_key_cache(ver, pub, sig, dig, exp, 65536, steps=a.steps)
                print(json.dumps({"ab": "cached", "keys_k6": k6, "rep": rep, **r}), flush=True)
    ver.set_option("k6", 0)
    ver.set_option("keys_k6", 1)
    ver.close()


if __name__ == "__main__":
    main()
