#!/usr/bin/env python3
"""The bench's c2_hostpath extra alone (bench_extras.c2_hostpath: sync and
submitted host-buffer batches, pageable and pinned), REPS times on one
context: per-entry-point rates, one JSON line per rep.  usage:
hostpath_line.py [reps] [dev_calls]
(dev_calls: device-resident C2 calls first, as the bench's headline runs
before its c2_hostpath extra)"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench as B  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    pub, sig, dig, exp = B.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, B.host_cores()["effective"])
    ver = gvm.Verifier([0])
    dev_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    if dev_calls:
        n = len(pub)
        d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
        for p, a in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, a)
        d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
        for _ in range(dev_calls):
            ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)
        ver.dev_sync()
        for p in d + [d_bits]:
            ver.dev_free(p)
    for _ in range(reps):
        r = X.c2_hostpath(ver, pub, sig, dig, exp)
        print(json.dumps({k: (round(v["value"] / 1e6, 1), v["ms_per_call"]) for k, v in r["entry_points"].items()}),
              flush=True)
    ver.close()


if __name__ == "__main__":
    main()
