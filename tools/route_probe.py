#!/usr/bin/env python3
"""One route of the C2 batch for rocprofv3 (kernel trace / PMC passes):
`calls` serialized device-resident calls (pipeline_dev 0, so each kernel's
duration is its own) after `warmup` calls.

  grouped  the headline route: gv_dev_verify_digests, keys grouped per call
  item     the per-item pub33 route (every key distinct: c2_unique_keys)
  keyed    the resident key arena (65,536 keys loaded once: c2_key_cache)

usage: route_probe.py MODE [items] [calls]
The workload is cached in /tmp between runs of one gpurun call."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench as B  # noqa: E402
import gpuverify as gvm  # noqa: E402


def workload(n, keys):
    path = f"/tmp/gv_route_probe_{n}_{keys}.npz"
    if os.path.exists(path):
        z = np.load(path)
        return z["pub"], z["sig"], z["dig"], z["exp"]
    pub, sig, dig, exp = B.make_digest_workload(n, 0xC2 if keys != n else 0xC2 ^ 0x5A5A, keys, 0.0,
                                                B.host_cores()["effective"])
    np.savez(path, pub=pub, sig=sig, dig=dig, exp=exp)
    return pub, sig, dig, exp


def main():
    mode = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    keys = n if mode == "item" else 65536
    pub, sig, dig, exp = workload(n, keys)
    ver = gvm.Verifier([0])
    ver.set_option("pipeline_dev", 0)
    nw = (n + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    if mode == "keyed":
        slots = ver.keys_load(pub[:keys])[np.arange(n) % keys].astype(np.uint32)
        d = [ver.dev_alloc(a.nbytes) for a in (slots, sig, dig)]
        for p, a in zip(d, (slots, sig, dig)):
            ver.dev_upload(p, a)
        run = lambda: ver.dev_verify_digests_keyed(0, n, d[0], d[1], d[2], d_bits)  # noqa: E731
    else:
        d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
        for p, a in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, a)
        run = lambda: ver.dev_verify_digests(0, n, d[0], d[1], d[2], d_bits)  # noqa: E731
    for _ in range(2):
        run()
    ver.dev_sync()
    r0 = ver.route_stats()
    for _ in range(calls):
        run()
        ver.dev_sync()
    r1 = ver.route_stats()
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    mm = int(np.count_nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[:n] != exp))
    print({"mode": mode, "items": n, "calls": calls, "mismatches": mm,
           "routes": {k: r1[k] - r0[k] for k in r1 if r1[k] != r0[k]}}, flush=True)
    ver.close()


if __name__ == "__main__":
    main()
