"""Host-buffer C2 (gv_verify_digests_bits from pageable numpy arrays, 1M items)
against the pipeline options: pipe_chunk (first chunk), pipe_growth and
stage_threads; the device-resident rate of the same batch beside it.  Prints
one JSON line.  usage: host_sweep.py [reps]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    n = 1_000_000
    pub, sig, dig, exp = bench.make_digest_workload(n, 0xC2, 65536, 0.0, 16)
    ver = gvm.Verifier([0])
    d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
    for p, a in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, a)
    bits = ver.dev_alloc(n // 8 + 64)
    ver.dev_verify_digests(0, n, d[0], d[1], d[2], bits)
    ver.dev_sync()
    t = time.perf_counter()
    for _ in range(reps):
        ver.dev_verify_digests(0, n, d[0], d[1], d[2], bits)
    ver.dev_sync()
    dev = n * reps / (time.perf_counter() - t)
    out = {"device_resident": round(dev, 1), "host": []}
    cfgs = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("SWEEP", "").split()] or [
        (262144, 1, 4), (65536, 4, 8), (131072, 4, 8), (65536, 4, 12), (131072, 4, 12)]
    for chunk, growth, stage in cfgs * int(os.environ.get("SWEEP_ROUNDS", "3")):
        ver.set_option("pipe_chunk", chunk)
        ver.set_option("pipe_growth", growth)
        ver.set_option("stage_threads", stage)
        ver.verify_batch_digests_bits(pub, sig, dig)
        t = time.perf_counter()
        for _ in range(reps):
            r = ver.verify_batch_digests_bits(pub, sig, dig)
        v = n * reps / (time.perf_counter() - t)
        bad = int(np.count_nonzero(np.unpackbits(r.view(np.uint8), bitorder="little")[:n] != exp))
        row = {"pipe_chunk": chunk, "pipe_growth": growth, "stage_threads": stage, "value": round(v, 1),
               "frac_of_device": round(v / dev, 4), "mismatches": bad}
        out["host"].append(row)
        print(row, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
