#!/usr/bin/env python3
"""Host-path probe: synchronous vs submitted (gv_submit_digests / gv_wait)
C2 batches from pageable and pinned buffers, per-call wall times, and the
cached-key line, on one context.  One JSON line per measurement."""
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    pub, sig, dig, exp = B.make_digest_workload(n, 0xC2, 65536, 0.0, B.host_cores()["effective"])
    ver = gvm.Verifier([0])
    hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
    for h, a in zip(hp, (pub, sig, dig)):
        h[...] = a
    for label, src in (("pageable", (pub, sig, dig)), ("pinned", hp)):
        for _ in range(2):
            ver.verify_batch_digests(*src)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            ver.verify_batch_digests(*src)
            ts.append(time.perf_counter() - t)
        print(json.dumps({"mode": "sync", "buf": label, "ms": [round(x * 1e3, 3) for x in ts],
                          "rate": round(n * reps / sum(ts), 1)}), flush=True)
        for _ in range(3):                                    # warm both grouping sets
            ps = [ver.submit_digests(*src) for _ in range(2)]
            for p in ps:
                ver.wait(p)
        t0 = time.perf_counter()
        ps = [ver.submit_digests(*src) for _ in range(reps)]
        t_sub = time.perf_counter() - t0
        done = []
        for p in ps:
            out = ver.wait(p)
            done.append(time.perf_counter() - t0)
            assert np.array_equal(out, exp)
        print(json.dumps({"mode": "async", "buf": label, "submit_ms": round(t_sub * 1e3, 3),
                          "done_ms": [round(x * 1e3, 3) for x in done],
                          "rate": round(n * reps / done[-1], 1)}), flush=True)
    for h in hp:
        ver.host_free(h)
    r = X.c2_key_cache(ver, pub, sig, dig, exp, 65536, steps=20)
    print(json.dumps({"mode": "key_cache", "value": r["value"], "route": r["route"], "stages": r["stages"]}),
          flush=True)
    ver.close()


if __name__ == "__main__":
    main()
