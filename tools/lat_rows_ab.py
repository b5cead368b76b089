#!/usr/bin/env python3
"""C5 pub33 small batches: k_verify_lat_sl (lat_rows_max 0) against
k_verify_lat_sl4 (row-parallel ladders, G from the 24-bit tables): verdicts
against the generator's, end-to-end p50 of gv_verify_digests and the fused
kernel's own p50 (HIP events) per batch size.  One JSON line per kernel."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402


def p50(ts):
    return round(float(np.percentile(np.array(ts) * 1e3, 50)), 4)


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1, 16, 64, 128, 256, 512, 1024]
    pub, sig, dig, exp = bench.make_digest_workload(8192, 0xC5, 1024, 0.25, 16)
    ver = gvm.Verifier([0])
    ver.set_option("lat_sl_max", 1 << 30)
    for rows in (0, 1 << 30):
        ver.set_option("lat_rows_max", rows)
        out = {"kernel": "k_verify_lat_sl4" if rows else "k_verify_lat_sl"}
        got = ver.verify_batch_digests(pub[:2048], sig[:2048], dig[:2048])
        out["mismatches_2048"] = int(np.count_nonzero(got != exp[:2048]))
        for n in sizes:
            for _ in range(10):
                ver.verify_batch_digests(pub[:n], sig[:n], dig[:n])
            ts, ks = [], []
            for r in range(200):
                o = (r * n) % (len(pub) - n)
                t = time.perf_counter()
                ver.verify_batch_digests(pub[o:o + n], sig[o:o + n], dig[o:o + n])
                ts.append(time.perf_counter() - t)
            ver.set_option("time_kernels", 1)
            for r in range(50):
                ver.verify_batch_digests(pub[:n], sig[:n], dig[:n])
                ks.append(ver.last_stage_ms()[1] * 1e-3)
            ver.set_option("time_kernels", 0)
            out[str(n)] = {"e2e_p50_ms": p50(ts), "kernel_p50_ms": p50(ks)}
        print(json.dumps(out), flush=True)
    ver.close()


if __name__ == "__main__":
    main()
