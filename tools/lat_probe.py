"""Where the CheckTx host-path latency goes (C5): end-to-end p50 of
gv_verify_digests per batch size next to the fused kernel's own duration (HIP
events, gv_last_stage_ms) and the floor of one synchronous 1-byte H2D copy.
Prints one JSON line."""
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
    pub, sig, dig, exp = bench.make_digest_workload(8192, 0xC5, 1024, 0.0, 16)
    ver = gvm.Verifier([0])
    out = {}
    d = ver.dev_alloc(64)
    one = np.zeros(1, np.uint8)
    for _ in range(20):
        ver.dev_upload(d, one)
    ts = []
    for _ in range(200):
        t = time.perf_counter()
        ver.dev_upload(d, one)
        ts.append(time.perf_counter() - t)
    out["h2d_1byte_sync_ms"] = p50(ts)
    ver.dev_free(d)
    slots = ver.keys_load(pub[:1024])[np.arange(len(pub)) % 1024]   # item i uses key i % 1024
    for n in (1, 16, 64, 256, 1024, 4096):
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
        kt, kk = [], []
        for r in range(100):
            o = (r * n) % (len(pub) - n)
            t = time.perf_counter()
            ver.verify_batch_digests_keyed(slots[o:o + n], sig[o:o + n], dig[o:o + n])
            kt.append(time.perf_counter() - t)
        ver.set_option("time_kernels", 1)
        for r in range(50):
            ver.verify_batch_digests_keyed(slots[:n], sig[:n], dig[:n])
            kk.append(ver.last_stage_ms()[1] * 1e-3)
        ver.set_option("time_kernels", 0)
        out[str(n)] = {"e2e_p50_ms": p50(ts), "fused_kernel_p50_ms": p50(ks),
                       "keyed_e2e_p50_ms": p50(kt), "keyed_kernel_p50_ms": p50(kk)}
    ver.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
