#!/usr/bin/env python3
"""C5 keyed small batches: k_verify_lat16_kn (the arena's kn tables, keys_k6
1) against k_verify_lat16_sl (its k4 tables, keys_k6 0): verdicts against
the generator's and end-to-end / kernel p50 per batch size.  One JSON line
per kernel."""
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
    sizes = [int(x) for x in sys.argv[1:]] or [1, 64, 256, 1024]
    pub, sig, dig, exp = bench.make_digest_workload(8192, 0xC6, 1024, 0.25, 16)
    ver = gvm.Verifier([0])
    slots = ver.keys_load(pub[:1024])[np.arange(len(pub)) % 1024].astype(np.uint32)
    # items use key i % 1024 (an adversarial item's own malformed key is not
    # the slot's): the verdicts of the two kernels are compared with each other
    ref = None
    for k6 in (1, 0):
        ver.set_option("keys_k6", k6)
        out = {"kernel": "k_verify_lat16_kn" if k6 else "k_verify_lat16_sl"}
        got = ver.verify_batch_digests_keyed(slots[:1500], sig[:1500], dig[:1500])
        ref = got if ref is None else ref
        out["accepted_1500"] = int(got.sum())
        out["differs_from_kn"] = int(np.count_nonzero(got != ref))
        for n in sizes:
            for _ in range(10):
                ver.verify_batch_digests_keyed(slots[:n], sig[:n], dig[:n])
            ts, ks = [], []
            for r in range(200):
                o = (r * n) % (len(pub) - n)
                t = time.perf_counter()
                ver.verify_batch_digests_keyed(slots[o:o + n], sig[o:o + n], dig[o:o + n])
                ts.append(time.perf_counter() - t)
            ver.set_option("time_kernels", 1)
            for r in range(50):
                ver.verify_batch_digests_keyed(slots[:n], sig[:n], dig[:n])
                ks.append(ver.last_stage_ms()[1] * 1e-3)
            ver.set_option("time_kernels", 0)
            out[str(n)] = {"e2e_p50_ms": p50(ts), "kernel_p50_ms": p50(ks)}
        print(json.dumps(out), flush=True)
    ver.set_option("keys_k6", 1)
    ver.close()


if __name__ == "__main__":
    main()
