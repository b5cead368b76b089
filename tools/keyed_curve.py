"""Host-path keyed batches (gv_verify_digests_keyed, keys resident) per batch
size on each schedule: the limb-sliced kernel, the 16-lanes-per-signature
kernel and the keyed pipeline (k_ecmult_k4) -- where the keyed crossovers
sit (block-sized batches: C1 10k, C4 30k leaves).  usage: keyed_curve.py n1,n2,..."""
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
    sizes = [int(x) for x in sys.argv[1].split(",")]
    nmax = max(sizes)
    pub, sig, dig, exp = bench.make_digest_workload(nmax, 0xCE, 16384, 0.0, 16)
    ver = gvm.Verifier([0])
    slots = ver.keys_load(pub[:16384])[np.arange(nmax) % 16384]
    out = {}
    for n in sizes:
        row = {}
        for name, lat, slm in (("sliced", 1 << 30, 1 << 30), ("lanes16", 1 << 30, 0), ("pipeline_k4", 0, 0)):
            ver.set_option("lat_max", lat)
            ver.set_option("lat_sl_max", slm)
            got = ver.verify_batch_digests_keyed(slots[:n], sig[:n], dig[:n])
            assert np.array_equal(got, exp[:n])
            ts = []
            for r in range(12):
                t = time.perf_counter()
                ver.verify_batch_digests_keyed(slots[:n], sig[:n], dig[:n])
                ts.append(time.perf_counter() - t)
            row[name] = round(float(np.median(ts[2:])) * 1e3, 3)
        out[str(n)] = row
        print(n, row, file=sys.stderr, flush=True)
    ver.reset_schedule()
    ver.close()
    print(json.dumps({"keyed_host_path_ms": out}))


if __name__ == "__main__":
    main()
