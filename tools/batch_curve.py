"""Device-resident verify time vs batch size for both schedules (the fused
latency kernel, gv_lat.hip, and the 4-kernel throughput pipeline), to place
the "lat_max" crossover.  Prints one JSON line.  usage: batch_curve.py [reps] [n1,n2,...]"""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sizes = ([int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else
             [1024, 4096, 8192, 16384, 32768, 65536, 131072, 262144])
    nmax = max(sizes)
    pub, sig, dig, exp = bench.make_digest_workload(nmax, 0xCC, 4096, 0.0, 16)
    ver = gvm.Verifier([0])
    d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
    for p, a in zip(d, (pub, sig, dig)):
        ver.dev_upload(p, a)
    bits = ver.dev_alloc(nmax // 8 + 64)
    out = {}
    for n in sizes:
        row = {}
        for name, lat, slm in (("latency_sliced", 1 << 30, 1 << 30), ("latency_onelane", 1 << 30, 0),
                               ("throughput_pipeline", 0, 0)):
            ver.set_option("lat_max", lat)
            ver.set_option("lat_sl_max", slm)
            ver.dev_verify_digests(0, n, d[0], d[1], d[2], bits)
            ver.dev_sync()
            t = time.perf_counter()
            for _ in range(reps):
                ver.dev_verify_digests(0, n, d[0], d[1], d[2], bits)
            ver.dev_sync()
            ms = (time.perf_counter() - t) / reps * 1e3
            got = np.zeros((n + 63) // 64, np.uint64)
            ver.dev_download(got, bits)
            ok = int(np.unpackbits(got.view(np.uint8), bitorder="little")[:n].sum())
            row[name] = {"ms": round(ms, 4), "verifies_per_s": round(n / ms * 1e3, 1), "accepted": ok}
        ver.reset_schedule()
        hp, hs, hd = (np.ascontiguousarray(a[:n]) for a in (pub, sig, dig))
        ver.verify_batch_digests_bits(hp, hs, hd)
        t = time.perf_counter()
        for _ in range(reps):
            r = ver.verify_batch_digests_bits(hp, hs, hd)
        ms = (time.perf_counter() - t) / reps * 1e3
        ok = int(np.unpackbits(r.view(np.uint8), bitorder="little")[:n].sum())
        row["host_path_default"] = {"ms": round(ms, 4), "verifies_per_s": round(n / ms * 1e3, 1), "accepted": ok}
        out[str(n)] = row
        print(n, row, file=sys.stderr, flush=True)
    print(json.dumps({"batch_curve": out}))


if __name__ == "__main__":
    main()
