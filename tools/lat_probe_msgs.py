"""C5 on the message path (gv_verify_msgs: SHA-256 of the StdSignBytes on the
GPU, then the small-batch kernel) -- what the Go drop-in's CheckTx calls --
next to the digest path: e2e p50 per batch size, pub33 and keyed.  Prints one
JSON line."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402


def p50(ts):
    return round(float(np.percentile(np.array(ts) * 1e3, 50)), 4)


def main():
    n_all = 4096
    pub, sig, (blob, off, ln), exp = X.c1_items(bench.workload_lib(), n_all, 16, 1024)
    ver = gvm.Verifier([0])
    if len(sys.argv) > 1:                      # lat_rows_max (0: k_verify_lat_sl for pub33)
        ver.set_option("lat_rows_max", int(sys.argv[1]))
        out0 = {"lat_rows_max": int(sys.argv[1])}
    else:
        out0 = {}
    slots = ver.keys_load(pub[:1024])[np.arange(n_all) % 1024]
    out = {**out0, "mean_msg_bytes": round(float(ln.mean()), 1)}
    for n in (1, 16, 64, 256, 1024):
        got = ver.verify_batch_msgs(pub[:n], sig[:n], (blob, off[:n], ln[:n]))
        assert np.array_equal(got, exp[:n])
        row = {}
        for label, keyed in (("msgs", False), ("msgs_keyed", True)):
            ts = []
            for r in range(205):
                o = (r * n) % (n_all - n)
                t = time.perf_counter()
                if keyed:
                    ver.verify_batch_msgs_keyed(slots[o:o + n], sig[o:o + n], (blob, off[o:o + n], ln[o:o + n]))
                else:
                    ver.verify_batch_msgs(pub[o:o + n], sig[o:o + n], (blob, off[o:o + n], ln[o:o + n]))
                ts.append(time.perf_counter() - t)
            row[label + "_e2e_p50_ms"] = p50(ts[5:])
        out[str(n)] = row
    ver.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
