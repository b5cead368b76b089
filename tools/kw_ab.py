#!/usr/bin/env python3
"""c2_key_cache with the resident arena's wide-window tables (keys_wide 1) against the
k6 tables (keys_wide 0), alternated on one context: one JSON line per run."""
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
    n = 1_000_000
    pub, sig, dig, exp = B.make_digest_workload(n, 0xC2, 65536, 0.0, B.host_cores()["effective"])
    ver = gvm.Verifier([0])
    for _ in range(reps):
        for kw in (2, 1, 0):
            ver.set_option("keys_wide", kw)
            r = X.c2_key_cache(ver, pub, sig, dig, exp, 65536, steps=20)
            print(json.dumps({"keys_wide": kw, "value": r["value"], "route": r["route"], "mismatches": r["mismatches"],
                              "keys_load_ms": r["keys_load_ms"], "ladder_ms": r["roofline"]["kernel_ms"],
                              "frac": r["roofline"]["frac"], "stages": r["stages"]}), flush=True)
    ver.set_option("keys_wide", 1)
    ver.close()


if __name__ == "__main__":
    main()
