#!/usr/bin/env python3
"""c2_hostpath on one context before and after bench.py's other extras ran
beside it (first_call's second context, checktx_latency's schedule switches,
the CPU baseline's thread pools): one JSON line per pass, per-call ms of every
host entry point."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import bench as B  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402


def show(tag, r):
    print(json.dumps({"pass": tag, "ms": {k: v["ms_per_call"] for k, v in r["entry_points"].items()}}), flush=True)


def main():
    steps = sys.argv[1].split(",") if len(sys.argv) > 1 else ["first_call", "latency", "cpu"]
    n = 1_000_000
    thr = B.host_cores()["effective"]
    pub, sig, dig, exp = B.make_digest_workload(n, 0xC2, 65536, 0.0, thr)
    ver = gvm.Verifier([0])
    show("fresh", X.c2_hostpath(ver, pub, sig, dig, exp))
    show("again", X.c2_hostpath(ver, pub, sig, dig, exp))
    for s in steps:
        if s == "first_call":
            X.first_call(pub, sig, dig, exp)
        elif s == "latency":
            B.checktx_latency(ver, pub, sig, dig, thr)
        elif s == "cpu":
            B.cpu_baseline(pub, sig, dig, thr, ver)
        show("after_" + s, X.c2_hostpath(ver, pub, sig, dig, exp))
    ver.close()


if __name__ == "__main__":
    main()
