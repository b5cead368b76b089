#!/usr/bin/env python3
"""First calls on a fresh context (bench_extras.first_call) alone, for a
rocprofv3 --hip-trace of where the first call's extra time goes.  One JSON
line; usage: first_call_probe.py [items] [calls]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import bench as B  # noqa: E402
import bench_extras as X  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    pub, sig, dig, exp = B.make_digest_workload(n, 0xC2, 65536, 0.0, B.host_cores()["effective"])
    print(json.dumps(X.first_call(pub, sig, dig, exp, calls=calls)), flush=True)


if __name__ == "__main__":
    main()
