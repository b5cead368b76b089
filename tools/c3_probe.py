#!/usr/bin/env python3
"""The C3 line of bench.py's extras alone (1M items, 25 % invalid over the
generator's six classes, 65,536 keys), one JSON line; argv[1] = steps."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402

ver = gvm.Verifier([0])
r = X.c3_adversarial(ver, bench.make_digest_workload, 1_000_000, 16, steps=int(sys.argv[1]) if len(sys.argv) > 1 else 5)
r["group_stats"] = ver.group_stats()
print(json.dumps(r), flush=True)
ver.close()
