"""The ed25519 bench line alone (tools/bench_extras.ed25519), one JSON line.
usage: ed_probe.py [n] [threads]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
th = int(sys.argv[2]) if len(sys.argv) > 2 else 16
ver = gvm.Verifier([0])
print(json.dumps(X.ed25519(ver, bench.workload_lib(), n=n, threads=th)), flush=True)
ver.close()
