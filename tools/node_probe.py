"""C1 and C4 node-path lines of bench.py's extras in a process of their own
(one-block-at-a-time and pipelined replay), to tell the host pipeline's own
rate from interference by the bench's earlier extras.
usage: node_probe.py [c1|c4|both] [threads]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "both"
thr = int(sys.argv[2]) if len(sys.argv) > 2 else 16
ver = gvm.Verifier([0])
out = {}
t = time.perf_counter()
if what in ("c1", "both"):
    r = X.c1_ante(ver, wl=bench.workload_lib(), threads=thr)
    out["c1"] = {k: r[k] for k in ("block_path", "block_path_steady", "replay_pipelined_steady")}
if what in ("c4", "both"):
    out["c4"] = X.c4_multisig(ver, bench.workload_lib(), threads=thr)
out["seconds"] = round(time.perf_counter() - t, 1)
ver.close()
print(json.dumps(out))
