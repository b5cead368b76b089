"""Same-box A/B of host-mirror builds (GVH_LIB): the C1 steady block path and
the C4 multisig replay of tools/bench_extras, one JSON line per run.
usage: GVH_LIB=lib.so python tools/host_ab.py"""
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
wl = bench.workload_lib()
c1 = X.c1_ante(ver)["block_path_steady"]
c4 = X.c4_multisig(ver, wl)
print(json.dumps({"lib": os.environ.get("GVH_LIB", "default"), "c1_steady_txs_per_s": c1["txs_per_s"],
                  "c1_ms_per_block": c1["ms_per_block"], "c4_leaves_per_s": c4["leaves_per_s"],
                  "c4_preverify_s": c4["preverify_s"], "c4_ante_loop_s": c4["ante_loop_s"], "c4_gpu_s": c4["gpu_s"],
                  "mismatches": c4["mismatches"]}))
