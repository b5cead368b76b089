"""c2_hostpath alone (1M C2 items from host buffers, PCIe included: pageable
and pinned, bytes and bits), `reps` times, for the library GV_LIB names.
usage: hostpath_ab.py [reps] [steps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras  # noqa: E402
import gpuverify as gvm  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
ver = gvm.Verifier([0])
for rep in range(reps):
    r = bench_extras.c2_hostpath(ver, pub, sig, dig, exp, steps=steps)
    row = {"rep": rep, "lib": os.environ.get("GV_LIB", "default"),
           **{k: v["value"] / 1e6 for k, v in r["entry_points"].items()},
           "mismatches": sum(v["mismatches"] for v in r["entry_points"].values())}
    print(json.dumps(row), flush=True)
ver.close()
