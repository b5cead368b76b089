"""Why the node-path lines (C1 / C4) run slower inside the full bench than in
a process of their own: run them after a chosen prefix of bench.py's extras
in the same process.  usage: interference_probe.py <prefix> ...
prefixes: none, hostpath, keycache, unique, c3, msg, all"""
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

what = sys.argv[1] if len(sys.argv) > 1 else "none"
ver = gvm.Verifier([0])
n, keys, th = 1_000_000, 65536, 16
t = time.perf_counter()
if what != "none":
    pub, sig, dig, exp = bench.make_digest_workload(n, 0xC2, keys, 0.0, th)
    steps = ["hostpath", "keycache", "unique", "c3", "msg"]
    upto = steps if what == "all" else steps[:steps.index(what) + 1]
    if "hostpath" in upto:
        X.c2_hostpath(ver, pub, sig, dig, exp)
    if "keycache" in upto:
        X.c2_key_cache(ver, pub, sig, dig, exp, keys)
    if "unique" in upto:
        X.c2_unique_keys(ver, bench.make_digest_workload, n, th)
    if "c3" in upto:
        X.c3_adversarial(ver, bench.make_digest_workload, n, th)
    if "msg" in upto:
        X.msg_path(ver, bench.workload_lib(), 500_000, th)
pre = time.perf_counter() - t
c4 = X.c4_multisig(ver, bench.workload_lib(), threads=th)
print(json.dumps({"prefix": what, "prefix_s": round(pre, 1), "c4_pipelined": c4["leaves_per_s"],
                  "c4_one_by_one": c4["one_block_at_a_time"]["leaves_per_s"], "front_s": c4["preverify_front_s"],
                  "loop_s": c4["ante_loop_s"], "gpu_s": c4["gpu_s"]}), flush=True)
ver.close()
