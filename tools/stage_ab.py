"""Host-path staging A/B: C2 (1M digests, pageable host buffers) through one
context at several stage_threads settings, alternated.  usage: stage_ab.py [t1,t2,..]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402

ts = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,12,16").split(",")]
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
res = {t: [] for t in ts}
with gvm.Verifier([0]) as v:
    for rnd in range(3):
        for t in ts:
            v.set_option("stage_threads", t)
            v.verify_batch_digests_bits(pub, sig, dig)
            t0 = time.perf_counter()
            for _ in range(4):
                v.verify_batch_digests_bits(pub, sig, dig)
            res[t].append(round(4e6 / (time.perf_counter() - t0) / 1e6, 2))
print(json.dumps({"Mverifies_s": res, "host": bench.host_cores()}))
