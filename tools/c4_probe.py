"""Per-stage timing of the C4 block path on a small multisig workload
(GVH_PROFILE laps of PreVerifyTxs + the deliver loop).  usage: c4_probe.py [accounts] [txs_per_account]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402
import gvhost  # noqa: E402

na = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
per = int(sys.argv[2]) if len(sys.argv) > 2 else 3
blob, offs, lens, accts, leaves = X.c4_workload(bench.workload_lib(), na, per, 16)
ver = gvm.Verifier([0])
app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
app.set_threads(16)
for addr, num in accts:
    app.set_account(addr, num, 0)
os.environ["GVH_PROFILE"] = "1"
for b0 in range(0, len(offs), 10000):
    t = time.perf_counter()
    rc, codes = app.deliver_block_blob(blob, offs[b0:b0 + 10000], lens[b0:b0 + 10000])
    print(f"block {b0 // 10000}: rc {rc} bad {int(np.count_nonzero(codes))} total {(time.perf_counter() - t) * 1e3:.2f} ms",
          file=sys.stderr, flush=True)
print(app.stats(), file=sys.stderr)
