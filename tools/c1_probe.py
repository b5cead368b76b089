"""Per-stage timing of the C1 block path (GVH_PROFILE laps of PreVerifyTxs,
resolve and the deliver loop) over steady blocks of single-signer MsgSends.
usage: c1_probe.py [txs_per_block] [steady_blocks] [threads]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gpuverify as gvm  # noqa: E402
import gvhost  # noqa: E402

ntx = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
thr = int(sys.argv[3]) if len(sys.argv) > 3 else 16
W = X.c1_blocks(bench.workload_lib(), ntx, nb, 16)
ver = gvm.Verifier([0])
app = gvhost.HostApp(ver, chain_id="gv-bench", height=1)
app.set_threads(thr)
for i in range(ntx):
    app.set_account(W["keys"][i][2], i, 0)
rc, codes = app.deliver_block_blob(*W["first_blob"])
assert rc == 0
os.environ["GVH_PROFILE"] = "1"
t0 = time.perf_counter()
for k, b in enumerate(W["later_blobs"]):
    t = time.perf_counter()
    rc, codes = app.deliver_block_blob(*b)
    print(f"block {k + 1}: rc {rc} bad {int((codes != 0).sum())} total {(time.perf_counter() - t) * 1e3:.2f} ms",
          file=sys.stderr, flush=True)
el = time.perf_counter() - t0
print(f"steady {ntx * nb / el:.0f} tx/s over {nb} blocks", file=sys.stderr)
print(app.stats(), file=sys.stderr)
