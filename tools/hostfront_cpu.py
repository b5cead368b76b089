"""Host-front timing of the mirror's block paths on the CPU, no GPU: the
mirror built at -O2 over the fake verifier (tests/sanitize: make
build/libgvhost_fake.so) with GVFAKE_TRUST=1 (every verdict true, no
verification math), so PreVerifyTxs' decode / prediction / plans / pack and
the DeliverTx loop are what is timed.  C1 steady blocks and C4 multisig
blocks, GVH_PROFILE laps on stderr.
usage: hostfront_cpu.py [c1|c4] [threads] [reps]"""
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(REPO, "tests", "sanitize", "build", "libgvhost_fake.so")
os.environ["GVH_LIB"] = FAKE
os.environ["GVFAKE_TRUST"] = "1"
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools"),
          os.path.join(REPO, "tools", "workload")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gvhost  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c4"
thr = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L = ctypes.CDLL(FAKE)
L.gvfake_open.restype = ctypes.c_void_p


class FakeVerifier:
    _ctx = ctypes.c_void_p(L.gvfake_open())


wl = bench.workload_lib()
if which == "c1":
    ntx = 10000
    W = X.c1_blocks(wl, ntx, 8, thr)

    def run():
        app = gvhost.HostApp(FakeVerifier, chain_id="gv-bench", height=1)
        app.set_threads(thr)
        for i in range(ntx):
            app.set_account(W["keys"][i][2], i, 0)
        rc, _ = app.deliver_block_blob(*W["first_blob"])
        assert rc == 0
        t = time.perf_counter()
        for b in W["later_blobs"]:
            rc, c = app.deliver_block_blob(*b)
            assert rc == 0 and (c == 0).all()
        el = time.perf_counter() - t
        st = app.stats()
        app.close()
        return ntx * len(W["later_blobs"]) / el, st
else:
    blob, offs, lens, accts, leaves = X.c4_workload(wl, 30000, 4, thr)
    n = len(offs)

    def run():
        app = gvhost.HostApp(FakeVerifier, chain_id="gv-bench", height=1)
        app.set_threads(thr)
        for addr, num in accts:
            app.set_account(addr, num, 0)
        t = time.perf_counter()
        for b0 in range(0, n, 10000):
            rc, codes = app.deliver_block_blob(blob, offs[b0:b0 + 10000], lens[b0:b0 + 10000])
            assert rc == 0 and not np.count_nonzero(codes)
        el = time.perf_counter() - t
        st = app.stats()
        app.close()
        return leaves / el, st

run()
if os.environ.get("LAPS"):
    os.environ["GVH_PROFILE"] = "1"
vals = []
for _ in range(reps):
    v, st = run()
    vals.append(v)
print(which, "threads", thr, "median %.0f per s" % statistics.median(vals), [round(v) for v in vals],
      "preverify_s %.3f loop_s %.3f" % (st["preverify_ns"] / 1e9, st["deliver_loop_ns"] / 1e9))
