"""PreVerifyTxs host-stage timing without a GPU: a HostApp with no verifier
runs decode, sequence prediction and the plans (sign bytes, digests, leaves,
cache keys) and stops where the GPU batch would start (GVH_ENOVERIFIER).  C4
multisig blocks (tools/bench_extras.c4_workload) at several thread counts;
GVH_PROFILE=1 prints the per-stage laps.  usage: host_probe.py [block] [threads...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import ctypes  # noqa: E402

import numpy as np  # noqa: E402

import bench  # noqa: E402
import bench_extras as X  # noqa: E402
import gvhost  # noqa: E402

block = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
ths = [int(x) for x in sys.argv[2:]] or [1, 8]
na = 30000
blob, offs, lens, accts, leaves = X.c4_workload(bench.workload_lib(), na, 1, 8)
app = gvhost.HostApp(None, chain_id="gv-bench", height=1)
for addr, num in accts:
    app.set_account(addr, num, 0)
ptrs = (np.uint64(blob.ctypes.data) + offs.astype(np.uint64))[:block]
ln = np.ascontiguousarray(lens[:block], dtype=np.uint64)
PP = ctypes.POINTER(ctypes.c_char_p)
for th in ths:
    app.set_threads(th)
    for rep in range(3):
        t = time.perf_counter()
        codes = np.zeros(block, np.uint32)             # DeliverBlock's PreVerifyTxs (keep = false)
        rc = app._L.gvh_deliver_block_codes(app._app, block, ptrs.ctypes.data_as(PP),
                                            ln.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)),
                                            codes.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        el = time.perf_counter() - t
        app.cache_clear()
        print(f"{th} threads: {el * 1e3:.2f} ms for {block} txs (rc {rc})", flush=True)
