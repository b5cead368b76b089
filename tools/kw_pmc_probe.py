#!/usr/bin/env python3
"""The resident arena's default keyed route for a PMC pass (tools/pmc_round.sh
MODE=kw): 65,536 keys loaded, then two device-resident 1M-item keyed calls
(the C2 batch by slot) on the wide-window ladder."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import bench as B  # noqa: E402
import gpuverify as gvm  # noqa: E402

n, nkeys = 1_000_000, 65536
pub, sig, dig, exp = B.make_digest_workload(n, 0xC2, nkeys, 0.0, B.host_cores()["effective"])
ver = gvm.Verifier([0])
slots = np.ascontiguousarray(ver.keys_load(pub[:nkeys])[np.arange(n) % nkeys])
d = [ver.dev_alloc(a.nbytes) for a in (slots, sig, dig)]
for p, a in zip(d, (slots, sig, dig)):
    ver.dev_upload(p, a)
d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
r0 = ver.route_stats()
for _ in range(2):
    ver.dev_verify_digests_keyed(0, n, d[0], d[1], d[2], d_bits)
ver.dev_sync()
r1 = ver.route_stats()
bits = np.zeros((n + 63) // 64, np.uint64)
ver.dev_download(bits, d_bits)
got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)
print({"route_kw": r1["kw"] - r0["kw"], "mismatches": int(np.count_nonzero(got != exp))}, flush=True)
ver.close()
