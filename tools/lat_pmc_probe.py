"""Driver for PMC passes over the small-batch kernels (MODE=lat in
tools/pmc_round.sh): 200 host-path calls of 64 pub33 signatures
(k_verify_lat_sl) and 200 of 64 keyed ones (k_verify_lat16_sl)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402

n = 64
pub, sig, dig, exp = bench.make_digest_workload(8192, 0xC5, 1024, 0.0, 16)
ver = gvm.Verifier([0])
slots = ver.keys_load(pub[:1024])[np.arange(len(pub)) % 1024]
for r in range(200):
    o = (r * n) % (len(pub) - n)
    assert np.array_equal(ver.verify_batch_digests(pub[o:o + n], sig[o:o + n], dig[o:o + n]), exp[o:o + n])
for r in range(200):
    o = (r * n) % (len(pub) - n)
    assert np.array_equal(ver.verify_batch_digests_keyed(slots[o:o + n], sig[o:o + n], dig[o:o + n]), exp[o:o + n])
ver.close()
print("ok")
