"""c2_hostpath A/B of runtime options on one box: 1M C2 items from pinned and
pageable caller buffers, settings alternated `reps` times.
usage: hostpath_ab4.py reps "name:opt=val,opt=val" ..."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402

reps = int(sys.argv[1])
specs = []
for a in sys.argv[2:]:
    name, _, kv = a.partition(":")
    specs.append((name, [(k, int(v)) for k, v in (x.split("=") for x in kv.split(",") if x)]))
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
ver = gvm.Verifier([0])
hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
for h, a in zip(hp, (pub, sig, dig)):
    h[...] = a
ver.verify_batch_digests_bits(*hp)
ver.verify_batch_digests_bits(pub, sig, dig)
out = []
for r in range(reps):
    for name, opts in specs:
        for k, v in opts:
            ver.set_option(k, v)
        row = {"name": name, "rep": r}
        for mode, arrs in (("pinned", hp), ("pageable", (pub, sig, dig))):
            ver.verify_batch_digests_bits(*arrs)
            t = time.perf_counter()
            for _ in range(5):
                bits = ver.verify_batch_digests_bits(*arrs)
            el = (time.perf_counter() - t) / 5
            bad = int(np.count_nonzero(bench.unpack_bits(bits, len(exp)) != exp))
            row[mode] = round(1e6 / el / 1e6, 2)
            row[mode + "_ms"] = round(el * 1e3, 3)
            row[mode + "_bad"] = bad
        print(json.dumps(row), flush=True)
        out.append(row)
        for k, v in opts:                              # back to the defaults given first
            ver.set_option(k, dict(specs[0][1]).get(k, v))
for h in hp:
    ver.host_free(h)
ver.close()
