"""c2_hostpath (1M C2 items from host buffers, PCIe included) over the
pipeline's chunk ramp: pipe_chunk (first chunk) x pipe_growth, pageable and
pinned caller buffers, each setting alternated twice.
usage: hostpath_sweep.py [steps]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tools")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
ver = gvm.Verifier([0])
hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
for h, a in zip(hp, (pub, sig, dig)):
    h[...] = a
res = []
grid = [(131072, 4), (65536, 4), (262144, 2), (262144, 4), (131072, 2), (131072, 8), (524288, 2), (0, 1)]
for rep in range(2):
    for chunk, growth in grid:
        ver.set_option("pipe_chunk", chunk)
        ver.set_option("pipe_growth", growth)
        row = {"pipe_chunk": chunk, "pipe_growth": growth, "rep": rep}
        for name, arrs in (("pageable", (pub, sig, dig)), ("pinned", hp)):
            ver.verify_batch_digests_bits(*arrs)
            t = time.perf_counter()
            for _ in range(steps):
                r = ver.verify_batch_digests_bits(*arrs)
            el = time.perf_counter() - t
            ok = np.unpackbits(r.view(np.uint8), bitorder="little")[:len(pub)].astype(bool)
            assert np.array_equal(ok, exp.astype(bool))
            row[name] = round(len(pub) * steps / el / 1e6, 2)
        res.append(row)
        print(json.dumps(row), flush=True)
for h in hp:
    ver.host_free(h)
ver.close()
