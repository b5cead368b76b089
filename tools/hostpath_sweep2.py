"""c2_hostpath (1M C2 items from host buffers, grouped keys, key-ordered lanes)
over the chunk ramp (pipe_chunk x pipe_growth), pinned and pageable caller
buffers, bits output, settings alternated `reps` times.
usage: hostpath_sweep2.py [reps] [steps]"""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0xC2, 65536, 0.0, 16)
ver = gvm.Verifier([0])
hp = [ver.host_array(a.shape, a.dtype) for a in (pub, sig, dig)]
for h, a in zip(hp, (pub, sig, dig)):
    h[...] = a
grid = [(262144, 4), (262144, 1), (131072, 2), (196608, 1), (131072, 1), (65536, 2)]
for rep in range(reps):
    for chunk, growth in grid:
        ver.set_option("pipe_chunk", chunk)
        ver.set_option("pipe_growth", growth)
        row = {"pipe_chunk": chunk, "pipe_growth": growth, "rep": rep}
        for name, arrs in (("pinned", hp), ("pageable", (pub, sig, dig))):
            ver.verify_batch_digests_bits(*arrs)
            t = time.perf_counter()
            for _ in range(steps):
                r = ver.verify_batch_digests_bits(*arrs)
            el = time.perf_counter() - t
            ok = np.unpackbits(r.view(np.uint8), bitorder="little")[:len(pub)].astype(bool)
            assert np.array_equal(ok, exp.astype(bool))
            row[name] = round(len(pub) * steps / el / 1e6, 2)
        print(json.dumps(row), flush=True)
for h in hp:
    ver.host_free(h)
ver.close()
