"""Large-scale accept/reject parity (north star: bit-exact on 10M mixed
valid/invalid signatures).  Opt-in: set GV_PARITY_MILLIONS=10 (it signs 10M
items with OpenSSL, ~15 s per million on 16 threads).

Each million: C3 adversarial mix (25 % invalid: high-S, r >= n, s = 0 or
2^256-1, random x, malformed prefix, wrong message), seed 0x5EED00 + chunk.
The full GPU bitmap is compared with the verdicts known by construction, and a
random 50k sample per chunk with the CPU oracle as well.  With GV_PARITY_OUT set,
a JSON summary is written there.
"""
import json
import os
import sys
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MILLIONS = int(os.environ.get("GV_PARITY_MILLIONS", "0"))


@pytest.mark.gpu
@pytest.mark.skipif(MILLIONS <= 0, reason="set GV_PARITY_MILLIONS to run")
def test_parity_millions():
    import bench
    import gpuverify as gvm
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    n = 1_000_000
    ver = gvm.Verifier([0])
    rng = np.random.default_rng(7)
    summary = {"chunks": [], "items": 0, "mismatch_vs_construction": 0, "oracle_sampled": 0,
               "mismatch_vs_oracle": 0, "invalid": 0}
    t0 = time.time()
    for c in range(MILLIONS):
        pub, sig, dig, exp = bench.make_digest_workload(n, 0x5EED00 + c, 65536, 0.25, threads)
        got = ver.verify_batch_digests(pub, sig, dig)
        mism = int(np.count_nonzero(got != exp))
        idx = rng.choice(n, 50_000, replace=False)
        ref = O.verify_digests(pub[idx], sig[idx], dig[idx], threads=threads)
        mo = int(np.count_nonzero(ref != got[idx]))
        summary["chunks"].append({"seed": 0x5EED00 + c, "mismatch": mism, "oracle_mismatch": mo,
                                  "invalid": int(n - exp.sum())})
        summary["items"] += n
        summary["mismatch_vs_construction"] += mism
        summary["oracle_sampled"] += len(idx)
        summary["mismatch_vs_oracle"] += mo
        summary["invalid"] += int(n - exp.sum())
        print(f"chunk {c}: mismatches {mism}, oracle sample mismatches {mo}, {time.time() - t0:.0f}s", flush=True)
    ver.close()
    summary["seconds"] = round(time.time() - t0, 1)
    out = os.environ.get("GV_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(summary, f, indent=1)
    assert summary["mismatch_vs_construction"] == 0
    assert summary["mismatch_vs_oracle"] == 0
