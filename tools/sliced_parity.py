"""Bit-exact parity of the limb-sliced small-batch kernels at scale: M x 1M
mixed signatures (25 % invalid over the generator's six classes) forced
through k_verify_lat_sl (pub33) and k_verify_lat16_sl (keyed), each 1M batch
against the verdicts the generator constructed and a 20k sample against the C
oracle.  usage: sliced_parity.py [M] [out.json]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
import bench  # noqa: E402
import gpuverify as gvm  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    ver = gvm.Verifier([0])
    ver.set_option("lat_max", 1 << 30)
    ver.set_option("lat_sl_max", 1 << 30)
    res = {"items_per_schedule": m * 1_000_000, "chunks": []}
    tot = {"pub33": 0, "keyed": 0, "oracle": 0, "invalid": 0}
    t0 = time.time()
    for c in range(m):
        pub, sig, dig, exp = bench.make_digest_workload(1_000_000, 0x5100 + c, 65536, 0.25, 16)
        got = ver.verify_batch_digests(pub, sig, dig)
        mp = int(np.count_nonzero(got != exp))
        uniq, inv = np.unique(pub, axis=0, return_inverse=True)
        slots = ver.keys_load(uniq)[inv.reshape(-1)]
        gk = ver.verify_batch_digests_keyed(slots, sig, dig)
        mk = int(np.count_nonzero(gk != exp))
        ver.keys_reset()
        idx = np.random.default_rng(c).choice(1_000_000, 20000, replace=False)
        mo = int(np.count_nonzero(O.verify_digests(pub[idx], sig[idx], dig[idx], threads=16) != exp[idx]))
        inval = int(np.count_nonzero(exp == 0))
        res["chunks"].append({"seed": 0x5100 + c, "mismatch_pub33": mp, "mismatch_keyed": mk, "mismatch_oracle_sample": mo,
                              "invalid": inval})
        tot["pub33"] += mp; tot["keyed"] += mk; tot["oracle"] += mo; tot["invalid"] += inval
        print(json.dumps(res["chunks"][-1]), flush=True)
    res.update({"mismatch_pub33": tot["pub33"], "mismatch_keyed": tot["keyed"], "mismatch_oracle_sample": tot["oracle"],
                "invalid": tot["invalid"], "seconds": round(time.time() - t0, 1)})
    ver.close()
    s = json.dumps(res)
    print(s)
    if out_path:
        open(out_path, "w").write(s)
    assert tot["pub33"] == 0 and tot["keyed"] == 0 and tot["oracle"] == 0


if __name__ == "__main__":
    main()
