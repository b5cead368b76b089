"""North-star parity (BASELINE.json: bit-exact accept/reject on 10M mixed
valid/invalid signatures), run by default under -m gpu.

GV_PARITY_MILLIONS (default 10) chunks of 1M items, seed 0x5EED00 + chunk:
the C3 adversarial mix of tools/workload (25 % invalid: high-S, r >= n,
s = 0 or 2^256-1, random x, malformed prefix, wrong message) with fresh
special cases written over random positions (tests/special_cases.py: point
at infinity, R.x in [n, p) with r = R.x - n (accept) and r = R.x (reject),
s = (n-1)/2 and (n+1)/2, small / lambda-related keys, forced (u1, u2)
exceptional additions and Booth-extreme windows, e in {0, n, n+1, 2^256-1}),
so the million-scale mix covers every acceptance and rejection rule.

Every chunk runs the throughput schedule (the headline path); one more 1M
chunk runs through the limb-sliced small-batch kernels (k_verify_lat_sl and
k_verify_lat_sl4 by pub33, k_verify_lat16_sl keyed) with the small-batch
bounds lifted, and through the resident key arena's throughput ladders (its
one-window wide tables and its k6 tables) with every key of the chunk loaded.  The GPU
bitmaps are compared in full with the verdicts known by construction, and
all special cases plus a random 20k sample per chunk with the C oracle.  A
JSON summary goes to GV_PARITY_OUT when set.  GV_PARITY_MILLIONS=0 skips.
"""
import json
import os
import sys
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MILLIONS = int(os.environ.get("GV_PARITY_MILLIONS", "10"))
SPECIAL_PER_KIND = 100


def sprinkle(rng, pub, sig, dig, exp, chunk):
    import special_cases as S
    sp, ss, sd, se, kinds = S.make(np.random.default_rng(0xC0FFEE + chunk), SPECIAL_PER_KIND)
    pos = rng.choice(len(pub), len(kinds), replace=False)
    pub[pos], sig[pos], dig[pos], exp[pos] = sp, ss, sd, se
    return pos, kinds


def check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, got):
    mism = int(np.count_nonzero(got != exp))
    idx = np.union1d(rng.choice(len(pub), 20_000, replace=False), pos)
    ref = O.verify_digests(pub[idx], sig[idx], dig[idx], threads=threads)
    mo = int(np.count_nonzero(ref != got[idx])) + int(np.count_nonzero(ref != exp[idx]))
    return mism, mo, len(idx)


@pytest.mark.gpu
@pytest.mark.skipif(MILLIONS <= 0, reason="GV_PARITY_MILLIONS=0")
def test_parity_millions():
    import bench
    import gpuverify as gvm
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    n = 1_000_000
    rng = np.random.default_rng(7)
    summary = {"chunks": [], "items": 0, "mismatch_vs_construction": 0, "oracle_checked": 0,
               "mismatch_vs_oracle": 0, "invalid": 0, "special": {}}
    t0 = time.time()
    with gvm.Verifier([0]) as ver:
        for c in range(MILLIONS + 1):
            sliced = c == MILLIONS                       # the extra chunk: small-batch kernels
            pub, sig, dig, exp = bench.make_digest_workload(n, 0x5EED00 + c, 65536, 0.25, threads)
            pos, kinds = sprinkle(rng, pub, sig, dig, exp, c)
            for k in kinds:
                summary["special"][k] = summary["special"].get(k, 0) + 1
            rec = {"seed": 0x5EED00 + c, "schedule": "throughput", "invalid": int(n - exp.sum()),
                   "special": len(kinds)}
            if not sliced:
                got = ver.verify_batch_digests(pub, sig, dig)
                rec["mismatch"], rec["oracle_mismatch"], checked = check_chunk(ver, O, rng, pub, sig, dig, exp, pos,
                                                                               threads, got)
            else:
                ver.set_option("lat_max", 1 << 30)       # every batch size through the sliced kernels
                ver.set_option("lat_sl_max", 1 << 30)
                ver.set_option("lat_rows_max", 0)        # k_verify_lat_sl
                got = ver.verify_batch_digests(pub, sig, dig)
                ver.set_option("lat_rows_max", 1 << 30)  # k_verify_lat_sl4
                gr = ver.verify_batch_digests(pub, sig, dig)
                ver.set_option("lat_rows_max", gvm.LAT_ROWS_MAX_DEFAULT)
                uniq, inv = np.unique(pub, axis=0, return_inverse=True)
                slots = ver.keys_load(np.ascontiguousarray(uniq))[inv.reshape(-1)]
                gk = ver.verify_batch_digests_keyed(np.ascontiguousarray(slots, np.uint32), sig, dig)
                ver.keys_reset()
                ver.reset_schedule()
                # the resident arena's throughput ladders on the same 1M items
                # (the node's default route): the one-window wide tables (kw)
                # and the k6 tables (kn), every key of the chunk loaded
                arena = {}
                try:
                    for wide, route in ((2, "kw"), (0, "kn")):
                        ver.set_option("keys_wide", wide)
                        sl = ver.keys_load(np.ascontiguousarray(uniq))[inv.reshape(-1)]
                        r0 = ver.route_stats()
                        arena[route] = ver.verify_batch_digests_keyed(np.ascontiguousarray(sl, np.uint32), sig, dig)
                        assert ver.route_stats()[route] > r0[route], route
                        ver.keys_reset()
                finally:
                    ver.set_option("keys_wide", 2)
                m1, o1, checked = check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, got)
                m2, o2, _ = check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, gk)
                m3, o3, _ = check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, gr)
                m4, o4, _ = check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, arena["kw"])
                m5, o5, _ = check_chunk(ver, O, rng, pub, sig, dig, exp, pos, threads, arena["kn"])
                rec.update({"schedule": "sliced pub33 (lat_sl, lat_sl4) + sliced keyed + arena kw / kn",
                            "mismatch": m1 + m2 + m3 + m4 + m5, "oracle_mismatch": o1 + o2 + o3 + o4 + o5,
                            "mismatch_pub33": m1, "mismatch_keyed": m2, "mismatch_pub33_rows": m3,
                            "mismatch_arena_kw": m4, "mismatch_arena_kn": m5})
                n_items = 5 * n
            summary["chunks"].append(rec)
            summary["items"] += n if not sliced else n_items
            summary["mismatch_vs_construction"] += rec["mismatch"]
            summary["oracle_checked"] += checked
            summary["mismatch_vs_oracle"] += rec["oracle_mismatch"]
            summary["invalid"] += rec["invalid"]
            print(f"chunk {c} ({rec['schedule']}): mismatches {rec['mismatch']}, oracle mismatches "
                  f"{rec['oracle_mismatch']}, {time.time() - t0:.0f}s", flush=True)
    summary["seconds"] = round(time.time() - t0, 1)
    out = os.environ.get("GV_PARITY_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "chunks"}))
    assert summary["mismatch_vs_construction"] == 0
    assert summary["mismatch_vs_oracle"] == 0
    assert summary["items"] >= MILLIONS * n
