#!/usr/bin/env python3
"""Phase breakdown of k_ed_lat_unc (uncached ed25519 small batches), built
with GV_LAT_TRACE=1 (`make ab NAME=trace DEFS=-DGV_LAT_TRACE=1`): 64
signatures over ~350-byte messages per call, median microseconds from the
block's start over blocks and repetitions.  One JSON line."""
import ctypes
import json
import os
import random
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("GV_LIB", os.path.join(REPO, "cosmos-sdk-rootchain_amd", "lib", "libgpuverify_trace.so"))
sys.path.insert(0, os.path.join(REPO, "cosmos-sdk-rootchain_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ed_openssl as OSSL  # noqa: E402
import gpuverify as gvm  # noqa: E402

MARKS = ["start", "hash_done(w0)", "A_decoded(w1)", "A_table_done(w1)", "R_decoded(w2)", "sB_done(w3)",
         "ladder_done(w0)", "end"]


def main():
    n = 64
    rng = random.Random(5)
    seeds = [rng.randbytes(32) for _ in range(n)]
    pubs = [OSSL.public_key(s) for s in seeds]
    msgs = [rng.randbytes(350) for _ in range(n)]
    sigs = [OSSL.sign(s, m) for s, m in zip(seeds, msgs)]
    pub = np.array([np.frombuffer(p, np.uint8) for p in pubs])
    sig = np.array([np.frombuffer(s, np.uint8) for s in sigs])
    ver = gvm.Verifier([0])
    ver.set_option("ed_unc_lat_max", 1 << 30)
    L = gvm._lib
    L.gv_debug_edl_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    acc = []
    for r in range(40):
        got = ver.verify_batch_ed25519(pub, sig, msgs)
        assert got.all()
        tr = np.zeros((n, 8), np.uint64)
        assert L.gv_debug_edl_trace(tr.ctypes.data, n) == 0
        t = tr.astype(np.int64)
        acc.append((t - t[:, :1]) * 0.01)
    med = np.median(np.concatenate(acc[5:]), 0)
    ver.close()
    print(json.dumps({k: round(float(v), 2) for k, v in zip(MARKS, med)}))


if __name__ == "__main__":
    main()
