"""GPU diagnostic: where do verdicts diverge from the oracle?"""
import os, sys, collections
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cosmos-sdk-rootchain_amd"), os.path.join(REPO, "tests")]
import gpuverify as gvm
from golden_io import load_digest_vectors
from oracle import oracle as O

pub, sig, dig, ok, cats = load_digest_vectors()
v = gvm.Verifier([0])
got = v.verify_batch_digests(pub, sig, dig)
bad = np.nonzero(got != ok)[0]
print("golden: n", len(ok), "mismatch", len(bad), collections.Counter(cats[i] for i in bad))
# same items one at a time and in different batch positions
single = np.array([v.verify_batch_digests(pub[i:i+1], sig[i:i+1], dig[i:i+1])[0] for i in bad[:20]])
print("bad items re-run alone ->", single.tolist(), "expected", ok[bad[:20]].tolist())
perm = np.random.default_rng(1).permutation(len(ok))
got2 = v.verify_batch_digests(pub[perm], sig[perm], dig[perm])
bad2 = np.nonzero(got2 != ok[perm])[0]
print("permuted batch mismatches", len(bad2), "overlap with first run:", len(set(perm[bad2]) & set(bad)))
for n in (64, 1024):
    sel = np.arange(n) % len(ok)
    g = v.verify_batch_digests(pub[sel], sig[sel], dig[sel])
    print("n", n, "mismatch", int((g != ok[sel]).sum()))
