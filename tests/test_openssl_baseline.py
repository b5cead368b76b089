"""The OpenSSL CPU baseline (SURVEY.md §8d "CPU timing beside it", line (iii))
gives the same verdicts as the oracle and as the workload's construction --
otherwise its timing would not be a like-for-like baseline.  CPU only."""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

WORK = os.path.join(REPO, "tools", "workload")


def _lib():
    so = os.path.join(WORK, "libgvwork.so")
    subprocess.run(["make", "-s", "-C", WORK], check=True)
    L = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    L.gvw_keys.argtypes = [ctypes.c_size_t, ctypes.c_uint64, vp, vp, ctypes.c_int]
    L.gvw_sign.argtypes = [ctypes.c_size_t, ctypes.c_uint64, ctypes.c_size_t, vp, vp, vp, vp, ctypes.c_double,
                           vp, vp, vp, vp, ctypes.c_int]
    L.gvw_openssl_verify.argtypes = [ctypes.c_size_t, vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
    L.gvw_msgsend_signbytes.restype = ctypes.c_longlong
    L.gvw_msgsend_signbytes.argtypes = [ctypes.c_size_t, vp, ctypes.c_size_t, ctypes.c_uint64, vp, ctypes.c_size_t,
                                        vp, vp]
    L.gvw_sha256_msgs.argtypes = [ctypes.c_size_t, vp, vp, vp, vp]
    return L


def _keys(L, nkeys, seed):
    priv = np.zeros((nkeys, 32), np.uint8)
    pub = np.zeros((nkeys, 33), np.uint8)
    L.gvw_keys(nkeys, seed, priv.ctypes.data, pub.ctypes.data, 4)
    return priv, pub


def test_openssl_digest_verdicts_match_oracle_and_construction():
    L = _lib()
    n = 3000
    priv, pubk = _keys(L, 37, 0x55)
    pub = np.zeros((n, 33), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    dig = np.zeros((n, 32), np.uint8)
    exp = np.zeros(n, np.uint8)
    L.gvw_sign(n, 0x55, 37, priv.ctypes.data, pubk.ctypes.data, None, None, 0.3, pub.ctypes.data, sig.ctypes.data,
               dig.ctypes.data, exp.ctypes.data, 4)
    got = np.zeros(n, np.uint8)
    L.gvw_openssl_verify(n, pub.ctypes.data, sig.ctypes.data, dig.ctypes.data, None, None, None, got.ctypes.data, 3)
    assert 0.6 < exp.mean() < 0.8
    assert np.array_equal(got, exp)
    assert np.array_equal(got, O.verify_digests(pub, sig, dig, threads=4))


def test_openssl_message_path_matches_oracle():
    L = _lib()
    n = 400
    priv, pubk = _keys(L, n, 0xC1)
    cap = n * 512
    blob = np.zeros(cap, np.uint8)
    off = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    total = L.gvw_msgsend_signbytes(n, pubk.ctypes.data, n, 0, blob.ctypes.data, cap, off.ctypes.data,
                                    ln.ctypes.data)
    assert total > 0
    mdig = np.zeros((n, 32), np.uint8)
    L.gvw_sha256_msgs(n, blob.ctypes.data, off.ctypes.data, ln.ctypes.data, mdig.ctypes.data)
    pub = np.zeros((n, 33), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    dig = np.zeros((n, 32), np.uint8)
    exp = np.zeros(n, np.uint8)
    L.gvw_sign(n, 0xC1, n, priv.ctypes.data, pubk.ctypes.data, None, mdig.ctypes.data, 0.2, pub.ctypes.data,
               sig.ctypes.data, dig.ctypes.data, exp.ctypes.data, 4)
    # the workload's "wrong message" mutation flips a bit of the digest, not of
    # the message, so verifying the messages accepts those items again:
    # construction gives a lower bound, the oracle the exact verdicts
    got = np.zeros(n, np.uint8)
    L.gvw_openssl_verify(n, pub.ctypes.data, sig.ctypes.data, None, blob.ctypes.data, off.ctypes.data,
                         ln.ctypes.data, got.ctypes.data, 2)
    want = O.verify_msgs(pub, sig, blob, off, ln, threads=4)
    assert np.array_equal(got, want)
    assert want.sum() >= exp.sum()
