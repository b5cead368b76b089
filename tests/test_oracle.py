"""CPU tests: pin the oracle before trusting it.

* k*G + SEC1 compression + address against the reference's own known-answer
  vectors (crypto/hd/testdata/test.json, used by crypto/hd/fundraiser_test.go:49-88).
* Canonical sign bytes against the reference's golden strings
  (x/auth/types/stdtx_test.go:53, x/bank/types/msgs_test.go:61,227).
* C oracle == pure-Python restatement on every committed golden vector.
* Both agree with OpenSSL 3 (an independent implementation) on every vector
  whose verdict does not depend on tendermint's low-S rule.
"""
import ctypes
import ctypes.util
import hashlib
import json
import os
import random

import numpy as np
import pytest

from golden_io import load_digest_vectors, load_msg_vectors
from oracle import oracle as O
from oracle import secp_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fundraiser_kat_pubkeys_and_addresses(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "fundraiser_kat.json")))["vectors"]
    assert len(kat) == 1000
    for v in kat:
        priv = bytes.fromhex(v["priv"])
        assert O.pubkey(priv).hex() == v["pub"]
        assert R.address(bytes.fromhex(v["pub"])).hex() == v["addr"]
    for v in kat[:20]:                      # pure-Python k*G too (slower)
        assert R.pubkey(int(v["priv"], 16)).hex() == v["pub"]


def test_sign_bytes_goldens(golden_dir):
    sb = json.load(open(os.path.join(golden_dir, "sign_bytes.json")))
    ms = sb["msg_send"]
    got = R.msg_send_sign_bytes(b"input", b"output", [(10, "atom")])
    assert got.decode() == ms["want"]
    mm = sb["msg_multisend"]
    j = {"type": "cosmos-sdk/MsgMultiSend", "value": {
        "inputs": [{"address": R.bech32_encode("cosmos", b"input"), "coins": R.coins_json([(10, "atom")])}],
        "outputs": [{"address": R.bech32_encode("cosmos", b"output"), "coins": R.coins_json([(10, "atom")])}]}}
    assert R.sort_json(j).decode() == mm["want"]
    st = sb["std_sign_bytes"]
    addr = R.bech32_encode("cosmos", R.address(R.pubkey(12345)))
    got = R.std_sign_bytes("1234", 3, 6, [(150, "atom")], 100000, [[addr]], "memo")
    assert got.decode() == st["want_template"] % addr


def test_c_oracle_matches_python_on_goldens():
    pub, sig, dig, ok, cats = load_digest_vectors()
    out = O.verify_digests(pub, sig, dig, threads=4)
    bad = [(i, cats[i]) for i in range(len(ok)) if out[i] != ok[i]]
    assert not bad, bad[:10]
    assert ok.sum() > 100 and (1 - ok).sum() > 100     # both verdicts well represented
    for i in range(0, len(ok), 37):                     # re-derive a sample in pure Python
        assert R.verify_digest(bytes(pub[i]), bytes(sig[i]), bytes(dig[i])) == bool(ok[i])


def test_c_oracle_message_path_on_goldens():
    pub, sig, msgs, ok, cats = load_msg_vectors()
    for i in range(len(msgs)):
        assert O.sha256(msgs[i]) == hashlib.sha256(msgs[i]).digest()
        assert O.verify_bytes(bytes(pub[i]), msgs[i], bytes(sig[i])) == bool(ok[i]), cats[i]


def test_every_rejection_class_present():
    _, _, _, ok, cats = load_digest_vectors()
    need_reject = {"high_s", "wrong_msg", "parity_flip", "bad_prefix", "r_range", "s_range",
                   "s_halfn_plus1", "x_ge_p", "x_nonresidue", "infinity", "x_in_n_p_rbig"}
    need_accept = {"valid", "s_halfn", "x_in_n_p", "small_q", "forced_uv", "digest_edge"}
    for c in need_reject:
        sel = [o for o, k in zip(ok, cats) if k == c]
        assert sel and not any(sel), c
    for c in need_accept:
        sel = [o for o, k in zip(ok, cats) if k == c]
        assert sel and all(sel), c


def test_rfc6979_signatures_deterministic_and_low_s():
    d = R.privkey_from_secret(b"rfc")
    priv = d.to_bytes(32, "big")
    assert O.privkey_from_secret(b"rfc") == priv
    for i in range(8):
        dig = hashlib.sha256(bytes([i])).digest()
        s1 = O.sign(priv, dig)
        assert s1 == R.sign_digest(d, dig) == O.sign(priv, dig)
        assert int.from_bytes(s1[32:], "big") <= R.HALF_N


# ---------------------------------------------------------------- OpenSSL
def _libcrypto():
    path = ctypes.util.find_library("crypto") or "libcrypto.so.3"
    try:
        L = ctypes.CDLL(path)
    except OSError:
        return None
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    L.EC_KEY_new_by_curve_name.restype = vp
    L.EC_KEY_new_by_curve_name.argtypes = [i32]
    L.EC_KEY_get0_group.restype = vp
    L.EC_KEY_get0_group.argtypes = [vp]
    L.EC_POINT_new.restype = vp
    L.EC_POINT_new.argtypes = [vp]
    L.EC_POINT_oct2point.argtypes = [vp, vp, ctypes.c_char_p, ctypes.c_size_t, vp]
    L.EC_KEY_set_public_key.argtypes = [vp, vp]
    L.ECDSA_SIG_new.restype = vp
    L.BN_bin2bn.restype = vp
    L.BN_bin2bn.argtypes = [ctypes.c_char_p, i32, vp]
    L.ECDSA_SIG_set0.argtypes = [vp, vp, vp]
    L.ECDSA_do_verify.argtypes = [ctypes.c_char_p, i32, vp, vp]
    L.ECDSA_SIG_free.argtypes = [vp]
    L.EC_POINT_free.argtypes = [vp]
    L.EC_KEY_free.argtypes = [vp]
    return L


def openssl_verify(L, pub, sig, dig):
    key = L.EC_KEY_new_by_curve_name(714)        # NID_secp256k1
    grp = L.EC_KEY_get0_group(key)
    pt = L.EC_POINT_new(grp)
    try:
        if L.EC_POINT_oct2point(grp, pt, bytes(pub), 33, None) != 1:
            return False
        L.EC_KEY_set_public_key(key, pt)
        s = L.ECDSA_SIG_new()
        L.ECDSA_SIG_set0(s, L.BN_bin2bn(bytes(sig[:32]), 32, None), L.BN_bin2bn(bytes(sig[32:]), 32, None))
        rc = L.ECDSA_do_verify(bytes(dig), 32, s, key)
        L.ECDSA_SIG_free(s)
        return rc == 1
    finally:
        L.EC_POINT_free(pt)
        L.EC_KEY_free(key)


def test_oracle_agrees_with_openssl():
    L = _libcrypto()
    if L is None:
        pytest.skip("libcrypto not available")
    pub, sig, dig, ok, cats = load_digest_vectors()
    n_checked = 0
    for i in range(len(ok)):
        s = int.from_bytes(bytes(sig[i][32:]), "big")
        ossl = openssl_verify(L, pub[i], sig[i], dig[i])
        # tendermint adds the low-S rule on top of plain ECDSA
        assert (ossl and s <= R.HALF_N) == bool(ok[i]), (i, cats[i])
        n_checked += 1
    rng = random.Random(7)
    privs = np.array([np.frombuffer(rng.randbytes(31).rjust(32, b"\0"), np.uint8) for _ in range(64)])
    digs = np.array([np.frombuffer(rng.randbytes(32), np.uint8) for _ in range(64)])
    pubs = O.pubkey_batch(privs)
    sigs = O.sign_batch(privs, digs)
    for i in range(64):
        assert openssl_verify(L, pubs[i], sigs[i], digs[i])
        bad = sigs[i].copy()
        bad[40] ^= 4
        assert openssl_verify(L, pubs[i], bad, digs[i]) == O.verify_digest(bytes(pubs[i]), bytes(bad), bytes(digs[i]))
    assert n_checked == len(ok)
