"""The GPU path on the reference's own key data: the 1,000 fundraiser
known-answer vectors (crypto/hd/testdata/test.json, checked by
crypto/hd/fundraiser_test.go:49-88: priv -> pub33 -> address).

* Every pub33 goes through gv_keys_load (the device's ParsePubKey:
  prefix, x < p, square root, parity) into the HBM key arena; every key must
  parse and the point the arena holds (read back with gv_keys_point) must be
  priv*G from the KAT's private key -- the GPU decompression checked against
  reference-held data, not against our own oracle alone.
* Signatures made with those reference-held private keys verify on the GPU
  (both schedules, pub33 and keyed), and one flipped digest bit rejects.
"""
import json
import os

import numpy as np
import pytest

import gpuverify as gvm
from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


@pytest.fixture(scope="module")
def kat():
    vs = json.load(open(os.path.join(HERE, "golden", "fundraiser_kat.json")))["vectors"]
    assert len(vs) == 1000
    priv = np.array([np.frombuffer(bytes.fromhex(v["priv"]), np.uint8) for v in vs])
    pub = np.array([np.frombuffer(bytes.fromhex(v["pub"]), np.uint8) for v in vs])
    return priv, pub


def test_kat_keys_parse_on_gpu_to_priv_times_g(ver, kat):
    priv, pub = kat
    bad = pub[:4].copy()
    bad[0, 0] = 0x04                                   # prefix not 02/03
    bad[1, 1:] = 0xFF                                  # x >= p
    bad[2, 0] ^= 1                                     # parity flip: still a valid point (-Q)
    bad[3, 1:] = np.frombuffer(bytes.fromhex("05" * 32), np.uint8)   # x = 0x0505..: x^3 + 7 non-residue?
    ver.keys_reset()
    slots = ver.keys_load(np.concatenate([pub, bad]))
    xy, ok = ver.keys_point(slots)
    assert ok[:1000].all(), np.nonzero(ok[:1000] == 0)[0][:10]
    for i in range(1000):
        want = O.point_mul(int.from_bytes(priv[i].tobytes(), "big"))
        x = int.from_bytes(xy[i, :32].tobytes(), "big")
        y = int.from_bytes(xy[i, 32:].tobytes(), "big")
        assert (x, y) == want, i
        assert pub[i, 0] == 2 + (y & 1) and int.from_bytes(pub[i, 1:].tobytes(), "big") == x
    # the malformed keys: verdicts equal the oracle's ParsePubKey
    for j in range(4):
        want = O.parse_pubkey(bad[j].tobytes())
        assert bool(ok[1000 + j]) == (want is not None), j
        if want is not None:
            assert (int.from_bytes(xy[1000 + j, :32].tobytes(), "big"),
                    int.from_bytes(xy[1000 + j, 32:].tobytes(), "big")) == want
    ver.keys_reset()


@pytest.mark.parametrize("lat_max", [0, 1 << 30])
def test_kat_keys_sign_and_verify(ver, kat, lat_max):
    priv, pub = kat
    rng = np.random.default_rng(49)
    dig = rng.integers(0, 256, size=(1000, 32), dtype=np.uint8)
    sig = O.sign_batch(np.ascontiguousarray(priv), dig, threads=8)
    bad = dig.copy()
    bad[:, 7] ^= 0x10
    ver.set_option("lat_max", lat_max)
    try:
        assert ver.verify_batch_digests(pub, sig, dig).all()
        assert not ver.verify_batch_digests(pub, sig, bad).any()
        ver.keys_reset()
        slots = ver.keys_load(pub)
        assert ver.verify_batch_digests_keyed(slots, sig, dig).all()
        assert not ver.verify_batch_digests_keyed(slots, sig, bad).any()
        # VerifyBytes over messages (SHA-256 on the device), signed with the KAT keys
        msgs = [b'{"account_number":"%d","chain_id":"fundraiser"}' % i for i in range(1000)]
        mdig = np.array([np.frombuffer(O.sha256(m), np.uint8) for m in msgs])
        msig = O.sign_batch(np.ascontiguousarray(priv), mdig, threads=8)
        assert ver.verify_batch_msgs(pub, msig, msgs).all()
        assert ver.verify_batch_msgs_keyed(slots, msig, msgs).all()
        assert not ver.verify_batch_msgs(pub, msig, [m + b" " for m in msgs]).any()
    finally:
        ver.reset_schedule()
        ver.keys_reset()
