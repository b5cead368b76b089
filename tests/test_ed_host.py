"""ed25519 kernel family on the CPU (no GPU): the oracle pinned, then the exact
device source (csrc/ed_fe29.cuh, ed_sha512.cuh, ed_scalar.cuh, ed_group.cuh)
compiled with g++ and overflow traps (tools/fe29/ed_host.cpp) checked against
the oracle.

Pins of oracle/ed25519_ref.py (go1.14 crypto/ed25519 semantics):
  * RFC 8032 §7.1 TEST 1-3 (tests/golden/ed25519_rfc8032.json): the oracle's
    keys and signatures equal the RFC bytes, and OpenSSL's Ed25519 signs the
    seeds to the same bytes;
  * OpenSSL agrees on random canonical valid / corrupted signatures.
The edge cases OpenSSL decides differently from Go (non-canonical keys, keys
of small order, x = 0 with the sign bit) rest on the restatement alone:
parity unpinned beyond the restatement for those categories.
"""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import tempfile

import pytest

import ed_openssl as OSSL
from oracle import ed25519_ref as E

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
P = E.P
B29 = 2**29 + 2**18
M29 = 2**29 - 1
PL = [(P >> (29 * i)) & M29 for i in range(9)]


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp()
    so = os.path.join(d, "ed_host.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(REPO, "tools", "fe29", "ed_host.cpp")], check=True)
    return ctypes.CDLL(so)


@pytest.fixture(scope="module")
def btab(lib):
    t = (ctypes.c_uint32 * (32 * 129 * 27))()
    lib.edh_btab(t)
    return t


def arr(v):
    return (ctypes.c_uint32 * len(v))(*v)


def val(limbs):
    return sum(x << (29 * i) for i, x in enumerate(limbs))


def words(b):
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(len(b) // 4)]


def host_verify(lib, btab, pub, msg, sig):
    mb = (ctypes.c_uint8 * max(1, len(msg)))(*msg)
    return bool(lib.edh_verify(arr(words(pub)), arr(words(sig)), mb, len(msg), btab))


# ------------------------------------------------------------ oracle pins
def test_oracle_rfc8032_and_openssl():
    vs = json.load(open(os.path.join(GOLD, "ed25519_rfc8032.json")))["vectors"]
    for v in vs:
        seed, pub, msg, sig = (bytes.fromhex(v[k]) for k in ("seed", "pub", "msg", "sig"))
        assert E.keypair(seed)[2] == pub and OSSL.public_key(seed) == pub
        assert E.sign(seed, msg) == sig and OSSL.sign(seed, msg) == sig
        assert E.verify(pub, msg, sig) and OSSL.verify(pub, msg, sig)
        assert not E.verify(pub, msg + b"\x00", sig)


def test_oracle_agrees_with_openssl_on_canonical_signatures():
    rng = random.Random(8032)
    for i in range(120):
        seed = rng.randbytes(32)
        msg = rng.randbytes(rng.randrange(0, 400))
        pub, sig = OSSL.public_key(seed), OSSL.sign(seed, msg)
        if i % 3 == 1:
            sig = bytearray(sig)
            sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(sig)
        elif i % 3 == 2:
            msg = msg + b"x"
        assert E.verify(pub, msg, sig) == OSSL.verify(pub, msg, sig), i


def test_golden_vectors_match_oracle():
    g = json.load(open(os.path.join(GOLD, "ed25519_vectors.json")))
    n = 0
    for cat, vs in g["categories"].items():
        for v in vs:
            pub, msg, sig = (bytes.fromhex(v[k]) for k in ("pub", "msg", "sig"))
            assert E.verify(pub, msg, sig) == v["ok"], (cat, v)
            n += 1
    assert n == g["count"] and n > 150
    # every category the reference semantics decide is represented, with both verdicts where possible
    cats = g["categories"]
    for c in ("pub_noncanonical", "pub_x0_sign", "small_order", "mixed_order"):
        assert any(v["ok"] for v in cats[c]) and not all(v["ok"] for v in cats[c]), c


# ------------------------------------------------ field layer (host build)
def rand_mag(rng, m, style):
    cap = m * B29
    if style == "max":
        return [cap] * 9
    if style == "p":
        return [x * m for x in PL]
    if style == "zero":
        return [0] * 9
    return [rng.randint(0, cap) for _ in range(9)]


STYLES = ["rand"] * 30 + ["max", "p", "zero"]


@pytest.mark.parametrize("ma,mb", [(1, 1), (2, 2), (1, 6), (6, 1), (2, 3), (3, 2)])
def test_e29_mul(lib, ma, mb):
    rng = random.Random(ma * 10 + mb)
    for _ in range(400):
        a, b = rand_mag(rng, ma, rng.choice(STYLES)), rand_mag(rng, mb, rng.choice(STYLES))
        r = (ctypes.c_uint32 * 9)()
        lib.edh_mul(arr(a), arr(b), r)
        assert val(r) % P == val(a) * val(b) % P and all(x <= B29 for x in r)


def test_e29_sqr_linear_words(lib):
    rng = random.Random(3)
    for _ in range(1500):
        a = rand_mag(rng, 2, rng.choice(STYLES))
        r = (ctypes.c_uint32 * 9)()
        lib.edh_sqr(arr(a), r)
        assert val(r) % P == val(a) ** 2 % P and all(x <= B29 for x in r)
        mb = rng.randint(1, 6)
        ma = rng.randint(0, 6 - mb)
        x = rand_mag(rng, ma, rng.choice(STYLES)) if ma else [0] * 9
        y = rand_mag(rng, mb, rng.choice(STYLES))
        assert lib.edh_sub(arr(x), arr(y), mb, r) == 0
        assert val(r) % P == (val(x) - val(y)) % P and all(v <= (ma + mb + 1) * B29 for v in r)
        assert lib.edh_neg(arr(y), mb, r) == 0 and val(r) % P == (-val(y)) % P
        c = rand_mag(rng, rng.randint(1, 7), rng.choice(STYLES))
        lib.edh_norm(arr(c), r)
        assert val(r) % P == val(c) % P and all(v <= B29 for v in r)
        w = (ctypes.c_uint32 * 8)()
        lib.edh_to_words(arr(c), w)
        assert sum(v << (32 * i) for i, v in enumerate(w)) == val(c) % P
    for v in [0, 1, P - 1, P, P + 5, 2**255 - 1, 2**255, 2**256 - 1] + [rng.getrandbits(256) for _ in range(300)]:
        w = [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
        r = (ctypes.c_uint32 * 9)()
        lib.edh_from_words(arr(w), r)
        assert val(r) == v & (2**255 - 1)                     # FeFromBytes: bit 255 dropped, not reduced


def test_e29_inv_pow(lib):
    rng = random.Random(4)
    for _ in range(60):
        a = rand_mag(rng, 1, "rand")
        r = (ctypes.c_uint32 * 9)()
        lib.edh_inv(arr(a), r)
        assert val(r) % P == pow(val(a) % P, P - 2, P)
        lib.edh_pow22523(arr(a), r)
        assert val(r) % P == pow(val(a) % P, (P - 5) // 8, P)


# ------------------------------------------------------ hash and scalars
def test_sha512_and_sc_reduce(lib):
    rng = random.Random(5)
    for n in list(range(0, 260, 7)) + [47, 48, 49, 111, 112, 113, 239, 240, 241, 1000]:
        pre, msg = rng.randbytes(64), rng.randbytes(n)
        mb = (ctypes.c_uint8 * max(1, n))(*msg)
        out = (ctypes.c_uint32 * 16)()
        lib.edh_sha512(arr(words(pre)), mb, n, out)
        dig = b"".join(x.to_bytes(4, "little") for x in out)
        assert dig == hashlib.sha512(pre + msg).digest(), n
        r = (ctypes.c_uint32 * 8)()
        lib.edh_sc_reduce(out, r)
        assert sum(v << (32 * i) for i, v in enumerate(r)) == int.from_bytes(dig, "little") % E.L
    for x in [0, E.L - 1, E.L, 2 * E.L, 2**512 - 1, 3 * E.L - 1] + [rng.getrandbits(512) for _ in range(300)]:
        w = [(x >> (32 * i)) & 0xFFFFFFFF for i in range(16)]
        r = (ctypes.c_uint32 * 8)()
        lib.edh_sc_reduce(arr(w), r)
        assert sum(v << (32 * i) for i, v in enumerate(r)) == x % E.L
    for s in [0, E.L - 1, E.L, E.L + 1, 2**253 - 1, 2**256 - 1]:
        w = [(s >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
        assert bool(lib.edh_sc_minimal(arr(w))) == (s < E.L), s


# ------------------------------------------------------- group + verify
def test_frombytes_matches_oracle(lib):
    rng = random.Random(6)
    encs = [E.encode_point(p) for p in E.small_order_points()]
    encs += [((y + P) | (s << 255)).to_bytes(32, "little") for y in range(19) for s in (0, 1)]
    encs += [(1 | (1 << 255)).to_bytes(32, "little"), ((P - 1) | (1 << 255)).to_bytes(32, "little")]
    encs += [rng.randbytes(32) for _ in range(60)]
    encs += [E.keypair(rng.randbytes(32))[2] for _ in range(20)]
    for enc in encs:
        want = E.decode_point(enc)
        xy = (ctypes.c_uint32 * 16)()
        ok = lib.edh_frombytes(arr(words(enc)), xy)
        assert bool(ok) == (want is not None), enc.hex()
        if want is not None:
            x = sum(v << (32 * i) for i, v in enumerate(xy[8:16]))
            assert x == want[0], enc.hex()


def test_btab_entries(lib, btab):
    for w, j in [(0, 0), (0, 1), (0, 2), (0, 128), (1, 1), (5, 77), (31, 128), (31, 1), (17, 3)]:
        base = (w * 129 + j) * 27
        ent = list(btab[base:base + 27])
        p = E.point_mul(j * 256**w, E.B)
        x, y = p
        assert val(ent[0:9]) % P == (y + x) % P
        assert val(ent[9:18]) % P == (y - x) % P
        assert val(ent[18:27]) % P == 2 * E.D * x * y % P


def test_host_verify_golden_vectors(lib, btab):
    g = json.load(open(os.path.join(GOLD, "ed25519_vectors.json")))
    for cat, vs in g["categories"].items():
        for v in vs:
            pub, msg, sig = (bytes.fromhex(v[k]) for k in ("pub", "msg", "sig"))
            assert host_verify(lib, btab, pub, msg, sig) == v["ok"], (cat, v)
    for v in json.load(open(os.path.join(GOLD, "ed25519_rfc8032.json")))["vectors"]:
        pub, msg, sig = (bytes.fromhex(v[k]) for k in ("pub", "msg", "sig"))
        assert host_verify(lib, btab, pub, msg, sig)


def test_host_verify_random_vs_oracle(lib, btab):
    rng = random.Random(7)
    for i in range(150):
        seed, msg = rng.randbytes(32), rng.randbytes(rng.randrange(0, 500))
        pub, sig = OSSL.public_key(seed), OSSL.sign(seed, msg)
        if i % 2:
            sig = bytearray(sig)
            sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(sig)
        assert host_verify(lib, btab, pub, msg, sig) == E.verify(pub, msg, sig), i
