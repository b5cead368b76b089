"""secp_ref.py -- TEST INFRASTRUCTURE ONLY (pure-Python restatement).

Independent, deliberately simple (Python big ints, affine/Jacobian textbook
formulas) restatement of the reference's transaction-signature semantics.  It
is used to generate and re-check the committed golden fixtures under
tests/golden/ and to cross-check the C oracle (oracle/secp256k1_oracle.c).
Never imported by the product path.

Restated functions (reference file:line, upstream modules pinned in go.mod):
  verify_bytes      x/auth/ante/sigverify.go:210 -> tendermint v0.33.4
                    crypto/secp256k1/secp256k1_nocgo.go VerifyBytes
  parse_pubkey      btcd v0.20.1-beta btcec/pubkey.go ParsePubKey/decompressPoint
  verify_digest     go1.14 crypto/ecdsa.Verify + verifyGeneric + hashToInt,
                    btcec ScalarBaseMult/ScalarMult/Add (complete group law)
  sign              btcec signRFC6979 / nonceRFC6979 (+ low-S), tendermint Sign
  privkey_from_secret  tendermint GenPrivKeySecp256k1 (SHA256(secret) mod (n-1)) + 1
  address           tendermint PubKeySecp256k1.Address = RIPEMD160(SHA256(pub33))
                    (pinned by crypto/hd/testdata/test.json "addr")
  bech32_encode     types/address.go:222-234 (HRP "cosmos", types/address.go:34)
  std_sign_bytes    x/auth/types/stdtx.go:292-312 + types/utils.go:22-43
  msg_send_sign_bytes  x/bank/types/msgs.go:43-45 (golden msgs_test.go:61)
"""
from __future__ import annotations

import hashlib
import hmac
import json

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
HALF_N = N >> 1
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)
INF = None  # btcec represents the point at infinity as (0, 0)
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72


# ----------------------------------------------------------------- group law
def _jac_double(p):
    if p is None:
        return None
    x, y, z = p
    if y == 0:
        return None
    a = x * x % P
    b = y * y % P
    c = b * b % P
    d = 2 * ((x + b) ** 2 - a - c) % P
    e = 3 * a % P
    f = e * e % P
    x3 = (f - 2 * d) % P
    y3 = (e * (d - x3) - 8 * c) % P
    z3 = 2 * y * z % P
    return (x3, y3, z3)


def _jac_add(p, q):
    """Complete Jacobian addition (doubling on P==Q, infinity on P==-Q)."""
    if p is None:
        return q
    if q is None:
        return p
    x1, y1, z1 = p
    x2, y2, z2 = q
    z1z1 = z1 * z1 % P
    z2z2 = z2 * z2 % P
    u1 = x1 * z2z2 % P
    u2 = x2 * z1z1 % P
    s1 = y1 * z2 * z2z2 % P
    s2 = y2 * z1 * z1z1 % P
    h = (u2 - u1) % P
    r = (s2 - s1) % P
    if h == 0:
        return _jac_double(p) if r == 0 else None
    hh = h * h % P
    hhh = h * hh % P
    v = u1 * hh % P
    x3 = (r * r - hhh - 2 * v) % P
    y3 = (r * (v - x3) - s1 * hhh) % P
    z3 = z1 * z2 * h % P
    return (x3, y3, z3)


def _to_affine(p):
    if p is None:
        return None
    x, y, z = p
    zi = pow(z, P - 2, P)
    return (x * zi * zi % P, y * zi * zi * zi % P)


def _to_jac(a):
    return None if a is None else (a[0], a[1], 1)


def point_add(a, b):
    """btcec KoblitzCurve.Add on affine points (complete)."""
    return _to_affine(_jac_add(_to_jac(a), _to_jac(b)))


def point_mul(k, a):
    """k * a (double-and-add, MSB first)."""
    acc = None
    pj = _to_jac(a)
    for bit in bin(k)[2:] if k > 0 else "":
        acc = _jac_double(acc)
        if bit == "1":
            acc = _jac_add(acc, pj)
    return _to_affine(acc)


def point_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def is_on_curve(x, y):
    return (y * y - x * x * x - 7) % P == 0


# ------------------------------------------------------------ pubkey parsing
def compress(a) -> bytes:
    x, y = a
    return bytes([2 | (y & 1)]) + x.to_bytes(32, "big")


def parse_pubkey(pub: bytes):
    """btcec ParsePubKey for a compressed key; returns (x, y) or None."""
    if len(pub) != 33:
        return None  # other lengths are out of scope (amino fixes 33 bytes)
    fmt = pub[0]
    ybit = fmt & 1
    fmt &= 0xFE
    if fmt != 0x02:
        return None  # "invalid magic in compressed pubkey string"
    x = int.from_bytes(pub[1:33], "big")
    x3 = (x * x * x + 7) % P
    y = pow(x3, (P + 1) // 4, P)
    if ybit != (y & 1):
        y = P - y
    if y * y % P != x3:
        return None  # "invalid square root"
    if ybit != (y & 1):
        return None  # "ybit doesn't match oddness"
    if x >= P or y >= P:
        return None  # "pubkey X/Y parameter is >= to P"
    if not is_on_curve(x, y):
        return None
    return (x, y)


# ------------------------------------------------------------------- verify
def verify_digest(pub: bytes, sig: bytes, digest: bytes) -> bool:
    """tendermint VerifyBytes with the message already hashed (digest = sha256(msg))."""
    if len(sig) != 64:
        return False
    q = parse_pubkey(pub)
    if q is None:
        return False
    r = int.from_bytes(sig[:32], "big")
    s = int.from_bytes(sig[32:], "big")
    if s > HALF_N:
        return False  # tendermint low-S rule
    if r <= 0 or s <= 0 or r >= N or s >= N:
        return False  # crypto/ecdsa.Verify range checks
    e = int.from_bytes(digest, "big")  # hashToInt: 256-bit order, no truncation
    w = pow(s, N - 2, N)
    u1 = e * w % N
    u2 = r * w % N
    p1 = point_mul(u1, G)
    p2 = point_mul(u2, q)
    R = point_add(p1, p2)
    if R is None:
        return False  # x==0 && y==0
    return R[0] % N == r


def verify_bytes(pub: bytes, msg: bytes, sig: bytes) -> bool:
    return verify_digest(pub, sig, hashlib.sha256(msg).digest())


# ----------------------------------------------------------------- signing
def _rfc6979_nonce(d: int, digest: bytes):
    x = d.to_bytes(32, "big")
    h = (int.from_bytes(digest, "big") % N).to_bytes(32, "big")
    V = b"\x01" * 32
    K = b"\x00" * 32
    K = hmac.new(K, V + b"\x00" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    K = hmac.new(K, V + b"\x01" + x + h, hashlib.sha256).digest()
    V = hmac.new(K, V, hashlib.sha256).digest()
    while True:
        V = hmac.new(K, V, hashlib.sha256).digest()
        k = int.from_bytes(V, "big")
        if 1 <= k < N:
            yield k
        K = hmac.new(K, V + b"\x00", hashlib.sha256).digest()
        V = hmac.new(K, V, hashlib.sha256).digest()


def sign_digest(d: int, digest: bytes) -> bytes:
    """btcec signRFC6979 + low-S; returns R||S (64 bytes)."""
    e = int.from_bytes(digest, "big")
    for k in _rfc6979_nonce(d, digest):
        R = point_mul(k, G)
        r = R[0] % N
        if r == 0:
            continue
        s = pow(k, N - 2, N) * (e + d * r) % N
        if s > HALF_N:
            s = N - s
        if s == 0:
            continue
        return r.to_bytes(32, "big") + s.to_bytes(32, "big")


def sign(d: int, msg: bytes) -> bytes:
    return sign_digest(d, hashlib.sha256(msg).digest())


def privkey_from_secret(secret: bytes) -> int:
    fe = int.from_bytes(hashlib.sha256(secret).digest(), "big")
    return fe % (N - 1) + 1


def pubkey(d: int) -> bytes:
    return compress(point_mul(d, G))


# --------------------------------------------------------------- RIPEMD-160
def _rol(x, n):
    return ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF


_RL = [
    list(range(16)),
    [7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8],
    [3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12],
    [1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2],
    [4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13],
]
_RR = [
    [5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12],
    [6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2],
    [15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13],
    [8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14],
    [12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11],
]
_SL = [
    [11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8],
    [7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13, 12],
    [11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5],
    [11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12],
    [9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6],
]
_SR = [
    [8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6],
    [9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13, 11],
    [9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5],
    [15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8],
    [8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11],
]
_KL = [0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E]
_KR = [0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000]


def _f(j, x, y, z):
    if j == 0:
        return x ^ y ^ z
    if j == 1:
        return (x & y) | (~x & z)
    if j == 2:
        return (x | ~y) ^ z
    if j == 3:
        return (x & z) | (y & ~z)
    return x ^ (y | ~z)


def ripemd160(data: bytes) -> bytes:
    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    msg = data + b"\x80" + b"\x00" * ((55 - len(data)) % 64) + (8 * len(data)).to_bytes(8, "little")
    for off in range(0, len(msg), 64):
        X = [int.from_bytes(msg[off + 4 * i: off + 4 * i + 4], "little") for i in range(16)]
        al, bl, cl, dl, el = h
        ar, br, cr, dr, er = h
        for j in range(5):
            for i in range(16):
                t = (al + (_f(j, bl, cl, dl) & 0xFFFFFFFF) + X[_RL[j][i]] + _KL[j]) & 0xFFFFFFFF
                t = (_rol(t, _SL[j][i]) + el) & 0xFFFFFFFF
                al, el, dl, cl, bl = el, dl, _rol(cl, 10), bl, t
                t = (ar + (_f(4 - j, br, cr, dr) & 0xFFFFFFFF) + X[_RR[j][i]] + _KR[j]) & 0xFFFFFFFF
                t = (_rol(t, _SR[j][i]) + er) & 0xFFFFFFFF
                ar, er, dr, cr, br = er, dr, _rol(cr, 10), br, t
        t = (h[1] + cl + dr) & 0xFFFFFFFF
        h[1] = (h[2] + dl + er) & 0xFFFFFFFF
        h[2] = (h[3] + el + ar) & 0xFFFFFFFF
        h[3] = (h[4] + al + br) & 0xFFFFFFFF
        h[4] = (h[0] + bl + cr) & 0xFFFFFFFF
        h[0] = t
    return b"".join(x.to_bytes(4, "little") for x in h)


def address(pub33: bytes) -> bytes:
    """tendermint PubKeySecp256k1.Address(): RIPEMD160(SHA256(pub))."""
    return ripemd160(hashlib.sha256(pub33).digest())


# ------------------------------------------------------------------- bech32
_CHARSET = "qpzry9x8gf2tvdw0s3jn54khce6mua7l"


def _polymod(values):
    gen = [0x3B6A57B2, 0x26508E6D, 0x1EA119FA, 0x3D4233DD, 0x2A1462B3]
    chk = 1
    for v in values:
        b = chk >> 25
        chk = (chk & 0x1FFFFFF) << 5 ^ v
        for i in range(5):
            chk ^= gen[i] if ((b >> i) & 1) else 0
    return chk


def bech32_encode(hrp: str, data: bytes) -> str:
    acc = bits = 0
    five = []
    for b in data:
        acc = (acc << 8) | b
        bits += 8
        while bits >= 5:
            bits -= 5
            five.append((acc >> bits) & 31)
    if bits:
        five.append((acc << (5 - bits)) & 31)
    hrp_exp = [ord(c) >> 5 for c in hrp] + [0] + [ord(c) & 31 for c in hrp]
    pm = _polymod(hrp_exp + five + [0] * 6) ^ 1
    chk = [(pm >> 5 * (5 - i)) & 31 for i in range(6)]
    return hrp + "1" + "".join(_CHARSET[d] for d in five + chk)


# ---------------------------------------------------- canonical sign bytes
def sort_json(obj) -> bytes:
    """sdk.MustSortJSON: Go encoding/json with sorted keys, no whitespace,
    HTML-escaping of <, >, & (types/utils.go:22-43)."""
    s = json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=False)
    s = s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    s = s.replace("\u2028", "\\u2028").replace("\u2029", "\\u2029")
    return s.encode("utf-8")


def coins_json(coins):
    return [{"amount": str(a), "denom": d} for a, d in coins]


def msg_send_json(from_addr: bytes, to_addr: bytes, coins):
    """MsgSend amino JSON (x/bank/types/msgs.go:43-45, codec name at
    x/bank/types/codec.go:26)."""
    return {
        "type": "cosmos-sdk/MsgSend",
        "value": {
            "amount": coins_json(coins),
            "from_address": bech32_encode("cosmos", from_addr),
            "to_address": bech32_encode("cosmos", to_addr),
        },
    }


def msg_send_sign_bytes(from_addr: bytes, to_addr: bytes, coins) -> bytes:
    return sort_json(msg_send_json(from_addr, to_addr, coins))


def std_sign_bytes(chain_id: str, accnum: int, seq: int, fee_coins, gas: int, msgs_json, memo: str) -> bytes:
    """StdSignBytes (x/auth/types/stdtx.go:292-312): each msg's own sign bytes
    are embedded as raw JSON, then the whole doc is MustSortJSON'd."""
    doc = {
        "account_number": str(accnum),
        "chain_id": chain_id,
        "fee": {"amount": coins_json(fee_coins), "gas": str(gas)},
        "memo": memo,
        "msgs": msgs_json,
        "sequence": str(seq),
    }
    return sort_json(doc)
