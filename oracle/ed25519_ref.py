"""ed25519_ref.py -- TEST INFRASTRUCTURE ONLY (pure-Python restatement).

The reference's ed25519 leaf check, restated with Python big ints so the GPU
kernel family (csrc/ed_verify.hip) can be checked bit-for-bit.  Never imported
by the product path.

Where it sits in the reference: a multisig sub-key of type PubKeyEd25519 is
charged gas and then verified (x/auth/ante/sigverify.go:303-306 charges it,
ConsumeMultisignatureVerificationGas :325-338 ignores the "unsupported" error
for sub-keys, and multisig.PubKeyMultisigThreshold.VerifyBytes calls the
sub-key's VerifyBytes).  The upstream code is a dependency absent from
/root/reference (go.mod: tendermint v0.33.4; go1.14):

  tendermint v0.33.4 crypto/ed25519/ed25519.go PubKeyEd25519.VerifyBytes:
      len(sig) != 64 -> false; else ed25519.Verify(pub[:], msg, sig)
      (golang.org/x/crypto/ed25519 = go1.14 crypto/ed25519 on go >= 1.13)
  go1.14 crypto/ed25519 Verify:
      len(sig) != 64 || sig[63] & 224 != 0      -> false
      A.FromBytes(pub) fails                     -> false   (edwards25519)
      h = SHA-512(sig[:32] || pub || msg) mod L  (ScReduce)
      s = sig[32:] must be < L                   (ScMinimal)   -> else false
      R' = [h](-A) + [s]B                        (GeDoubleScalarMultVartime)
      encode(R') == sig[:32]                     (bytes.Equal on ToBytes)
  go1.14 crypto/ed25519/internal/edwards25519 ExtendedGroupElement.FromBytes:
      y = bytes mod 2^255 (bit 255 dropped, y >= p NOT rejected: arithmetic
      mod p); x = u v^3 (u v^7)^((p-5)/8), u = y^2 - 1, v = d y^2 + 1;
      v x^2 == u ok; v x^2 == -u -> x *= sqrt(-1); else fail;
      if parity(x) != bit 255: x = -x   (x = 0 with bit 255 set is accepted)

Cofactorless check: small-order / mixed-order keys behave exactly as the
group arithmetic says, and R is compared as canonical bytes (a non-canonical
R encoding in the signature is rejected).

Signing (RFC 8032 §5.1.6) is included to build fixtures; pinned by the RFC 8032
§7.1 test vectors in tests/golden/ed25519_rfc8032.json, which OpenSSL's
Ed25519 reproduces byte for byte (tests/test_ed25519_oracle.py).
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = -121665 * pow(121666, P - 2, P) % P
D2 = 2 * D % P
SQRTM1 = pow(2, (P - 1) // 4, P)
BY = 4 * pow(5, P - 2, P) % P


def _recover_x(y, sign):
    """x with the given parity for y (None if y is not on the curve)."""
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vxx = v * x * x % P
    if (vxx - u) % P != 0:
        if (vxx + u) % P != 0:
            return None
        x = x * SQRTM1 % P
    if (x & 1) != sign:
        x = (-x) % P
    return x


BX = _recover_x(BY, 0)
B = (BX, BY)
IDENT = (0, 1)


# ----------------------------------------------------------------- group law
# Extended coordinates (X, Y, Z, T), x = X/Z, y = Y/Z, x y = T/Z; the
# twisted-Edwards (a = -1) unified formulas are complete on this curve.
def _ext(p):
    x, y = p
    return (x, y, 1, x * y % P)


def _add(p, q):
    x1, y1, z1, t1 = p
    x2, y2, z2, t2 = q
    a = (y1 - x1) * (y2 - x2) % P
    b = (y1 + x1) * (y2 + x2) % P
    c = t1 * D2 % P * t2 % P
    d = 2 * z1 * z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _affine(p):
    x, y, z, _ = p
    zi = pow(z, P - 2, P)
    return (x * zi % P, y * zi % P)


def point_mul(k, pt):
    """k * pt (k >= 0) by double-and-add on extended coordinates."""
    r = _ext(IDENT)
    q = _ext(pt)
    while k:
        if k & 1:
            r = _add(r, q)
        q = _add(q, q)
        k >>= 1
    return _affine(r)


def point_add(p, q):
    return _affine(_add(_ext(p), _ext(q)))


def point_neg(p):
    return ((-p[0]) % P, p[1])


def on_curve(p):
    x, y = p
    return (-x * x + y * y - 1 - D * x * x * y * y) % P == 0


# ------------------------------------------------------------ encodings
def encode_point(p):
    """edwards25519 ToBytes: canonical y, bit 255 = parity of canonical x."""
    x, y = p
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def decode_point(b: bytes):
    """ExtendedGroupElement.FromBytes semantics (see header): None on failure."""
    assert len(b) == 32
    v = int.from_bytes(b, "little")
    y = (v & ((1 << 255) - 1)) % P
    x = _recover_x(y, v >> 255)
    return None if x is None else (x, y)


def sc_reduce(h64: bytes) -> int:
    return int.from_bytes(h64, "little") % L


# --------------------------------------------------------------- verify
def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    """tendermint PubKeyEd25519.VerifyBytes(msg, sig) on a 32-byte key."""
    if len(pub) != 32:
        raise ValueError("ed25519: bad public key length")   # go panics; PubKeyEd25519 is [32]byte
    if len(sig) != 64 or sig[63] & 224:
        return False
    a = decode_point(pub)
    if a is None:
        return False
    h = sc_reduce(hashlib.sha512(sig[:32] + pub + msg).digest())
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return False
    r = point_add(point_mul(h, point_neg(a)), point_mul(s, B))
    return encode_point(r) == sig[:32]


# ------------------------------------------------------------------ sign
def keypair(seed: bytes):
    """RFC 8032 §5.1.5: (scalar a, prefix, pub32) from a 32-byte seed."""
    hd = hashlib.sha512(seed).digest()
    a = int.from_bytes(hd[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, hd[32:], encode_point(point_mul(a, B))


def sign(seed: bytes, msg: bytes) -> bytes:
    """RFC 8032 §5.1.6 (what tendermint PrivKeyEd25519.Sign computes)."""
    a, prefix, pub = keypair(seed)
    r = sc_reduce(hashlib.sha512(prefix + msg).digest())
    rb = encode_point(point_mul(r, B))
    k = sc_reduce(hashlib.sha512(rb + pub + msg).digest())
    return rb + ((r + k * a) % L).to_bytes(32, "little")


def sign_with(a: int, pub: bytes, r: int, msg: bytes, rpoint=None) -> bytes:
    """Signature with an explicit scalar / nonce for crafted vectors: R = r B
    (+ rpoint if given), S = r + H(R||pub||msg) a mod L."""
    rp = point_mul(r, B) if rpoint is None else point_add(point_mul(r, B), rpoint)
    rb = encode_point(rp)
    k = sc_reduce(hashlib.sha512(rb + pub + msg).digest())
    return rb + ((r + k * a) % L).to_bytes(32, "little")


# ------------------------------------------------- small-order points
def small_order_points():
    """The 8 points of order dividing 8 (the torsion subgroup)."""
    pts = {IDENT, (0, P - 1)}                 # orders 1, 2
    pts.add((SQRTM1, 0))                      # order 4: (+-sqrt(-1), 0)
    pts.add(((-SQRTM1) % P, 0))
    y8 = _order8_y()                          # order 8: the halves of the order-4 points
    for yy in (y8, (-y8) % P):
        for sgn in (0, 1):
            x = _recover_x(yy, sgn)
            if x is not None:
                pts.add((x, yy))
    out = sorted(pts)
    for p in out:
        assert on_curve(p) and point_mul(8, p) == IDENT
    assert len(out) == 8
    return out


def _order8_y():
    # a point Q with 2Q = (sqrt(-1), 0): doubling on a=-1 twisted Edwards gives
    # y(2Q) = (y^2 + x^2) / (2 - y^2 - x^2) ... solve y(2Q) = 0 -> x^2 = -y^2,
    # with the curve: -x^2 + y^2 = 1 + d x^2 y^2 -> 2 y^2 = 1 - d y^4
    # -> d y^4 + 2 y^2 - 1 = 0 -> y^2 = (-1 +- sqrt(1 + d)) / d
    disc = (1 + D) % P
    s = pow(disc, (P + 3) // 8, P)
    if s * s % P != disc:
        s = s * SQRTM1 % P
    assert s * s % P == disc
    for root in (s, (-s) % P):
        y2 = (root - 1) * pow(D, P - 2, P) % P
        y = pow(y2, (P + 3) // 8, P)
        if y * y % P != y2:
            y = y * SQRTM1 % P
        if y * y % P == y2:
            return y
    raise AssertionError("no order-8 point")
