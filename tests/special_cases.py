"""Fresh special-case signatures at scale, for sprinkling into the million-item
parity chunks (SURVEY.md §8c recipes, §8d C3 "sprinkled infinity and
x in [n, p) cases").  The same constructions as tests/golden/make_golden.py,
but with the C oracle's scalar multiplication so thousands per chunk take a
second; every item's verdict is known by construction and the test checks it
against the C oracle as well.  Test infrastructure only.

Kinds (accept / reject by construction):
  infinity        d = -e r^-1: u1 G + u2 Q = infinity                 reject
  x_in_n_p        R.x = n + delta (delta < p - n), r = delta          accept
  x_in_n_p_rbig   the same R, r = n + delta (>= n)                    reject
  s_halfn         s = (n-1)/2 by key recovery                         accept
  s_halfn_plus1   s = (n+1)/2                                         reject
  small_q         Q = dG, d in {1..17, 2^k, n-1, n-2, lambda, ...}    accept
  forced_uv       u1, u2 chosen (small, lambda-related, Booth extremes)
                  with Q = +-G, 2G, ...: the ladder's exceptional adds accept
  digest_edge     e in {0, n, n+1, 2^256-1}                           accept
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from oracle import oracle as O        # noqa: E402
from oracle import secp_ref as R      # noqa: E402

P, N, G, HALF_N, LAM = R.P, R.N, R.G, R.HALF_N, R.LAMBDA


def _b32(x):
    return (x % 2**256).to_bytes(32, "big")


def _lift(x, odd):
    c = (x * x * x + 7) % P
    y = pow(c, (P + 1) // 4, P)
    if y * y % P != c:
        return None
    return (x, y if (y & 1) == odd else P - y)


def _mul(k, pt=None):
    """k * pt (pt affine or None = G) with the C oracle; None = infinity"""
    k %= N
    if k == 0:
        return None
    return O.point_mul(k, R.compress(pt) if pt is not None else None)


def _add(a, b):
    return R.point_add(a, b)


def _recover(Rp, r, s, e):
    """Q = r^-1 (s R - e G): (r, s) verifies over e with key Q (R.x mod n == r)."""
    rinv = pow(r, N - 2, N)
    return _add(_mul(rinv * s, Rp), _mul(-rinv * e))


def _sig_for_uv(u1, u2, Q):
    Rp = _add(_mul(u1), _mul(u2, Q))
    if Rp is None or Rp[0] % N == 0:
        return None
    r = Rp[0] % N
    w = u2 * pow(r, N - 2, N) % N
    s = pow(w, N - 2, N)
    e = u1 * s % N
    if s > HALF_N:                # low-S: negating w negates u1 and u2, R -> -R, same x
        s = N - s
    return r, s, e


_DELTAS = None


def _deltas():
    global _DELTAS
    if _DELTAS is None:
        _DELTAS = [d for d in range(1, 20000) if N + d < P and _lift(N + d, 0) is not None]
    return _DELTAS


def make(rng: np.random.Generator, per_kind: int = 200):
    """(pub33, sig64, dig32, expected, kinds) arrays of fresh special cases."""
    rows = []

    def add(kind, pub, r, s, e, ok):
        rows.append((kind, pub, _b32(r) + _b32(s), _b32(e), ok))

    def rand_scalar(bits=256):
        return int.from_bytes(rng.bytes(32), "big") % N if bits == 256 else int(rng.integers(1, 2**min(bits, 62)))

    for _ in range(per_kind):                                   # infinity
        e = rand_scalar()
        r = rand_scalar() or 1
        d = (-e * pow(r, N - 2, N)) % N
        if d == 0:
            continue
        s = int(rng.integers(1, 2**62))
        add("infinity", R.compress(_mul(d)), r, s, e, False)
    deltas = _deltas()
    for _ in range(per_kind // 2):                              # x in [n, p)
        delta = deltas[int(rng.integers(len(deltas)))]
        Rp = _lift(N + delta, int(rng.integers(2)))
        s = rand_scalar() % HALF_N or 1
        e = rand_scalar()
        Q = _recover(Rp, delta, s, e)
        if Q is None:
            continue
        pub = R.compress(Q)
        add("x_in_n_p", pub, delta, s, e, True)
        add("x_in_n_p_rbig", pub, N + delta, s, e, False)
    for _ in range(per_kind // 4):                              # high-S boundary
        for kind, s, ok in (("s_halfn", HALF_N, True), ("s_halfn_plus1", HALF_N + 1, False)):
            Rp = _mul(rand_scalar() or 1)
            r = Rp[0] % N
            e = rand_scalar()
            Q = _recover(Rp, r, s, e)
            if Q is None:
                continue
            add(kind, R.compress(Q), r, s, e, ok)
    smalls = [1, 2, 3, 4, 7, 8, 9, 15, 16, 17, 128, 129, 255, 256, N - 1, N - 2, LAM, N - LAM, LAM * LAM % N]
    for i in range(per_kind):                                   # small / structured keys
        d = smalls[i % len(smalls)]
        dig = rng.bytes(32)
        sig = O.sign(_b32(d), dig)
        rows.append(("small_q", O.pubkey(_b32(d)), sig, dig, True))
    small = [1, 2, 3, 5, 8, 9, 16, 17, 127, 128, 129, 256, LAM, N - 1, 2**128 - 1, 2**127, 0x7F80, 0x7F807F80]
    tries = 0
    made = 0
    while made < per_kind and tries < 20 * per_kind:            # forced (u1, u2): exceptional adds
        tries += 1
        u1 = small[int(rng.integers(len(small)))] * int(rng.choice([1, 1, 3, LAM])) % N
        u2 = small[int(rng.integers(len(small)))] % N
        dq = int(rng.choice([1, 2, 3, N - 1, N - 2, 240]))
        Q = _mul(dq)
        out = _sig_for_uv(u1, u2, Q)
        if out is None:
            continue
        r, s, e = out
        add("forced_uv", R.compress(Q), r, s, e, True)
        made += 1
    for i, e in enumerate((0, N, N + 1, 2**256 - 1) * max(1, per_kind // 16)):   # u1 = 0, e >= n
        d = rand_scalar() or 1
        dig = _b32(e)
        rows.append(("digest_edge", O.pubkey(_b32(d)), O.sign(_b32(d), dig), dig, True))
    kinds = [r[0] for r in rows]
    pub = np.array([np.frombuffer(r[1], np.uint8) for r in rows])
    sig = np.array([np.frombuffer(r[2], np.uint8) for r in rows])
    dig = np.array([np.frombuffer(r[3], np.uint8) for r in rows])
    exp = np.array([r[4] for r in rows], np.uint8)
    return pub, sig, dig, exp, kinds
