#!/usr/bin/env python3
"""Generate the committed golden fixtures tests/golden/vectors_*.json.

Expected verdicts come from the pure-Python restatement oracle/secp_ref.py
(the reference's Go path is not runnable here: SURVEY.md §8c).  The recipes
follow SURVEY.md §8c "Golden fixture recipes".  Deterministic: seeded.

Categories (digest path unless noted):
  valid            RFC6979 low-S signatures over random digests
  valid_msg        (message path) RFC6979 over MsgSend StdSignBytes
  high_s           s' = n - s of a valid signature                 -> reject
  s_halfn          otherwise-valid signature with s == (n-1)/2     -> accept
  s_halfn_plus1    otherwise-valid signature with s == (n+1)/2     -> reject
  r_range / s_range  r in {0,n,n+1,2^256-1}, s in {0,n,2^256-1}    -> reject
  bad_prefix       prefix in {00,01,04,05,06,07,FF}                -> reject
  x_ge_p           x = p + x' (x' a valid x)                        -> reject
  x_nonresidue     x^3+7 not a square                              -> reject
  parity_flip      valid point, other y, original signature        -> reject
  wrong_msg        one-bit flip of the digest                      -> reject
  infinity         u1*G + u2*Q = O                                 -> reject
  x_in_n_p         R.x in [n,p): r = R.x - n                        -> accept
  x_in_n_p_rbig    same R, r = R.x (>= n)                          -> reject
  small_q          Q in {G,-G,2G,3G,lambda G,...} valid signatures
  forced_uv        chosen (u1,u2,Q) hitting exceptional additions
  digest_edge      e in {0, n, n+1, 2^256-1}, valid signatures
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import secp_ref as R  # noqa: E402

P, N, G, HALF_N = R.P, R.N, R.G, R.HALF_N


def b32(x):
    return (x % 2**256).to_bytes(32, "big")


def sig_bytes(r, s):
    return b32(r) + b32(s)


def rec(cat, pub, sig, dig):
    ok = R.verify_digest(pub, sig, dig)
    return {"cat": cat, "pub": pub.hex(), "sig": sig.hex(), "dig": dig.hex(), "ok": bool(ok)}


def lift_x(x, odd=0):
    c = (x * x * x + 7) % P
    y = pow(c, (P + 1) // 4, P)
    if y * y % P != c:
        return None
    if (y & 1) != odd:
        y = P - y
    return (x, y)


def sig_for_uv(u1, u2, Q):
    """Signature (r, s) and digest e such that verification computes exactly
    u1*G + u2*Q (w = s^-1, u1 = e*w, u2 = r*w)."""
    Rpt = R.point_add(R.point_mul(u1, G), R.point_mul(u2, Q))
    if Rpt is None:
        return None
    r = Rpt[0] % N
    if r == 0:
        return None
    w = u2 * pow(r, N - 2, N) % N
    s = pow(w, N - 2, N)
    e = u1 * s % N
    return r, s, e


def main():
    rng = random.Random(0xC3)
    dv, mv = [], []

    keys = [R.privkey_from_secret(b"gv-golden-" + i.to_bytes(8, "little")) for i in range(24)]
    pubs = [R.pubkey(d) for d in keys]

    # valid + derived rejects
    for i in range(160):
        d = keys[i % len(keys)]
        pub = pubs[i % len(keys)]
        dig = rng.randbytes(32)
        sig = R.sign_digest(d, dig)
        dv.append(rec("valid", pub, sig, dig))
        r = int.from_bytes(sig[:32], "big")
        s = int.from_bytes(sig[32:], "big")
        if i < 40:
            dv.append(rec("high_s", pub, sig_bytes(r, N - s), dig))
        if i < 40:
            bad = bytearray(dig)
            bad[rng.randrange(32)] ^= 1 << rng.randrange(8)
            dv.append(rec("wrong_msg", pub, sig, bytes(bad)))
        if i < 24:
            flipped = bytes([pub[0] ^ 1]) + pub[1:]
            dv.append(rec("parity_flip", flipped, sig, dig))
        if i < 14:
            pre = [0x00, 0x01, 0x04, 0x05, 0x06, 0x07, 0xFF][i % 7]
            dv.append(rec("bad_prefix", bytes([pre]) + pub[1:], sig, dig))
        if i < 8:
            rr = [0, N, N + 1, 2**256 - 1][i % 4]
            dv.append(rec("r_range", pub, sig_bytes(rr, s), dig))
            ss = [0, N, 2**256 - 1, N - 1][i % 4]
            dv.append(rec("s_range", pub, sig_bytes(r, ss), dig))

    # s == halfN (accept) / halfN + 1 (reject): key recovery with chosen s
    for i in range(6):
        for cat, s in (("s_halfn", HALF_N), ("s_halfn_plus1", HALF_N + 1)):
            k = rng.randrange(1, N)
            Rp = R.point_mul(k, G)
            r = Rp[0] % N
            dig = rng.randbytes(32)
            e = int.from_bytes(dig, "big")
            rinv = pow(r, N - 2, N)
            # Q = r^-1 (s R - e G)
            Q = R.point_mul(rinv, R.point_add(R.point_mul(s, Rp), R.point_neg(R.point_mul(e, G))))
            dv.append(rec(cat, R.compress(Q), sig_bytes(r, s), dig))

    # x >= p, non-residue x
    for i in range(6):
        xs = rng.randrange(1, 2**32 - 977)
        while lift_x(xs) is None or xs + P >= 2**256:
            xs = rng.randrange(1, 2**32 - 977)
        pub = bytes([2 + (i & 1)]) + b32(xs + P)
        dv.append(rec("x_ge_p", pub, R.sign_digest(keys[0], b"\x11" * 32), b"\x11" * 32))
        xn = rng.randrange(P)
        while lift_x(xn) is not None:
            xn = rng.randrange(P)
        pub = bytes([2 + (i & 1)]) + b32(xn)
        dv.append(rec("x_nonresidue", pub, R.sign_digest(keys[1], b"\x22" * 32), b"\x22" * 32))
    # x == p exactly and x == 2^256-1
    for x in (P, 2**256 - 1, 0):
        dv.append(rec("x_ge_p" if x >= P else "x_zero", bytes([2]) + b32(x), R.sign_digest(keys[0], b"\x33" * 32),
                      b"\x33" * 32))

    # infinity: d = -e r^-1, Q = dG  ->  u1 G + u2 Q = w(e + r d) G = O
    for i in range(8):
        dig = rng.randbytes(32)
        e = int.from_bytes(dig, "big") % N
        r = rng.randrange(1, N)
        d = (-e * pow(r, N - 2, N)) % N
        if d == 0:
            continue
        s = rng.randrange(1, HALF_N)
        dv.append(rec("infinity", R.pubkey(d), sig_bytes(r, s), dig))

    # x in [n, p): R.x = n + delta with delta small (smallest: delta = 2 -> r = 2)
    deltas = [d for d in range(1, 400) if N + d < P and lift_x(N + d) is not None][:6]
    for j, delta in enumerate(deltas):
        Rp = lift_x(N + delta, odd=j & 1)
        r = delta
        s = rng.randrange(1, HALF_N)
        dig = rng.randbytes(32)
        e = int.from_bytes(dig, "big")
        rinv = pow(r, N - 2, N)
        Q = R.point_mul(rinv, R.point_add(R.point_mul(s, Rp), R.point_neg(R.point_mul(e, G))))
        pub = R.compress(Q)
        dv.append(rec("x_in_n_p", pub, sig_bytes(r, s), dig))
        dv.append(rec("x_in_n_p_rbig", pub, sig_bytes(N + delta, s), dig))

    # small / structured public keys (exceptional additions in the ladder)
    lam = R.LAMBDA
    for d in (1, 2, 3, 4, 7, 8, 9, 15, 16, 17, 128, 129, 255, 256, N - 1, N - 2, lam, N - lam, (lam * lam) % N):
        Q = R.pubkey(d)
        for t in range(3):
            dig = rng.randbytes(32) if t else b32(d)
            dv.append(rec("small_q", Q, R.sign_digest(d, dig), dig))

    # forced (u1, u2, Q): accumulator meets +-table entry inside the Strauss ladder
    ALT15 = sum((0x4000 if j % 2 == 0 else 0x3FFF) << (15 * j) for j in range(8))
    ALT20 = sum((0x80000 if j % 2 == 0 else 0x7FFFF) << (20 * j) for j in range(6))
    forced = []
    small = [1, 2, 3, 5, 8, 9, 16, 17, 127, 128, 129, 256]
    for a in small:
        for b in (1, 2, 3, 8, 9):
            forced.append((a, b, 1))
            forced.append((a, b, N - 1))
    for (a, b, dq) in [(1, 1, 2), (2, 1, 3), (lam, 1, 1), (1, lam, 1), (lam, lam, 1), (N - 1, 2, 1),
                       (2**128 - 1, 2**128 - 1, 1), (2**128, 1, 1), (1, 2**128, 1), (N - 2**128, 1, 1),
                       (16, 1, 240), (1, 1, N - 2), (3, 5, 7), (2**127, 2**127, 1),
                       # Booth extremes: +128 in an 8-bit G window, +8 in a 4-bit Q window
                       (0x7F80, 3, 1), (0x7F807F80, 0x78, 5), (0x7F80 << 64, 0x7878, 1),
                       (N - 0x7F80, 0x78 << 100, 9), (0x7F80 << 112, 2**127 + 0x78, 1),
                       # Booth extremes of 15-bit G windows: alternating -2^14 / +2^14 digits
                       (ALT15, 3, 1), ((lam * ALT15) % N, 5, 1), (ALT15 | 2**127, 2, 3),
                       (ALT15 + (lam * (ALT15 >> 15)) % N, 9, 1), (0x1FFFC000, 1, 7),
                       ((lam * 0x1FFFC000) % N, 0x78, 1),
                       # ... and of 20-bit G windows: alternating -2^19 / +2^19 digits
                       (ALT20, 3, 1), ((lam * ALT20) % N, 5, 1), (ALT20 | 2**127, 2, 3),
                       (ALT20 + (lam * (ALT20 >> 20)) % N, 9, 1), ((0x7FFFF << 20) | (1 << 19), 1, 7)]:
        forced.append((a, b, dq))
    for (u1, u2, dq) in forced:
        Q = R.point_mul(dq, G)
        out = sig_for_uv(u1 % N, u2 % N, Q)
        if out is None:
            continue
        r, s, e = out
        if s > HALF_N:
            s = N - s                 # negating w negates u1, u2: R -> -R, same x
            e = e                     # e = u1*s_old; with s_new = -s_old: u1_new = -u1
        dv.append(rec("forced_uv", R.compress(Q), sig_bytes(r, s), b32(e)))

    # digest edge values (u1 = 0, e >= n)
    for i, e in enumerate((0, N, N + 1, 2**256 - 1, N - 1, 1)):
        d = keys[i]
        dv.append(rec("digest_edge", pubs[i], R.sign_digest(d, b32(e)), b32(e)))

    # message path: MsgSend StdSignBytes (C1 recipe)
    for i in range(48):
        d = keys[i % len(keys)]
        pub = pubs[i % len(keys)]
        frm = R.address(pub)
        to = R.address(pubs[(i + 1) % len(keys)])
        msg_json = R.msg_send_json(frm, to, [(10, "foocoin")])
        memo = "" if i % 3 else "memo-" + "x" * (i * 5)   # vary the block count
        sb = R.std_sign_bytes("gv-bench", i, i % 5, [(0, "stake")], 1000000, [msg_json], memo)
        sig = R.sign(d, sb)
        ok = R.verify_bytes(pub, sb, sig)
        mv.append({"cat": "valid_msg", "pub": pub.hex(), "sig": sig.hex(), "msg": sb.hex(), "ok": bool(ok)})
        if i % 4 == 0:
            tampered = sb.replace(b'"sequence":"', b'"sequence":"1')
            mv.append({"cat": "wrong_seq_msg", "pub": pub.hex(), "sig": sig.hex(), "msg": tampered.hex(),
                       "ok": bool(R.verify_bytes(pub, tampered, sig))})
    # SHA-256 padding boundaries: lengths 0, 55, 56, 63, 64, 119, 120
    for L in (0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 1000):
        msg = bytes((7 * j + L) & 0xFF for j in range(L))
        d = keys[L % len(keys)]
        sig = R.sign(d, msg)
        mv.append({"cat": "len_edge_msg", "pub": R.pubkey(d).hex(), "sig": sig.hex(), "msg": msg.hex(),
                   "ok": bool(R.verify_bytes(R.pubkey(d), msg, sig))})

    with open(os.path.join(HERE, "vectors_digest.json"), "w") as f:
        json.dump(dv, f, indent=0)
    with open(os.path.join(HERE, "vectors_msg.json"), "w") as f:
        json.dump(mv, f, indent=0)
    cats = {}
    for v in dv + mv:
        cats.setdefault(v["cat"], [0, 0])[0 if v["ok"] else 1] += 1
    print(json.dumps({k: {"accept": a, "reject": r} for k, (a, r) in sorted(cats.items())}, indent=1))


if __name__ == "__main__":
    main()
