#!/usr/bin/env python3
"""Writes tests/golden/ed25519_vectors.json: ed25519 VerifyBytes vectors with
verdicts from oracle/ed25519_ref.py (go1.14 crypto/ed25519 semantics), one
list per category of the edge cases the reference semantics decide:

  valid            RFC 8032 signatures over 0..700-byte messages (block edges)
  wrong_msg        a flipped message bit
  bad_r / bad_s    a flipped bit in R / in S
  s_high_bits      sig[63] & 224 != 0 (rejected before anything else)
  s_ge_l           S + L (< 2^253): ScMinimal rejects a malleated S
  s_eq_l           S = L exactly
  pub_not_on_curve y with no x (FromBytes fails)
  pub_noncanonical y + p for y < 19 that decode (accepted by FromBytes)
  pub_x0_sign      encoding of a point with x = 0 and bit 255 set (accepted)
  small_order      the 8 torsion points as keys, crafted valid signatures
  mixed_order      A = aB + T, signatures valid iff [h]T = 0 (cofactorless)
  r_noncanonical   R' = identity encoded as y = 1 + p / with bit 255 set
  r_identity       S = 0 with A of small order: R' = -[h]A

Run from the repo root: python tests/golden/make_ed25519_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ed25519_ref as E  # noqa: E402

P, L = E.P, E.L


def vec(pub, msg, sig):
    return {"pub": pub.hex(), "msg": msg.hex(), "sig": sig.hex(), "ok": E.verify(pub, msg, sig)}


def main():
    rng = random.Random(25519)
    cats = {}
    seeds = [rng.randbytes(32) for _ in range(8)]
    keys = [E.keypair(s) for s in seeds]

    def signed(i, msg):
        return keys[i % 8][2], E.sign(seeds[i % 8], msg)

    lens = [0, 1, 31, 32, 47, 48, 63, 64, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 350, 700]
    cats["valid"] = []
    for i, n in enumerate(lens):
        m = rng.randbytes(n)
        pub, sig = signed(i, m)
        cats["valid"].append(vec(pub, m, sig))

    def mutate(kind, count):
        out = []
        for i in range(count):
            m = rng.randbytes(rng.randrange(0, 300))
            pub, sig = signed(i, m)
            sig = bytearray(sig)
            if kind == "wrong_msg":
                m = bytearray(m + b"\x00")
                j = rng.randrange(len(m))
                m[j] ^= 1 << rng.randrange(8)
                m = bytes(m)
            elif kind == "bad_r":
                sig[rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif kind == "bad_s":
                sig[32 + rng.randrange(31)] ^= 1 << rng.randrange(8)
            elif kind == "s_high_bits":
                sig[63] |= 1 << rng.randrange(5, 8)
            elif kind == "s_ge_l":
                s = int.from_bytes(sig[32:], "little") + L
                if s >= 2**253:
                    continue
                sig[32:] = s.to_bytes(32, "little")
            out.append(vec(pub, m, bytes(sig)))
        return out

    for k in ("wrong_msg", "bad_r", "bad_s", "s_high_bits", "s_ge_l"):
        cats[k] = mutate(k, 12)
    m = b"s equals L"
    pub, sig = signed(0, m)
    cats["s_eq_l"] = [vec(pub, m, sig[:32] + L.to_bytes(32, "little"))]

    # keys that do not decode
    bad = []
    while len(bad) < 10:
        y = rng.randrange(P)
        enc = (y | (rng.randrange(2) << 255)).to_bytes(32, "little")
        if E.decode_point(enc) is None:
            m = rng.randbytes(40)
            bad.append(vec(enc, m, E.sign(seeds[0], m)))
    cats["pub_not_on_curve"] = bad

    tors = E.small_order_points()

    def crafted_valid(pub_enc, a_point, msg, tries=64):
        """A signature valid for a key of small order: s = r, R = rB + T with
        T = -[h]A (T in the torsion subgroup); found by trying the 8 T."""
        for _ in range(tries):
            r = rng.randrange(1, L)
            rb = E.point_mul(r, E.B)
            for t in tors:
                rp = E.point_add(rb, t)
                enc = E.encode_point(rp)
                h = E.sc_reduce(hashlib.sha512(enc + pub_enc + msg).digest())
                if E.point_mul(h, E.point_neg(a_point)) == t:
                    return enc + r.to_bytes(32, "little")
        return None

    # non-canonical y encodings that decode
    nonc = []
    for y0 in range(19):
        enc_v = y0 + P
        for sgn in (0, 1):
            enc = (enc_v | (sgn << 255)).to_bytes(32, "little")
            a = E.decode_point(enc)
            if a is None:
                continue
            m = b"noncanonical key %d %d" % (y0, sgn)
            sig = crafted_valid(enc, a, m)
            if sig is not None:
                nonc.append(vec(enc, m, sig))
            nonc.append(vec(enc, m, E.sign(seeds[1], m)))
    cats["pub_noncanonical"] = nonc

    # x = 0 with bit 255 set: the identity (y = 1) and (0, -1)
    x0 = []
    for y in (1, P - 1):
        enc = (y | (1 << 255)).to_bytes(32, "little")
        a = E.decode_point(enc)
        m = b"x0 sign %d" % y
        sig = crafted_valid(enc, a, m)
        x0.append(vec(enc, m, sig))
        x0.append(vec(enc, m + b"!", sig))
    cats["pub_x0_sign"] = x0

    so = []
    for t in tors:
        enc = E.encode_point(t)
        m = b"small order %d" % len(so)
        sig = crafted_valid(enc, t, m)
        if sig is not None:
            so.append(vec(enc, m, sig))
        so.append(vec(enc, m, E.sign(seeds[2], m)))
    cats["small_order"] = so

    mixed = []
    for i, t in enumerate(tors[1:]):
        a, prefix, _ = keys[i]
        ap = E.point_add(E.point_mul(a, E.B), t)
        enc = E.encode_point(ap)
        for _ in range(3):
            m = rng.randbytes(24)
            r = rng.randrange(1, L)
            mixed.append(vec(enc, m, E.sign_with(a, enc, r, m)))
    cats["mixed_order"] = mixed

    # R' = identity: A of small order with [h]A = 0 and S = 0
    rid = []
    ident = E.encode_point(E.IDENT)
    for enc_r in (ident, (1 + P).to_bytes(32, "little"), (1 | (1 << 255)).to_bytes(32, "little")):
        m = b"identity R"
        sig = enc_r + bytes(32)
        rid.append(vec(ident, m, sig))                      # A = identity: R' = [0]B - [h]O = O
    cats["r_noncanonical"] = rid[1:]
    cats["r_identity"] = rid[:1]

    total = sum(len(v) for v in cats.values())
    oks = sum(v["ok"] for c in cats.values() for v in c)
    out = {"generator": "tests/golden/make_ed25519_golden.py (verdicts: oracle/ed25519_ref.py)",
           "count": total, "accepted": oks, "categories": cats}
    path = os.path.join(HERE, "ed25519_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, total, "vectors,", oks, "accepted")
    for k, v in cats.items():
        print(f"  {k:18s} {len(v):3d}  accepted {sum(x['ok'] for x in v)}")


if __name__ == "__main__":
    main()
