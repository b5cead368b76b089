"""Reduced-radix (10 x 26) field layer, host build, against Python integers.

tools/field26/secp_field26.cuh (a 10 x 26 prototype kept outside the product tree) is plain C++ apart from its qualifiers, so the exact
source the kernels use is compiled with g++ here and driven through ctypes:
random and extreme limb patterns at the maximum magnitudes the group formulas
are allowed to feed in (mul/sqr inputs <= 16, normalize/is_zero <= 32).
"""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "field26", "f26_host.cpp")
P = 2**256 - 2**32 - 977
M26 = (1 << 26) - 1
M22 = (1 << 22) - 1
PL = [0x3FFFC2F, 0x3FFFFBF] + [M26] * 7 + [M22]


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp()
    so = os.path.join(d, "f26.so")
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", so, SRC], check=True)
    L = ctypes.CDLL(so)
    return L


def arr(limbs):
    return (ctypes.c_uint32 * len(limbs))(*limbs)


def val(limbs):
    return sum(x << (26 * i) for i, x in enumerate(limbs))


def rand_mag(rng, m, style):
    """limbs with magnitude m (limb i <= m*M26, limb 9 <= m*M22)."""
    cap = [m * M26] * 9 + [m * M22]
    if style == "max":
        return cap[:]
    if style == "zero":
        return [0] * 10
    if style == "p":
        return [x * m for x in PL]
    return [rng.randint(0, c) for c in cap]


def out(L, fn, *args, n=10):
    r = (ctypes.c_uint32 * n)()
    getattr(L, fn)(*args, r)
    return list(r)


def check_mag1(limbs):
    assert all(x <= M26 + 1 for x in limbs[:9]) and limbs[9] <= M22 + 1, [hex(x) for x in limbs]


@pytest.mark.parametrize("ma,mb", [(1, 1), (16, 16), (16, 1), (3, 9), (10, 15)])
def test_mul_sqr(lib, ma, mb):
    rng = random.Random(ma * 100 + mb)
    styles = ["rand"] * 300 + ["max", "zero", "p"]
    for sa in styles:
        sb = rng.choice(styles)
        a, b = rand_mag(rng, ma, sa), rand_mag(rng, mb, sb)
        r = out(lib, "f26_mul", arr(a), arr(b))
        assert val(r) % P == val(a) * val(b) % P
        check_mag1(r)
        s = out(lib, "f26_sqr", arr(a))
        assert val(s) % P == val(a) ** 2 % P
        check_mag1(s)


def test_sub_neg_norm_words(lib):
    rng = random.Random(7)
    for it in range(2000):
        ma, mb = rng.randint(1, 12), rng.randint(1, 12)
        a = rand_mag(rng, ma, rng.choice(["rand", "rand", "max", "zero", "p"]))
        b = rand_mag(rng, mb, rng.choice(["rand", "rand", "max", "zero", "p"]))
        r = out(lib, "f26_sub", arr(a), arr(b), mb)
        assert val(r) % P == (val(a) - val(b)) % P
        assert all(x <= (ma + mb + 1) * M26 for x in r[:9]) and r[9] <= (ma + mb + 1) * M22
        ng = out(lib, "f26_neg", arr(b), mb)
        assert val(ng) % P == (-val(b)) % P
        m = rng.randint(1, 32)
        c = rand_mag(rng, m, rng.choice(["rand", "max", "zero", "p"]))
        nm = out(lib, "f26_norm", arr(c))
        assert val(nm) % P == val(c) % P
        check_mag1(nm)
        w = out(lib, "f26_to_words", arr(c), n=8)
        assert sum(x << (32 * i) for i, x in enumerate(w)) == val(c) % P
        assert lib.f26_is_zero(arr(c)) == (val(c) % P == 0)


def test_words_roundtrip_and_zero(lib):
    rng = random.Random(9)
    for v in [0, 1, P - 1, P, P + 5, 2**256 - 1, 2**255] + [rng.getrandbits(256) for _ in range(500)]:
        w = [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
        limbs = out(lib, "f26_from_words", arr(w))
        assert val(limbs) == v
        back = out(lib, "f26_to_words", arr(limbs), n=8)
        assert sum(x << (32 * i) for i, x in enumerate(back)) == v % P
    for z in [[0] * 10, PL, [2 * x for x in PL], [5 * x for x in PL]]:
        assert lib.f26_is_zero(arr(z)) == 1
    assert lib.f26_is_zero(arr([1] + [0] * 9)) == 0
