"""9 x 29 reduced-radix field layer (csrc/secp_fe29.cuh), host build, against
Python integers.

The header is plain C++ apart from its qualifiers, so the exact source the
kernels use is compiled with g++ here -- with GV_F29_CHECK, which aborts on any
wrapping u64 mad or u32 limb add -- and driven through ctypes at the maximum
magnitudes the group formulas are allowed to feed in (mul: mag(a)*mag(b) <= 6,
sqr: <= 2, linear results <= 7).
"""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "fe29", "f29_host.cpp")
P = 2**256 - 2**32 - 977
B = 2**29 + 2**18          # per-limb bound of magnitude 1
M29 = 2**29 - 1
PL = [(P >> (29 * i)) & M29 for i in range(9)]


@pytest.fixture(scope="module", params=[1, 2], ids=["one-chain", "two-chain"])
def lib(request):
    """Both product engines (F29_NCH = 1: throughput kernels, 2: latency kernels)."""
    d = tempfile.mkdtemp()
    so = os.path.join(d, f"f29_{request.param}.so")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-DF29_NCH={request.param}", "-shared", "-fPIC",
                    "-o", so, SRC], check=True)
    return ctypes.CDLL(so)


def arr(limbs):
    return (ctypes.c_uint32 * len(limbs))(*limbs)


def val(limbs):
    return sum(x << (29 * i) for i, x in enumerate(limbs))


def rand_mag(rng, m, style):
    cap = m * B
    if style == "max":
        return [cap] * 9
    if style == "zero":
        return [0] * 9
    if style == "p":
        return [x * m for x in PL]
    if style == "hi":
        return [rng.randint(cap - 2**20, cap) for _ in range(9)]
    return [rng.randint(0, cap) for _ in range(9)]


STYLES = ["rand"] * 40 + ["max", "zero", "p", "hi", "hi"]


def out(L, fn, *args, n=9):
    r = (ctypes.c_uint32 * n)()
    rc = getattr(L, fn)(*args, r)
    return list(r), rc


def is_mag(limbs, m):
    return all(x <= m * B for x in limbs)


@pytest.mark.parametrize("ma,mb", [(1, 1), (2, 2), (1, 6), (6, 1), (2, 3), (3, 2)])
def test_mul(lib, ma, mb):
    rng = random.Random(ma * 100 + mb)
    for it in range(600):
        a = rand_mag(rng, ma, rng.choice(STYLES))
        b = rand_mag(rng, mb, rng.choice(STYLES))
        r, _ = out(lib, "f29h_mul", arr(a), arr(b))
        assert val(r) % P == val(a) * val(b) % P
        assert is_mag(r, 1), [hex(x) for x in r]


@pytest.mark.parametrize("m", [1, 2])
def test_sqr(lib, m):
    rng = random.Random(m)
    for it in range(1500):
        a = rand_mag(rng, m, rng.choice(STYLES))
        r, _ = out(lib, "f29h_sqr", arr(a))
        assert val(r) % P == val(a) ** 2 % P
        assert is_mag(r, 1), [hex(x) for x in r]


def test_linear_and_norm(lib):
    rng = random.Random(7)
    for it in range(3000):
        mb = rng.randint(1, 6)
        ma = rng.randint(0, 6 - mb)
        a = rand_mag(rng, ma, rng.choice(STYLES)) if ma else [0] * 9
        b = rand_mag(rng, mb, rng.choice(STYLES))
        r, rc = out(lib, "f29h_sub", arr(a), arr(b), mb)
        assert rc == 0
        assert val(r) % P == (val(a) - val(b)) % P
        assert is_mag(r, ma + mb + 1)
        ng, rc = out(lib, "f29h_neg", arr(b), mb)
        assert val(ng) % P == (-val(b)) % P and is_mag(ng, mb + 1)
        m = rng.randint(1, 7)
        c = rand_mag(rng, m, rng.choice(STYLES))
        nm, _ = out(lib, "f29h_norm", arr(c))
        assert val(nm) % P == val(c) % P and is_mag(nm, 1)
        w, _ = out(lib, "f29h_to_words", arr(c), n=8)
        assert sum(x << (32 * i) for i, x in enumerate(w)) == val(c) % P
        assert lib.f29h_is_zero(arr(c)) == (val(c) % P == 0)
        s = rng.randint(1, 3)
        d = rand_mag(rng, 1, rng.choice(STYLES))
        sh, rc = out(lib, "f29h_shl_norm", arr(d), s)
        assert rc == 0 and val(sh) % P == (val(d) << s) % P and is_mag(sh, 1)


def test_words_roundtrip_and_zero(lib):
    rng = random.Random(9)
    for v in [0, 1, P - 1, P, P + 5, 2**256 - 1, 2**255] + [rng.getrandbits(256) for _ in range(500)]:
        w = [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]
        limbs, _ = out(lib, "f29h_from_words", arr(w))
        assert val(limbs) == v and is_mag(limbs, 1)
        back, _ = out(lib, "f29h_to_words", arr(limbs), n=8)
        assert sum(x << (32 * i) for i, x in enumerate(back)) == v % P
    for k in range(0, 8):
        z = [x * k for x in PL]
        assert lib.f29h_is_zero(arr(z)) == 1
    assert lib.f29h_is_zero(arr([1] + [0] * 8)) == 0


@pytest.mark.parametrize("dbl25,ilp", [(0, 0), (0, 1), (1, 1)], ids=["3M4S", "3M4S-ilp", "2M5S"])
def test_jacobian_double_variants(dbl25, ilp):
    """gej29_double (csrc/secp_group29.cuh) in each formula variant, host build
    with overflow traps, at the point invariant's extreme magnitudes (X, Y
    magnitude 1, Z <= 2): same point as affine doubling, output invariant kept."""
    d = tempfile.mkdtemp()
    so = os.path.join(d, "g29.so")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-DGV_DBL25={dbl25}", f"-DGV_ILP={ilp}", "-shared", "-fPIC",
                    "-o", so, os.path.join(REPO, "tools", "fe29", "g29_host.cpp")], check=True)
    L = ctypes.CDLL(so)
    rng = random.Random(dbl25 * 10 + ilp)
    Gx = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
    Gy = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
    for it in range(250):
        k = rng.randrange(1, 2**64)
        # a random multiple of G in affine form via Python double-and-add
        x, y = Gx, Gy
        ax = ay = None
        for bit in bin(k)[2:]:
            if ax is not None:
                lam = 3 * ax * ax * pow(2 * ay, P - 2, P) % P
                nx = (lam * lam - 2 * ax) % P
                ay = (lam * (ax - nx) - ay) % P
                ax = nx
            if bit == "1":
                if ax is None:
                    ax, ay = x, y
                else:
                    lam = (ay - y) * pow(ax - x, P - 2, P) % P
                    nx = (lam * lam - ax - x) % P
                    ay = (lam * (x - nx) - y) % P
                    ax = nx
        z = rng.randrange(1, P)
        X, Y = ax * z * z % P, ay * z * z * z % P

        def limbs(v, m):            # v + k*p limb-wise, k < m: magnitude m at most
            k = rng.randrange(0, m)
            return [((v >> (29 * i)) & M29) + k * PL[i] for i in range(9)]
        inp = limbs(X, 1) + limbs(Y, 1) + limbs(z, 2)
        assert val(inp[:9]) % P == X and val(inp[9:18]) % P == Y and val(inp[18:]) % P == z
        r = (ctypes.c_uint32 * 27)()
        L.g29h_double(arr(inp), r)
        r = list(r)
        X3, Y3, Z3 = val(r[:9]) % P, val(r[9:18]) % P, val(r[18:]) % P
        assert is_mag(r[:9], 1) and is_mag(r[9:18], 1) and is_mag(r[18:], 2)
        lam = 3 * ax * ax * pow(2 * ay, P - 2, P) % P
        ex = (lam * lam - 2 * ax) % P
        ey = (lam * (ax - ex) - ay) % P
        zi = pow(Z3, P - 2, P)
        assert X3 * zi * zi % P == ex and Y3 * zi * zi * zi % P == ey


@pytest.mark.parametrize("m", [1, 2])
def test_multi_stream_products(lib, m):
    """f29_multi: independent squares / products in lockstep == separate calls."""
    rng = random.Random(40 + m)
    for it in range(800):
        xs = [rand_mag(rng, m, rng.choice(STYLES)) for _ in range(3)]
        ys = [rand_mag(rng, m, rng.choice(STYLES)) for _ in range(3)]
        r = (ctypes.c_uint32 * 27)()
        lib.f29h_multi(arr(sum(xs, [])), arr(sum(ys, [])), r)
        r = list(r)
        want = [val(xs[0]) ** 2 % P, val(xs[1]) ** 2 % P, val(xs[2]) * val(ys[2]) % P]
        for s in range(3):
            limbs = r[9 * s:9 * s + 9]
            assert val(limbs) % P == want[s] and is_mag(limbs, 1)
