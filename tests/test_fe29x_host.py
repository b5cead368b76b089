"""Fused 9 x 29 product engine (csrc/secp_fe29x.cuh) and the throughput
ladder's group law on it (csrc/secp_group29x.cuh), host build with the
overflow traps (GV_F29_CHECK aborts on any wrapping mad / limb add), against
Python integers at the magnitude extremes the formulas feed in."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

from test_fe29_host import B, P, PL, M29, STYLES, arr, is_mag, rand_mag, val

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "fe29", "f29x_host.cpp")
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


@pytest.fixture(scope="module", params=[(1, 1), (0, 1), (1, 2)],
                ids=["hicarry-mad", "hicarry-classic", "two-chain"])
def lib(request):
    """Both high-column carry variants (throughput ladder) and the two-chain
    accumulator of the latency kernels (F29X_NCH = 2)."""
    hic, nch = request.param
    d = tempfile.mkdtemp()
    so = os.path.join(d, f"f29x_{hic}_{nch}.so")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-DGV_F29X_HICARRY={hic}", f"-DF29X_NCH={nch}", "-shared",
                    "-fPIC", "-o", so, SRC], check=True)
    return ctypes.CDLL(so)


def call(L, fn, *args):
    r = (ctypes.c_uint32 * 9)()
    getattr(L, fn)(*args, r)
    return list(r)


@pytest.mark.parametrize("ma,mb", [(1, 1), (2, 2), (1, 6), (6, 1), (2, 3), (3, 2), (1, 3)])
def test_mul_with_extras(lib, ma, mb):
    rng = random.Random(ma * 10 + mb)
    for it in range(500):
        a = rand_mag(rng, ma, rng.choice(STYLES))
        b = rand_mag(rng, mb, rng.choice(STYLES))
        c = rand_mag(rng, 4, rng.choice(STYLES))
        e = rand_mag(rng, 2, rng.choice(STYLES))
        for mode, want in ((0, 0), (1, val(c)), (2, 8 * val(c)), (3, val(c) + 8 * val(e))):
            r = call(lib, "f29xh_mul", arr(a), arr(b), arr(c), arr(e), mode)
            assert val(r) % P == (val(a) * val(b) + want) % P, (mode, it)
            assert is_mag(r, 1), [hex(x) for x in r]


@pytest.mark.parametrize("ma,mb,mc,md", [(1, 3, 2, 1), (1, 1, 1, 1), (2, 1, 1, 4), (1, 5, 1, 1), (3, 1, 1, 3)])
def test_mul2_sum_of_products(lib, ma, mb, mc, md):
    rng = random.Random(ma * 1000 + mb * 100 + mc * 10 + md)
    for it in range(500):
        a, b, c, d = (rand_mag(rng, m, rng.choice(STYLES)) for m in (ma, mb, mc, md))
        e = rand_mag(rng, 2, rng.choice(STYLES))
        for mode in (0, 1):
            r = (ctypes.c_uint32 * 9)()
            lib.f29xh_mul2(arr(a), arr(b), arr(c), arr(d), arr(e), mode, r)
            r = list(r)
            want = val(a) * val(b) + val(c) * val(d) + (8 * val(e) if mode else 0)
            assert val(r) % P == want % P, (mode, it)
            assert is_mag(r, 1), [hex(x) for x in r]


@pytest.mark.parametrize("m", [1, 2])
def test_sqr_with_extras(lib, m):
    rng = random.Random(70 + m)
    for it in range(800):
        a = rand_mag(rng, m, rng.choice(STYLES))
        c = rand_mag(rng, 4, rng.choice(STYLES))
        modes = [(0, val(a) ** 2), (1, val(a) ** 2 + val(c)), (2, val(a) ** 2 + 8 * val(c))]
        if m == 1:
            modes += [(3, 3 * val(a) ** 2), (4, 3 * val(a) ** 2 + 8 * val(c))]
        for mode, want in modes:
            r = call(lib, "f29xh_sqr", arr(a), arr(c), mode)
            assert val(r) % P == want % P, (mode, it)
            assert is_mag(r, 1), [hex(x) for x in r]


def affine_mul(k):
    """k*G affine by Python double-and-add (k >= 1)."""
    ax = ay = None
    for bit in bin(k)[2:]:
        if ax is not None:
            lam = 3 * ax * ax * pow(2 * ay, P - 2, P) % P
            nx = (lam * lam - 2 * ax) % P
            ay, ax = (lam * (ax - nx) - ay) % P, nx
        if bit == "1":
            if ax is None:
                ax, ay = GX, GY
            else:
                lam = (ay - GY) * pow(ax - GX, P - 2, P) % P
                nx = (lam * lam - ax - GX) % P
                ay, ax = (lam * (GX - nx) - GY) % P, nx
    return ax, ay


def limbs_of(rng, v, m):
    """v + k*p limb-wise for a random k < m: magnitude <= m."""
    k = rng.randrange(0, m)
    return [((v >> (29 * i)) & M29) + k * PL[i] for i in range(9)]


def jac(rng, x, y, mz=2):
    z = rng.randrange(1, P)
    return limbs_of(rng, x * z * z % P, 1) + limbs_of(rng, y * z ** 3 % P, 1) + limbs_of(rng, z, mz)


def to_affine(r):
    X, Y, Z = val(r[:9]) % P, val(r[9:18]) % P, val(r[18:]) % P
    zi = pow(Z, P - 2, P)
    return X * zi * zi % P, Y * zi ** 3 % P


def test_double(lib):
    rng = random.Random(5)
    for it in range(250):
        ax, ay = affine_mul(rng.randrange(1, 2 ** 64))
        inp = jac(rng, ax, ay)
        r = (ctypes.c_uint32 * 27)()
        lib.g29xh_double(arr(inp), r)
        r = list(r)
        assert is_mag(r[:9], 1) and is_mag(r[9:18], 1) and is_mag(r[18:], 1)
        lam = 3 * ax * ax * pow(2 * ay, P - 2, P) % P
        ex = (lam * lam - 2 * ax) % P
        assert to_affine(r) == (ex, (lam * (ax - ex) - ay) % P)


def test_add_scaled(lib):
    """acc + (x, y) where the entry is scaled by az: generic, a == b (doubling),
    a == -b (infinity); negated entries (y magnitude 2)."""
    rng = random.Random(6)
    for it in range(300):
        k1 = rng.randrange(1, 2 ** 64)
        kind = it % 5
        k2 = k1 if kind == 1 else rng.randrange(1, 2 ** 64)
        ax, ay = affine_mul(k1)
        bx, by = affine_mul(k2)
        if kind == 2:                       # a == -b
            bx, by = ax, (-ay) % P
        # the entry lives on the curve scaled by s: (x, y) = (bx / s^2, by / s^3) and
        # az = Z1 * s, so x az^2 = bx Z1^2 as on the accumulator's own curve
        s = rng.randrange(1, P)
        si = pow(s, P - 2, P)
        ex_, ey_ = bx * si * si % P, by * si ** 3 % P
        inp = jac(rng, ax, ay)
        z1 = val(inp[18:]) % P
        az = limbs_of(rng, z1 * s % P, 2)
        ylimbs = limbs_of(rng, ey_, 1)
        if kind == 3:                        # negated entry, magnitude 2 (f29_neg<1>)
            ylimbs = limbs_of(rng, (-ey_) % P, 2)
            by = (-by) % P
        out = (ctypes.c_uint32 * 27)()
        inf = lib.g29xh_add_scaled(arr(inp), arr(limbs_of(rng, ex_, 1)), arr(ylimbs), arr(az), out)
        out = list(out)
        if kind == 2:
            assert inf == 1
            continue
        assert inf == 0
        assert is_mag(out[:9], 1) and is_mag(out[9:18], 1) and is_mag(out[18:], 1)
        if (ax, ay) == (bx, by):
            lam = 3 * ax * ax * pow(2 * ay, P - 2, P) % P
        else:
            lam = (by - ay) * pow(bx - ax, P - 2, P) % P
        nx = (lam * lam - ax - bx) % P
        assert to_affine(out) == (nx, (lam * (ax - nx) - ay) % P), (it, kind)
