"""s^-1 mod n by divsteps (csrc/secp_modinv.cuh, the latency kernel's scalar
inverse), host build, against Python's pow(x, -1, n): random and edge
scalars, the round bound, and the transition-matrix bound of one batch."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp()
    so = os.path.join(d, "mi.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(REPO, "tools", "fe29", "modinv_host.cpp")], check=True)
    L = ctypes.CDLL(so)
    L.mi_divsteps.restype = ctypes.c_int32
    return L


def words(x):
    return (ctypes.c_uint32 * 8)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def inv(L, x):
    w = (ctypes.c_uint32 * 8)()
    rounds = L.mi_inv(words(x), w)
    return sum(v << (32 * i) for i, v in enumerate(w)), rounds


def test_random_and_edge_inverses(lib):
    rng = random.Random(5)
    xs = [1, 2, 3, N - 1, N - 2, (N - 1) // 2, (N + 1) // 2, 2**255, 2**128 + 1, 0xFFFFFFFF, 1 << 30, (1 << 30) - 1]
    xs += [rng.randrange(1, N) for _ in range(3000)]
    xs += [rng.randrange(1, 2**k) for k in (8, 32, 64, 129, 200) for _ in range(40)]
    worst = 0
    for x in xs:
        got, rounds = inv(lib, x)
        assert got == pow(x, -1, N), hex(x)
        worst = max(worst, rounds)
    assert worst <= 25


def test_zero_gives_zero(lib):
    assert inv(lib, 0)[0] == 0


def test_batch_matrix_bound(lib):
    """|u| + |v| <= 2^30 and |q| + |r| <= 2^30 after 30 divsteps, and the
    matrix maps the low words exactly (2^30 f' = u f + v g mod 2^32)."""
    rng = random.Random(7)
    for _ in range(3000):
        f = rng.getrandbits(32) | 1
        g = rng.getrandbits(32)
        delta = rng.randrange(-40, 41)
        t = (ctypes.c_int32 * 4)()
        lib.mi_divsteps(delta, f, g, t)
        u, v, q, r = t
        assert abs(u) + abs(v) <= 2**30 and abs(q) + abs(r) <= 2**30
        assert (u * f + v * g) % 2**30 == 0 and (q * f + r * g) % 2**30 == 0


def inv_var(L, x):
    w = (ctypes.c_uint32 * 8)()
    rounds = L.mi_inv_var(words(x), w)
    return sum(v << (32 * i) for i, v in enumerate(w)), rounds


def test_var_time_inverses(lib):
    """The variable-time divsteps (s30_modinv_var, gv_lat.hip's lat_scalars)
    give the same inverse on random and edge scalars, within the round cap."""
    rng = random.Random(11)
    xs = [1, 2, 3, N - 1, N - 2, (N - 1) // 2, (N + 1) // 2, 2**255, 2**128 + 1, 0xFFFFFFFF, 1 << 30, (1 << 30) - 1]
    xs += [rng.randrange(1, N) for _ in range(5000)]
    xs += [rng.randrange(1, 2**k) for k in (8, 32, 64, 129, 200) for _ in range(40)]
    worst = 0
    for x in xs:
        got, rounds = inv_var(lib, x)
        assert got == pow(x, -1, N), hex(x)
        worst = max(worst, rounds)
    assert worst <= 20
    assert inv_var(lib, 0)[0] == 0


def test_var_batch_matches_single_steps(lib):
    """One var-time batch is the same transition as 30 single divsteps of the
    eta form (delta = -eta), hence the same matrix bound."""
    lib.mi_divsteps_var.restype = ctypes.c_int32
    rng = random.Random(13)
    for _ in range(5000):
        f = rng.getrandbits(32) | 1
        g = rng.getrandbits(32)
        eta = rng.randrange(-40, 41)
        t = (ctypes.c_int32 * 4)()
        eta2 = lib.mi_divsteps_var(eta, f, g, t)
        # reference: 30 single eta-form divsteps on Python ints
        uu, vv, qq, rr, ff, gg, e = 1, 0, 0, 1, f, g, eta
        for _ in range(30):
            if e < 0 and gg & 1:
                e, ff, gg, uu, vv, qq, rr = -e, gg, -ff, qq, rr, -uu, -vv
            if gg & 1:
                gg, qq, rr = gg + ff, qq + uu, rr + vv
            e, gg, uu, vv = e - 1, gg >> 1, uu << 1, vv << 1
        assert eta2 == e
        assert list(t) == [uu, vv, qq, rr], (f, g, eta)
        assert abs(uu) + abs(vv) <= 2**30 and abs(qq) + abs(rr) <= 2**30
