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
