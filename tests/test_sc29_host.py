"""Radix-2^29 Montgomery arithmetic mod n (csrc/secp_sc29.cuh), host build with
overflow traps, against Python integers: products, squares, the Fermat
inverse schedule (tools/gen_sc29_inv.py), conversions."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "fe29", "sc29_host.cpp")
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
R = 2**261
M29 = 2**29 - 1


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp()
    so = os.path.join(d, "sc29.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so, SRC], check=True)
    return ctypes.CDLL(so)


def limbs(v):
    return [(v >> (29 * i)) & M29 for i in range(9)]


def val(ls):
    return sum(x << (29 * i) for i, x in enumerate(ls))


def call(L, fn, *vals, n=9):
    r = (ctypes.c_uint32 * n)()
    args = [(ctypes.c_uint32 * 9)(*limbs(v)) for v in vals]
    getattr(L, fn)(*args, r)
    return list(r)


def norm_ok(ls):
    return all(x <= M29 for x in ls) and val(ls) < 2 * N


EDGE = [0, 1, 2, N - 1, N, N + 1, 2 * N - 1, 2**256 - 1, 2**257 - 1, 2**255, R % N]


def test_montmul_sqr(lib):
    rng = random.Random(3)
    vals = EDGE + [rng.randrange(2**258) for _ in range(1500)]
    rinv = pow(R, -1, N)
    for it in range(2500):
        a, b = rng.choice(vals), rng.choice(vals)
        r = call(lib, "sc29h_mul", a, b)
        assert val(r) % N == a * b * rinv % N and norm_ok(r)
        s = call(lib, "sc29h_sqr", a)
        assert val(s) % N == a * a * rinv % N and norm_ok(s)


def test_inverse_and_conversions(lib):
    rng = random.Random(5)
    for x in [1, 2, N - 1, N - 2, 3, 2**128] + [rng.randrange(1, N) for _ in range(200)]:
        xm = call(lib, "sc29h_to_mont", x)
        assert val(xm) % N == x * R % N and norm_ok(xm)
        im = call(lib, "sc29h_inv", val(xm))
        assert val(im) % N == pow(x, N - 2, N) * R % N and norm_ok(im)
        plain = call(lib, "sc29h_mul", val(im), 1)          # from Montgomery form
        w = call(lib, "sc29h_to_words", val(plain), n=8)
        assert sum(v << (32 * i) for i, v in enumerate(w)) == pow(x, N - 2, N)
    for v in [0, 1, N - 1, N, 2**256 - 1] + [rng.getrandbits(256) for _ in range(300)]:
        ws = (ctypes.c_uint32 * 8)(*[(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
        r = (ctypes.c_uint32 * 9)()
        lib.sc29h_from_words(ws, r)
        assert val(list(r)) == v
