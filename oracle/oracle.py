"""ctypes loader for the C oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (libgpuverify.so) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_verify_digest.argtypes = [u8p, u8p, u8p]
        L.oracle_verify_digest.restype = ctypes.c_int
        L.oracle_verify_bytes.argtypes = [u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.oracle_verify_bytes.restype = ctypes.c_int
        L.oracle_verify_digests.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, u8p, ctypes.c_int]
        L.oracle_verify_msgs.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint32), u8p, ctypes.c_int]
        L.oracle_sign_batch.argtypes = [ctypes.c_size_t, u8p, u8p, u8p, ctypes.c_int]
        L.oracle_pubkey_batch.argtypes = [ctypes.c_size_t, u8p, u8p, ctypes.c_int]
        L.oracle_sign.argtypes = [u8p, u8p, u8p]
        L.oracle_sign.restype = ctypes.c_int
        L.oracle_pubkey.argtypes = [u8p, u8p]
        L.oracle_pubkey.restype = ctypes.c_int
        L.oracle_parse_pubkey.argtypes = [u8p, u8p, u8p]
        L.oracle_parse_pubkey.restype = ctypes.c_int
        L.oracle_point_mul.argtypes = [u8p, u8p, u8p]
        L.oracle_point_mul.restype = ctypes.c_int
        L.oracle_privkey_from_secret.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.oracle_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _buf(b: bytes):
    return (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")


def verify_digest(pub: bytes, sig: bytes, dig: bytes) -> bool:
    assert len(pub) == 33 and len(sig) == 64 and len(dig) == 32
    return bool(lib().oracle_verify_digest(_buf(pub), _buf(sig), _buf(dig)))


def verify_bytes(pub: bytes, msg: bytes, sig: bytes) -> bool:
    return bool(lib().oracle_verify_bytes(_buf(pub), _buf(msg), len(msg), _buf(sig), len(sig)))


def verify_digests(pub33: np.ndarray, sig64: np.ndarray, dig32: np.ndarray, threads: int = 1) -> np.ndarray:
    n = pub33.shape[0]
    out = np.zeros(n, dtype=np.uint8)
    lib().oracle_verify_digests(n, _p(pub33), _p(sig64), _p(dig32), _p(out), threads)
    return out


def verify_msgs(pub33, sig64, blob, off, ln, threads: int = 1) -> np.ndarray:
    n = pub33.shape[0]
    out = np.zeros(n, dtype=np.uint8)
    lib().oracle_verify_msgs(n, _p(pub33), _p(sig64), _p(blob),
                             off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                             ln.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _p(out), threads)
    return out


def sign_batch(priv32: np.ndarray, dig32: np.ndarray, threads: int = 1) -> np.ndarray:
    n = priv32.shape[0]
    out = np.zeros((n, 64), dtype=np.uint8)
    lib().oracle_sign_batch(n, _p(priv32), _p(dig32), _p(out), threads)
    return out


def pubkey_batch(priv32: np.ndarray, threads: int = 1) -> np.ndarray:
    n = priv32.shape[0]
    out = np.zeros((n, 33), dtype=np.uint8)
    lib().oracle_pubkey_batch(n, _p(priv32), _p(out), threads)
    return out


def sign(priv: bytes, dig: bytes) -> bytes:
    out = (ctypes.c_uint8 * 64)()
    assert lib().oracle_sign(_buf(priv), _buf(dig), out)
    return bytes(out)


def pubkey(priv: bytes) -> bytes:
    out = (ctypes.c_uint8 * 33)()
    assert lib().oracle_pubkey(_buf(priv), out)
    return bytes(out)


def parse_pubkey(pub: bytes):
    x = (ctypes.c_uint8 * 32)()
    y = (ctypes.c_uint8 * 32)()
    if not lib().oracle_parse_pubkey(_buf(pub), x, y):
        return None
    return int.from_bytes(bytes(x), "big"), int.from_bytes(bytes(y), "big")


def point_mul(k: int, pub: bytes | None = None):
    """k*G (pub None) or k*Q; returns (x, y) or None for infinity."""
    xy = (ctypes.c_uint8 * 64)()
    rc = lib().oracle_point_mul(_buf(pub) if pub is not None else None, _buf(k.to_bytes(32, "big")), xy)
    if rc <= 0:
        return None
    b = bytes(xy)
    return int.from_bytes(b[:32], "big"), int.from_bytes(b[32:], "big")


def privkey_from_secret(secret: bytes) -> bytes:
    out = (ctypes.c_uint8 * 32)()
    lib().oracle_privkey_from_secret(_buf(secret), len(secret), out)
    return bytes(out)


def sha256(msg: bytes) -> bytes:
    out = (ctypes.c_uint8 * 32)()
    lib().oracle_sha256(_buf(msg), len(msg), out)
    return bytes(out)
