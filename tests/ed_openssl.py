"""OpenSSL's Ed25519 (libcrypto via ctypes) as an independent second opinion
for the ed25519 oracle -- test infrastructure only.  OpenSSL agrees with
go1.14 crypto/ed25519 on canonical keys and signatures; the edge cases where
implementations differ (non-canonical keys, small-order points) are decided by
oracle/ed25519_ref.py alone."""
import ctypes
import ctypes.util

EVP_PKEY_ED25519 = 1087

_C = ctypes.CDLL(ctypes.util.find_library("crypto"))
_vp = ctypes.c_void_p
_C.EVP_PKEY_new_raw_private_key.restype = _vp
_C.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, _vp, ctypes.c_char_p, ctypes.c_size_t]
_C.EVP_PKEY_new_raw_public_key.restype = _vp
_C.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, _vp, ctypes.c_char_p, ctypes.c_size_t]
_C.EVP_PKEY_get_raw_public_key.argtypes = [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
_C.EVP_PKEY_free.argtypes = [_vp]
_C.EVP_MD_CTX_new.restype = _vp
_C.EVP_MD_CTX_free.argtypes = [_vp]
_C.EVP_DigestSignInit.argtypes = [_vp, _vp, _vp, _vp, _vp]
_C.EVP_DigestSign.argtypes = [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
_C.EVP_DigestVerifyInit.argtypes = [_vp, _vp, _vp, _vp, _vp]
_C.EVP_DigestVerify.argtypes = [_vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]


def public_key(seed: bytes) -> bytes:
    k = _C.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    out = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    assert _C.EVP_PKEY_get_raw_public_key(k, out, ctypes.byref(n)) == 1
    _C.EVP_PKEY_free(k)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    k = _C.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    c = _C.EVP_MD_CTX_new()
    assert _C.EVP_DigestSignInit(c, None, None, None, k) == 1
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(64)
    assert _C.EVP_DigestSign(c, out, ctypes.byref(n), msg, len(msg)) == 1
    _C.EVP_MD_CTX_free(c)
    _C.EVP_PKEY_free(k)
    return out.raw


def verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    k = _C.EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, None, pub, 32)
    if not k:
        return False
    c = _C.EVP_MD_CTX_new()
    ok = _C.EVP_DigestVerifyInit(c, None, None, None, k) == 1 and \
        _C.EVP_DigestVerify(c, sig, len(sig), msg, len(msg)) == 1
    _C.EVP_MD_CTX_free(c)
    _C.EVP_PKEY_free(k)
    return ok
