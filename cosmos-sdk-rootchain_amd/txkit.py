"""txkit.py -- client-side transaction kit for the host mirror and benchmarks.

Builds what a Cosmos SDK client produces (the reference's client/keyring side,
out of the GPU path): amino pubkey / multisig encodings, MsgSend sign bytes,
StdFee JSON, signatures, and the flat decoded-tx encoding that libgvhost
accepts (host/gvhost.h).  Signing uses OpenSSL via tools/workload/libgvwork.so
(secp256k1, low-S) and libcrypto EVP (ed25519); nothing here is the oracle.

Formats (reference pins): amino prefixes crypto/encode_test.go:51-60
(secp256k1 EB5AE987/0x21, multisig 22C1F7E2); MsgSend sign bytes
x/bank/types/msgs_test.go:61; StdSignBytes x/auth/types/stdtx_test.go:53;
Multisignature / CompactBitArray: tendermint v0.33.4 crypto/multisig (SURVEY.md
Appendix B).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import hashlib
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
_WORK = os.path.join(REPO, "tools", "workload", "libgvwork.so")

PREFIX_SECP = bytes.fromhex("eb5ae987")
PREFIX_ED = bytes.fromhex("1624de64")
PREFIX_MULTI = bytes.fromhex("22c1f7e2")
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141

_w = None
_crypto = None


def _work():
    global _w
    if _w is None:
        if not os.path.exists(_WORK):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.dirname(_WORK)], check=True)
        _w = ctypes.CDLL(_WORK)
        _w.gvw_pubkey.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
        _w.gvw_sign_digest.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
    return _w


def _libcrypto():
    global _crypto
    if _crypto is None:
        L = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
        vp = ctypes.c_void_p
        L.EVP_PKEY_new_raw_private_key.restype = vp
        L.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, vp, ctypes.c_char_p, ctypes.c_size_t]
        L.EVP_PKEY_get_raw_public_key.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_size_t)]
        L.EVP_MD_CTX_new.restype = vp
        L.EVP_DigestSignInit.argtypes = [vp, vp, vp, vp, vp]
        L.EVP_DigestSign.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
        L.EVP_MD_CTX_free.argtypes = [vp]
        L.EVP_PKEY_free.argtypes = [vp]
        _crypto = L
    return _crypto


# ------------------------------------------------------------------- keys
def privkey_from_secret(secret: bytes) -> bytes:
    """tendermint GenPrivKeySecp256k1: (SHA256(secret) mod (n-1)) + 1."""
    fe = int.from_bytes(hashlib.sha256(secret).digest(), "big")
    return (fe % (N - 1) + 1).to_bytes(32, "big")


def secp_pubkey(priv: bytes) -> bytes:
    out = ctypes.create_string_buffer(33)
    assert _work().gvw_pubkey(priv, out) == 0
    return out.raw


def secp_sign(priv: bytes, msg: bytes) -> bytes:
    """tendermint PrivKeySecp256k1.Sign(msg): ECDSA over SHA256(msg), low-S, R||S."""
    out = ctypes.create_string_buffer(64)
    assert _work().gvw_sign_digest(priv, hashlib.sha256(msg).digest(), out) == 0
    return out.raw


def ed25519_keypair(seed: bytes):
    L = _libcrypto()
    k = L.EVP_PKEY_new_raw_private_key(1087, None, seed, 32)   # NID_ED25519
    pub = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    L.EVP_PKEY_get_raw_public_key(k, pub, ctypes.byref(n))
    L.EVP_PKEY_free(k)
    return seed, pub.raw


def ed25519_sign(seed: bytes, msg: bytes) -> bytes:
    L = _libcrypto()
    k = L.EVP_PKEY_new_raw_private_key(1087, None, seed, 32)
    c = L.EVP_MD_CTX_new()
    assert L.EVP_DigestSignInit(c, None, None, None, k) == 1
    sig = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(64)
    assert L.EVP_DigestSign(c, sig, ctypes.byref(n), msg, len(msg)) == 1
    L.EVP_MD_CTX_free(c)
    L.EVP_PKEY_free(k)
    return sig.raw


# ------------------------------------------------------------------ amino
def uvarint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def amino_bytes_field(field: int, b: bytes) -> bytes:
    return uvarint((field << 3) | 2) + uvarint(len(b)) + b


def amino_secp(pub33: bytes) -> bytes:
    return PREFIX_SECP + uvarint(33) + pub33


def amino_ed25519(pub32: bytes) -> bytes:
    return PREFIX_ED + uvarint(32) + pub32


def amino_multisig(k: int, pubs_amino) -> bytes:
    body = (uvarint(1 << 3) + uvarint(k) if k else b"") + b"".join(amino_bytes_field(2, p) for p in pubs_amino)
    return PREFIX_MULTI + body


def compact_bit_array(bits) -> bytes:
    n = len(bits)
    elems = bytearray((n + 7) // 8)
    for i, b in enumerate(bits):
        if b:
            elems[i >> 3] |= 1 << (7 - (i % 8))
    extra = n % 8
    body = (uvarint(1 << 3) + uvarint(extra) if extra else b"") + (amino_bytes_field(2, bytes(elems)) if elems else b"")
    return body


def multisignature(bits, sigs) -> bytes:
    """tendermint multisig.Multisignature amino binary (BitArray field 1, Sigs field 2)."""
    return amino_bytes_field(1, compact_bit_array(bits)) + b"".join(amino_bytes_field(2, s) for s in sigs)


def address(pub_amino: bytes) -> bytes:
    """crypto.PubKey.Address() for an amino-encoded key (computed by libgvhost:
    Python's hashlib has no RIPEMD-160 in this image)."""
    import gvhost
    return gvhost.pubkey_address(pub_amino)


# ------------------------------------------------------------ sign bytes
def sort_json(obj) -> str:
    s = json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=False)
    s = s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
    return s.replace("\u2028", "\\u2028").replace("\u2029", "\\u2029")   # Go escapes U+2028/9 too


def bech32(hrp: str, data: bytes) -> str:
    cs = "qpzry9x8gf2tvdw0s3jn54khce6mua7l"
    acc = bits = 0
    five = []
    for b in data:
        acc = (acc << 8) | b
        bits += 8
        while bits >= 5:
            bits -= 5
            five.append((acc >> bits) & 31)
    if bits:
        five.append((acc << (5 - bits)) & 31)
    gen = [0x3B6A57B2, 0x26508E6D, 0x1EA119FA, 0x3D4233DD, 0x2A1462B3]
    chk = 1
    for v in [ord(c) >> 5 for c in hrp] + [0] + [ord(c) & 31 for c in hrp] + five + [0] * 6:
        top = chk >> 25
        chk = (chk & 0x1FFFFFF) << 5 ^ v
        for i in range(5):
            chk ^= gen[i] if (top >> i) & 1 else 0
    chk ^= 1
    return hrp + "1" + "".join(cs[d] for d in five + [(chk >> 5 * (5 - i)) & 31 for i in range(6)])


def msg_send_json(frm: bytes, to: bytes, coins) -> str:
    return sort_json({"type": "cosmos-sdk/MsgSend", "value": {
        "amount": [{"amount": str(a), "denom": d} for a, d in coins],
        "from_address": bech32("cosmos", frm), "to_address": bech32("cosmos", to)}})


def fee_json(coins, gas: int) -> str:
    return sort_json({"amount": [{"amount": str(a), "denom": d} for a, d in coins], "gas": str(gas)})


def std_sign_bytes(chain_id: str, accnum: int, seq: int, fee: str, msgs, memo: str) -> bytes:
    doc = {"account_number": str(accnum), "chain_id": chain_id, "fee": json.loads(fee), "memo": memo,
           "msgs": [json.loads(m) for m in msgs], "sequence": str(seq)}
    return sort_json(doc).encode()


# --------------------------------------------------------------- flat tx
def flat_tx(msgs, fee: str, memo: str, signers, sigs) -> bytes:
    """sigs: list of (pub_amino or b'', signature bytes)."""
    def blob(b: bytes) -> bytes:
        return struct.pack("<I", len(b)) + b
    out = struct.pack("<I", len(msgs)) + b"".join(blob(m.encode()) for m in msgs)
    out += blob(fee.encode()) + blob(memo.encode())
    out += struct.pack("<I", len(signers)) + b"".join(signers)
    out += struct.pack("<I", len(sigs)) + b"".join(blob(p) + blob(s) for p, s in sigs)
    return out
