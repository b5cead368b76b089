"""txkit.py -- client-side transaction kit for the host mirror and benchmarks.

Builds what a Cosmos SDK client produces (the reference's client/keyring side,
out of the GPU path): amino pubkey / multisig encodings, bank MsgSend /
MsgMultiSend (amino binary + sign-bytes JSON), StdFee, signatures, and the
amino binary StdTx a node receives (DefaultTxEncoder, x/auth/types/stdtx.go),
which libgvhost decodes (host/gvhost.h).  An independent Python restatement of
the go-amino v0.15 binary encoding (registered-name prefixes, field keys,
unpacked lists, zero values omitted).  Signing uses OpenSSL via
tools/workload/libgvwork.so (secp256k1, low-S) and libcrypto EVP (ed25519);
nothing here is the oracle.

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
_WORK = os.path.join(HERE, "libgvwork.so")

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


def amino_prefix(name: str) -> bytes:
    """go-amino registered-concrete prefix: SHA256(name), skip zero bytes, 3
    disambiguation bytes, skip zero bytes, next 4 bytes."""
    bz = hashlib.sha256(name.encode()).digest()
    while bz[0] == 0:
        bz = bz[1:]
    bz = bz[3:]
    while bz[0] == 0:
        bz = bz[1:]
    return bz[:4]


PREFIX_STDTX = amino_prefix("cosmos-sdk/StdTx")
PREFIX_MSGSEND = amino_prefix("cosmos-sdk/MsgSend")
PREFIX_MULTISEND = amino_prefix("cosmos-sdk/MsgMultiSend")
assert amino_prefix("tendermint/PubKeySecp256k1") == PREFIX_SECP    # crypto/encode_test.go:58


def _opt_bytes(field: int, b: bytes) -> bytes:
    return amino_bytes_field(field, b) if b else b""


def coins_amino(field: int, coins) -> bytes:
    """sdk.Coins as an unpacked list of Coin{Denom 1, Amount 2 (sdk.Int text)}."""
    return b"".join(amino_bytes_field(field, _opt_bytes(1, d.encode()) + _opt_bytes(2, str(a).encode()))
                    for a, d in coins)


class MsgSend:
    """x/bank MsgSend (types.pb.go:30-34, amino name cosmos-sdk/MsgSend)."""

    def __init__(self, frm: bytes, to: bytes, coins):
        self.frm, self.to, self.coins = frm, to, list(coins)

    def json(self) -> str:
        return msg_send_json(self.frm, self.to, self.coins)

    def amino(self) -> bytes:
        return PREFIX_MSGSEND + _opt_bytes(1, self.frm) + _opt_bytes(2, self.to) + coins_amino(3, self.coins)

    def signers(self):
        return [self.frm]


class MsgMultiSend:
    """x/bank MsgMultiSend: inputs / outputs of (address, coins)."""

    def __init__(self, inputs, outputs):
        self.inputs, self.outputs = list(inputs), list(outputs)

    def json(self) -> str:
        io = lambda xs: [{"address": bech32("cosmos", a), "coins": [{"amount": str(x), "denom": d} for x, d in c]}
                         for a, c in xs]
        return sort_json({"type": "cosmos-sdk/MsgMultiSend", "value": {"inputs": io(self.inputs),
                                                                         "outputs": io(self.outputs)}})

    def amino(self) -> bytes:
        io = lambda f, xs: b"".join(amino_bytes_field(f, _opt_bytes(1, a) + coins_amino(2, c)) for a, c in xs)
        return PREFIX_MULTISEND + io(1, self.inputs) + io(2, self.outputs)

    def signers(self):
        return [a for a, _ in self.inputs]


class Fee:
    def __init__(self, coins, gas: int):
        self.coins, self.gas = list(coins), gas

    def json(self) -> str:
        return fee_json(self.coins, self.gas)

    def amino(self) -> bytes:
        return coins_amino(1, self.coins) + (uvarint(2 << 3) + uvarint(self.gas) if self.gas else b"")


def std_tx(msgs, fee: Fee, memo: str, sigs) -> bytes:
    """Amino binary StdTx (DefaultTxEncoder): prefix, Msgs 1 (interfaces), Fee 2,
    Signatures 3 {PubKey 1, Signature 2}, Memo 4.  sigs: (pub_amino or b'', sig)."""
    out = PREFIX_STDTX
    out += b"".join(amino_bytes_field(1, m.amino()) for m in msgs)
    out += amino_bytes_field(2, fee.amino())
    out += b"".join(amino_bytes_field(3, _opt_bytes(1, p) + _opt_bytes(2, s)) for p, s in sigs)
    out += _opt_bytes(4, memo.encode())
    return out


def tx_signers(msgs):
    """StdTx.GetSigners(): msg signers in order, duplicates dropped."""
    out = []
    for m in msgs:
        for a in m.signers():
            if a not in out:
                out.append(a)
    return out


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


def std_sign_bytes(chain_id: str, accnum: int, seq: int, fee, msgs, memo: str) -> bytes:
    """fee: JSON str or Fee; msgs: JSON strs or Msg objects."""
    fee = fee.json() if isinstance(fee, Fee) else fee
    msgs = [m if isinstance(m, str) else m.json() for m in msgs]
    doc = {"account_number": str(accnum), "chain_id": chain_id, "fee": json.loads(fee), "memo": memo,
           "msgs": [json.loads(m) for m in msgs], "sequence": str(seq)}
    return sort_json(doc).encode()
