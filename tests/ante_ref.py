"""Python restatement of the reference ante chain (x/auth/ante/ante.go:13-31)
for the C++ mirror's tests: the result (code, log) and the gas of one StdTx,
with every charge made where the reference makes it.  Test infrastructure
only (the checker, never the product path).

Gas charged, in chain order (SetUpContext's meter: the tx's fee gas, or
infinite at height 0 -- x/auth/ante/setup.go:67-76):

  ValidateMemo       GetParams                              basic.go:61-77
  ConsumeTxSize      GetParams; 10 x len(txBytes)           basic.go:98-148
  SetPubKey          per tx-supplied key: account read, + write if the key is stored   sigverify.go:60-99
  ValidateSigCount   GetParams                              sigverify.go:275-294
  DeductFee          the fee payer's account read           fee.go:84-108 (zero fees only)
  SigGasConsume      GetParams; per signer: account read + DefaultSigVerificationGasConsumer
                                                            sigverify.go:117-153, 299-338
  SigVerification    per signer, in order, until the first failure: account read   sigverify.go:170-216
  IncrementSequence  per signer: account read + write       sigverify.go:237-259

An account read is gaskv Get: 1000 + 3 x len(value); a write is Set: 2000 +
30 x len(value) (store/gaskv/store.go:36-52, store/types/gas.go:165-173).
The value is proto std.Account{BaseAccount} (std/codec.go:41-48,
x/auth/types/types.proto:11-19).  GetParams = five Gets of amino-JSON uint64
values (x/params/types/subspace.go:100-109,218-222; x/auth/types/params.go:55-62).
Signature verdicts come from the oracle (secp256k1) and oracle.ed25519_ref.
Absolute gas is parity-unpinned (no Go toolchain runs the reference); the
ORDER of the charges is what this restatement exists to check.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import txkit as T                       # noqa: E402
from oracle import oracle as O          # noqa: E402
from oracle import ed25519_ref as ED    # noqa: E402

READ_FLAT, READ_BYTE, WRITE_FLAT, WRITE_BYTE = 1000, 3, 2000, 30
TX_SIZE_COST, MAX_MEMO = 10, 256
PFX_SECP, PFX_ED, PFX_MULTI = bytes.fromhex("eb5ae987"), bytes.fromhex("1624de64"), bytes.fromhex("22c1f7e2")
SIM_PUB = bytes.fromhex("eb5ae98721035ad6810a47f073553ff30d2fcc7e0d3b1c0b74b61a1aaa2582344037151e143a")
ERR_DESC = {2: "tx parse error", 4: "unauthorized", 8: "invalid pubkey", 9: "unknown address", 11: "out of gas",
            12: "memo too large", 14: "maximum number of signatures exceeded"}
UNAUTH_MSG = "signature verification failed; verify correct account sequence and chain-id"


class OutOfGas(Exception):
    pass


class Fail(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code, self.msg = code, msg


class Panic(Exception):
    """A reference panic inside the ante chain; runTx recovers it into
    ErrPanic (baseapp/baseapp.go:490-512): code 111222, codespace undefined."""


class Meter:
    def __init__(self, limit):
        self.limit, self.used = limit, 0              # limit None: infinite

    def consume(self, amount, desc):
        self.used += amount
        if self.limit is not None and self.used > self.limit:
            raise OutOfGas(desc)


def uvarint_len(v):
    return len(T.uvarint(v))


def account_value_len(pub: bytes, number: int, seq: int) -> int:
    inner = 2 + 20
    if pub:
        inner += 1 + uvarint_len(len(pub)) + len(pub)
    if number:
        inner += 1 + uvarint_len(number)
    if seq:
        inner += 1 + uvarint_len(seq)
    return 1 + uvarint_len(inner) + inner


def _read_uvarint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def _fields(b):
    """amino/proto binary fields: [(field, wiretype, value)]"""
    i, out = 0, []
    while i < len(b):
        key, i = _read_uvarint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_uvarint(b, i)
        elif wt == 2:
            n, i = _read_uvarint(b, i)
            v, i = b[i:i + n], i + n
            if len(v) != n:
                raise ValueError("truncated")
        else:
            raise ValueError("wire type")
        out.append((f, wt, v))
    return out


def decode_pubkey(amino: bytes):
    """('secp', pub33) | ('ed', pub32) | ('multi', k, [subkeys]); raises on malformed bytes."""
    if amino[:4] == PFX_SECP and len(amino) == 38 and amino[4] == 0x21:
        return ("secp", amino[5:])
    if amino[:4] == PFX_ED and len(amino) == 37 and amino[4] == 0x20:
        return ("ed", amino[5:])
    if amino[:4] == PFX_MULTI:
        k, subs = 0, []
        for f, wt, v in _fields(amino[4:]):
            if f == 1 and wt == 0:
                k = v
            elif f == 2 and wt == 2:
                subs.append(decode_pubkey(v))
            else:
                raise ValueError("multisig field")
        return ("multi", k, subs)
    raise ValueError("unknown pubkey")


def decode_multisig(sig: bytes):
    """tendermint multisig.Multisignature: (bit list, [sigs])"""
    bits, sigs = [], []
    for f, wt, v in _fields(sig):
        if f == 1 and wt == 2:
            extra, elems = 0, b""
            for g, wt2, w in _fields(v):
                if g == 1 and wt2 == 0:
                    extra = w
                elif g == 2 and wt2 == 2:
                    elems = w
            size = 8 * len(elems) if extra == 0 else 8 * (len(elems) - 1) + extra
            bits = [bool(elems[i // 8] >> (7 - i % 8) & 1) for i in range(size)]
        elif f == 2 and wt == 2:
            sigs.append(v)
        else:
            raise ValueError("multisignature field")
    return bits, sigs


def verify_bytes(pk, msg: bytes, sig: bytes) -> bool:
    """crypto.PubKey.VerifyBytes for secp256k1 / ed25519 / multisig threshold keys"""
    if pk[0] == "secp":
        return len(sig) == 64 and O.verify_bytes(pk[1], msg, sig)
    if pk[0] == "ed":
        return len(sig) == 64 and ED.verify(pk[1], msg, sig)
    _, k, subs = pk
    try:
        bits, sigs = decode_multisig(sig)
    except Exception:
        return False
    size = len(bits)
    if len(subs) != size or len(sigs) < k or len(sigs) > size or sum(bits) < k:
        return False
    j = 0
    for i, b in enumerate(bits):
        if b:
            if not verify_bytes(subs[i], msg, sigs[j]):
                return False
            j += 1
    return True


class Account:
    def __init__(self, number, sequence=0, pub=b""):
        self.number, self.sequence, self.pub = number, sequence, pub

    def value_len(self):
        return account_value_len(self.pub, self.number, self.sequence)


class AnteRef:
    def __init__(self, chain_id, height=1, recheck=False, gas_limit=0, sig_limit=7, cost_secp=1000, cost_ed=590):
        self.chain_id, self.height, self.recheck, self.gas_limit = chain_id, height, recheck, gas_limit
        self.sig_limit, self.cost_secp, self.cost_ed = sig_limit, cost_secp, cost_ed
        self.accounts = {}
        # StdSignBytes (x/auth/types/stdtx.go:292-312); a test may substitute a
        # function that raises Panic (a Msg whose GetSignBytes panics)
        self.sign_bytes = T.std_sign_bytes

    def set_account(self, addr, number, sequence=0, pub=b""):
        self.accounts[addr] = Account(number, sequence, pub)

    # -- gas pieces
    def _params(self, m):
        for v in (MAX_MEMO, self.sig_limit, TX_SIZE_COST, self.cost_ed, self.cost_secp):
            m.consume(READ_FLAT, "ReadFlat")
            m.consume(READ_BYTE * (len(str(v)) + 2), "ReadPerByte")

    def _read(self, m, addr):
        acc = self.accounts.get(addr)
        m.consume(READ_FLAT, "ReadFlat")
        m.consume(READ_BYTE * (acc.value_len() if acc else 0), "ReadPerByte")
        return acc

    def _write(self, m, acc):
        m.consume(WRITE_FLAT, "WriteFlat")
        m.consume(WRITE_BYTE * acc.value_len(), "WritePerByte")

    def _sig_gas(self, m, sig, pk, top):
        if pk[0] == "ed":
            m.consume(self.cost_ed, "ante verify: ed25519")
            if top:
                raise Fail(8, "ED25519 public keys are unsupported")
        elif pk[0] == "secp":
            m.consume(self.cost_secp, "ante verify: secp256k1")
        else:
            bits, sigs = decode_multisig(sig)
            j = 0
            for i, b in enumerate(bits):
                if b:
                    self._sig_gas(m, sigs[j], pk[2][i], False)
                    j += 1

    def ante(self, msgs, fee, memo, sigs, tx_len):
        """(code, log, gas_used) of one tx; state changes applied on success."""
        signers = T.tx_signers(msgs)
        wanted = fee.gas
        infinite = self.gas_limit == 0 and self.height == 0
        m = Meter(None if infinite else (self.gas_limit or wanted))
        saved = {a: (acc.sequence, acc.pub) for a, acc in self.accounts.items()}
        try:
            self._params(m)                                                   # ValidateMemo
            if len(memo.encode()) > MAX_MEMO:
                raise Fail(12, f"maximum number of characters is {MAX_MEMO} but received "
                               f"{len(memo.encode())} characters")
            self._params(m)                                                   # ConsumeTxSize
            m.consume(TX_SIZE_COST * tx_len, "txSize")
            for i, (pub, _) in enumerate(sigs):                                # SetPubKey
                if not pub:
                    continue
                pk = decode_pubkey(pub)
                if T.address(pub) != signers[i]:
                    raise Fail(8, f"pubKey does not match signer address {T.bech32('cosmos', signers[i])} "
                                  f"with signer index: {i}")
                acc = self._read(m, signers[i])
                if acc is None:
                    raise Fail(9, f"account {T.bech32('cosmos', signers[i])} does not exist")
                if not acc.pub:
                    acc.pub = pub
                    self._write(m, acc)
                del pk
            self._params(m)                                                   # ValidateSigCount
            count = 0
            for pub, _ in sigs:
                pk = decode_pubkey(pub) if pub else None
                count += len(pk[2]) if pk and pk[0] == "multi" else 1
                if count > self.sig_limit:
                    raise Fail(14, f"signatures: {count}, limit: {self.sig_limit}")
            if self._read(m, signers[0]) is None:                              # DeductFee
                raise Fail(9, f"fee payer address: {T.bech32('cosmos', signers[0])} does not exist")
            self._params(m)                                                   # SigGasConsume
            for i, (_, sig) in enumerate(sigs):
                acc = self._read(m, signers[i])
                if acc is None:
                    raise Fail(9, f"account {T.bech32('cosmos', signers[i])} does not exist")
                if not acc.pub:
                    raise Fail(8, "unrecognized public key type: <nil>")
                self._sig_gas(m, sig, decode_pubkey(acc.pub), True)
            if not self.recheck:                                               # SigVerification
                if len(sigs) != len(signers):
                    raise Fail(4, f"invalid number of signer;  expected: {len(signers)}, got {len(sigs)}")
                for i, (_, sig) in enumerate(sigs):
                    acc = self._read(m, signers[i])
                    if acc is None:
                        raise Fail(9, f"account {T.bech32('cosmos', signers[i])} does not exist")
                    # sign bytes before the nil-key check (sigverify.go:201-207)
                    accnum = 0 if self.height == 0 else acc.number
                    sb = self.sign_bytes(self.chain_id, accnum, acc.sequence, fee, msgs, memo)
                    if not acc.pub:
                        raise Fail(8, "pubkey on account is not set")
                    if not verify_bytes(decode_pubkey(acc.pub), sb, sig):
                        raise Fail(4, UNAUTH_MSG)
                for a in signers:                                              # IncrementSequence
                    acc = self._read(m, a)
                    acc.sequence += 1
                    self._write(m, acc)
        except Fail as f:
            self._restore(saved)
            return f.code, f"{f.msg}: {ERR_DESC[f.code]}", m.used
        except Panic as p:
            self._restore(saved)
            return 111222, f"{p}: panic", m.used
        except OutOfGas as o:
            self._restore(saved)
            return 11, (f"out of gas in location: {o}; gasWanted: {wanted}, gasUsed: {m.used}: out of gas"), m.used
        return 0, "", m.used

    def _restore(self, saved):
        for a, (seq, pub) in saved.items():
            self.accounts[a].sequence, self.accounts[a].pub = seq, pub
