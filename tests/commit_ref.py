"""Python restatement (test infrastructure) of the commit checks the IBC
07-tendermint light client runs -- tendermint v0.33.4 types/validator_set.go
VerifyCommit and VerifyCommitTrusting, reached from
x/ibc/07-tendermint/update.go:88 (lite2 Verify -> VerifyAdjacent /
VerifyNonAdjacent) and misbehaviour.go:88-97 -- one signature at a time, in
the reference's loop order, each signature checked with the ed25519 oracle
(oracle/ed25519_ref.py: go1.14 crypto/ed25519.Verify; tendermint's
PubKeyEd25519.VerifyBytes rejects signatures that are not 64 bytes first).

The tendermint module is not in /root/reference (go.mod dependency
github.com/tendermint/tendermint v0.33.4), so the loops are restated from its
published source; `vote_sign_bytes` lays out a CanonicalVote the way
tendermint's amino codec does (length-prefixed struct: type, fixed64 height
and round, block id, timestamp, chain id) -- parity of that encoding is
unpinned (no amino here), and the hook under test takes the sign bytes from
its caller, so the verdict logic does not depend on it.

Commit layout used by the tests (and gvhost.HostApp.verify_commits):
  vals = [(pub32, addr20, power)], sigs = [(flag, addr20, sig, sign_bytes)],
  flag 1 absent, 2 commit (tallied), 3 nil (verified, not tallied).
"""
import hashlib
import struct

from oracle import ed25519_ref as E

ABSENT, COMMIT, NIL = 1, 2, 3


def address(pub32: bytes) -> bytes:
    """tendermint crypto/ed25519 PubKeyEd25519.Address: SHA256(pub)[:20]."""
    return hashlib.sha256(pub32).digest()[:20]


def _uvarint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _uvarint(num << 3 | wire) + payload


def vote_sign_bytes(chain_id: str, height: int, round_: int, block_hash: bytes, parts_total: int, parts_hash: bytes,
                    ts_seconds: int, ts_nanos: int, for_block: bool) -> bytes:
    """CanonicalVote{Type: Precommit, Height, Round, BlockID, Timestamp, ChainID}
    (types/canonical.go), length-prefixed -- see the module note."""
    body = _field(1, 0, _uvarint(2))                                   # SignedMsgType precommit
    if height:
        body += _field(2, 1, struct.pack("<q", height))
    if round_:
        body += _field(3, 1, struct.pack("<q", round_))
    if for_block:
        psh = _field(1, 0, _uvarint(parts_total)) + _field(2, 2, _uvarint(len(parts_hash)) + parts_hash)
        bid = _field(1, 2, _uvarint(len(block_hash)) + block_hash) + _field(2, 2, _uvarint(len(psh)) + psh)
        body += _field(4, 2, _uvarint(len(bid)) + bid)
    ts = _field(1, 0, _uvarint(ts_seconds)) + (_field(2, 0, _uvarint(ts_nanos)) if ts_nanos else b"")
    body += _field(5, 2, _uvarint(len(ts)) + ts)
    cid = chain_id.encode()
    body += _field(6, 2, _uvarint(len(cid)) + cid)
    return _uvarint(len(body)) + body


def _verify_bytes(pub32: bytes, msg: bytes, sig: bytes) -> bool:
    """tendermint crypto/ed25519 PubKeyEd25519.VerifyBytes."""
    if len(sig) != 64:
        return False
    return E.verify(pub32, msg, sig)


def verify_commit(vals, sigs, basic_ok=True):
    """VerifyCommit: size check, verifyCommitBasic, then every present
    signature (validator i signs signature i) verified in order; +2/3 of the
    total power must be tallied from commit-flagged signatures."""
    if len(vals) != len(sigs):
        return ("size", -1, -1, 0, 0)
    if not basic_ok:
        return ("basic", -1, -1, 0, 0)
    total = sum(v[2] for v in vals)
    needed = total * 2 // 3
    tallied = 0
    for idx, (flag, _addr, sig, msg) in enumerate(sigs):
        if flag == ABSENT:
            continue
        pub, _, power = vals[idx]
        if not _verify_bytes(pub, msg, sig):
            return ("wrong_sig", idx, -1, tallied, needed)
        if flag == COMMIT:
            tallied += power
    if tallied <= needed:
        return ("not_enough", -1, -1, tallied, needed)
    return ("ok", -1, -1, tallied, needed)


def verify_commit_trusting(vals, sigs, num=1, den=3, basic_ok=True):
    """VerifyCommitTrusting: trust level in [1/3, 1] (else the reference
    panics), verifyCommitBasic, then validators looked up by address, a
    repeated validator is a double vote, unknown ones are skipped, and the
    loop returns as soon as more than total * num / den is tallied."""
    if den <= 0 or num * 3 < den or num > den:
        return ("bad_trust", -1, -1, 0, 0)
    if not basic_ok:
        return ("basic", -1, -1, 0, 0)
    total = sum(v[2] for v in vals)
    needed = total * num // den
    by_addr = {v[1]: i for i, v in enumerate(vals)}
    seen = {}
    tallied = 0
    for idx, (flag, addr, sig, msg) in enumerate(sigs):
        if flag == ABSENT:
            continue
        vi = by_addr.get(addr, -1)
        if vi in seen:
            return ("double_vote", seen[vi], idx, tallied, needed)
        if vi < 0:
            continue
        seen[vi] = idx
        pub, _, power = vals[vi]
        if not _verify_bytes(pub, msg, sig):
            return ("wrong_sig", idx, -1, tallied, needed)
        if flag == COMMIT:
            tallied += power
        if tallied > needed:
            return ("ok", -1, -1, tallied, needed)
    return ("not_enough", -1, -1, tallied, needed)
