"""CPU tests of libgvhost's DefaultTxDecoder restatement (amino binary StdTx,
x/auth/types/stdtx.go:321-338) and of StdTx.GetSignBytes over the decoded tx.

Encodings come from txkit.std_tx (an independent Python restatement of the
go-amino v0.15.1 encoder).  Pins: the amino registered-name prefixes
reproduce crypto/encode_test.go:58-59; the sign bytes equal the Python
StdSignBytes restatement, itself pinned by x/auth/types/stdtx_test.go:53 and
x/bank/types/msgs_test.go:61,227 (tests/test_oracle.py).  The reference holds
no amino StdTx byte fixtures, so malformed-input error TEXT is parity-unpinned
(the code, ErrTxDecode = 2, is what the tests assert).
"""
import pytest

import gvhost
import txkit as T

A, B, C = b"\x01" * 20, b"\x02" * 20, b"\x03" * 20
FEE = T.Fee([(150, "atom")], 200000)


def sb(tx, chain="c", accnum=3, seq=7):
    return gvhost.tx_sign_bytes(tx, chain, accnum, seq)


def test_prefixes_match_reference_pins():
    assert T.amino_prefix("tendermint/PubKeySecp256k1").hex() == "eb5ae987"            # crypto/encode_test.go:58
    assert T.amino_prefix("tendermint/PubKeyMultisigThreshold").hex() == "22c1f7e2"    # crypto/encode_test.go:59


@pytest.mark.parametrize("memo", ["", "memo", 'a<b>&"\\\n é ', "x" * 256])
def test_msgsend_sign_bytes(memo):
    msgs = [T.MsgSend(A, B, [(10, "atom"), (3, "foo")])]
    tx = T.std_tx(msgs, FEE, memo, [(b"", b"\x00" * 64)])
    assert sb(tx) == T.std_sign_bytes("c", 3, 7, FEE, msgs, memo)


def test_multisend_multiple_msgs_and_empty_fee():
    msgs = [T.MsgMultiSend([(A, [(5, "atom")]), (B, [(6, "atom")])], [(C, [(11, "atom")])]),
            T.MsgSend(C, A, [(1, "x")])]
    fee = T.Fee([], 0)
    tx = T.std_tx(msgs, fee, "", [(b"", b"\x00" * 64)] * 3)
    got = sb(tx, "chain-Ω", 0, 0)
    assert got == T.std_sign_bytes("chain-Ω", 0, 0, fee, msgs, "")
    assert b'"fee":{"amount":[],"gas":"0"}' in got                  # StdFee.Bytes normalises [] (stdtx.go:47-58)


def _coin_tx(amount_text: bytes):
    coin = T.amino_bytes_field(1, b"atom") + T.amino_bytes_field(2, amount_text)
    msg = T.PREFIX_MSGSEND + T.amino_bytes_field(1, A) + T.amino_bytes_field(2, B) + T.amino_bytes_field(3, coin)
    return T.PREFIX_STDTX + T.amino_bytes_field(1, msg) + T.amino_bytes_field(2, FEE.amino())


@pytest.mark.parametrize("text,want", [
    (b"10", "10"), (b"+10", "10"), (b"-5", "-5"), (b"-0", "0"), (b"007", "7"), (b"0x1F", "31"), (b"0X1f", "31"),
    (b"0b101", "5"), (b"0o17", "15"), (b"1_000", "1000"), (b"0_7", "7"), (b"0", "0"),
    (str(2**255 - 1).encode(), str(2**255 - 1)), (b"-" + str(2**255 - 1).encode(), "-" + str(2**255 - 1)),
])
def test_sdk_int_amounts_canonicalised(text, want):
    """sdk.Int amino bytes are big.Int.UnmarshalText (base 0) text; the sign bytes print the decimal."""
    got = sb(_coin_tx(text))
    assert b'"amount":[{"amount":"%s","denom":"atom"}]' % want.encode() in got


@pytest.mark.parametrize("text", [b"08", b"0x", b"_1", b"1_", b"1__0", b"12a", b"-", b"0b2", b" 1",
                                  str(2**255).encode()])
def test_sdk_int_rejects(text):
    with pytest.raises(ValueError):
        sb(_coin_tx(text))


def test_malformed_txs_do_not_decode():
    good = T.std_tx([T.MsgSend(A, B, [(1, "a")])], FEE, "m", [(b"", b"\x00" * 64)])
    sb(good)
    bad = [
        b"",                                              # "tx bytes are empty"
        b"\x00\x01\x02\x03" + good[4:],                   # wrong registered prefix
        good[:-1],                                        # truncated
        good[:4] + T.amino_bytes_field(2, FEE.amino()) + T.amino_bytes_field(1, good[6:6]),   # field 1 after 2
        good[:4] + T.amino_bytes_field(1, b"\xde\xad\xbe\xef"),                              # unregistered msg
        good[:4] + T.uvarint((2 << 3) | 0) + T.uvarint(5),                                  # wrong typ3 for Fee
        good + T.amino_bytes_field(3, b""),                                                 # Signatures after Memo
    ]
    for b in bad:
        with pytest.raises(ValueError):
            sb(b)


def test_unknown_trailing_field_is_consumed():
    """go-amino consumes unknown fields after the last known one."""
    good = T.std_tx([T.MsgSend(A, B, [(1, "a")])], FEE, "m", [(b"", b"\x00" * 64)])
    assert sb(good + T.uvarint((9 << 3) | 0) + T.uvarint(12345)) == sb(good)


def test_disambiguation_bytes_accepted():
    """An interface value may carry 0x00 + 3 disambiguation bytes before its prefix."""
    import hashlib
    h = hashlib.sha256(b"cosmos-sdk/MsgSend").digest()
    i = 0
    while h[i] == 0:
        i += 1
    dis = h[i:i + 3]
    m = T.MsgSend(A, B, [(2, "z")])
    body = m.amino()[4:]
    tx = T.PREFIX_STDTX + T.amino_bytes_field(1, b"\x00" + dis + T.PREFIX_MSGSEND + body) + \
        T.amino_bytes_field(2, FEE.amino())
    assert sb(tx) == T.std_sign_bytes("c", 3, 7, FEE, [m], "")
    bad = T.PREFIX_STDTX + T.amino_bytes_field(1, b"\x00\x00\x00\x00" + T.PREFIX_MSGSEND + body)
    with pytest.raises(ValueError):
        sb(bad)


def test_undecodable_tx_gets_err_tx_decode():
    app = gvhost.HostApp(None)
    for tx in (b"", b"\x01\x02", T.PREFIX_STDTX + b"\xff"):
        rc, r = app.ante(tx)
        assert rc == 0 and r["code"] == 2 and r["codespace"] == "sdk" and r["log"].endswith(": tx parse error")


def test_pipelined_replay_without_gpu_work():
    """gvh_deliver_blocks on blocks that never reach a signature (undecodable
    txs, unknown signers) runs on the CPU alone and returns the codes of
    delivering the blocks one by one; a block that does need the GPU reports
    GVH_ENOVERIFIER instead of a verdict."""
    app = gvhost.HostApp(None)
    m = T.MsgSend(A, B, [(1, "x")])
    unknown = T.std_tx([m], FEE, "", [(b"", b"\x00" * 64)])
    blocks = [[b"", unknown, b"\x01\x02"], [unknown], [], [T.PREFIX_STDTX + b"\xff", unknown]]
    rc, codes = app.deliver_blocks(blocks)
    assert rc == 0
    one = [list(app.deliver_block_codes(b)[1]) for b in blocks]
    assert [list(c) for c in codes] == one
    assert one[0] == [2, 9, 2] and one[3] == [2, 9]
    app.set_account(A, 1, 0, T.amino_secp(bytes([2]) + bytes(range(1, 33))))
    rc, _ = app.deliver_blocks([[unknown], [unknown]])
    assert rc == gvhost.GVH_ENOVERIFIER
    app.close()
