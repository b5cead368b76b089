"""Gas of the batch decorator equals the reference's signer-by-signer loop.

The reference's SigVerificationDecorator reads signer i's account (a
gas-metered KV read, types/context.go:211-212, store/gaskv/store.go:36-43)
only after signers 0..i-1 verified, and returns at the first failure
(x/auth/ante/sigverify.go:194-213).  The batch decorator verifies every
signer's leaves at once, so it must still charge the reads in that order and
stop where the loop stops -- otherwise a tx whose first signature fails is
charged for reads the reference never made, and a tx near its gas limit ends
with ErrOutOfGas instead of ErrUnauthorized.

Every result of the C++ mirror (libgvhost) is compared with tests/ante_ref.py,
a Python restatement of the chain that charges each read where the reference
makes it.  Multi-signer txs are bank MsgMultiSends with 2 and 3 inputs
(ante_test.go:416-464's shape); fee gas limits are set to the reference's
consumption, one below it, and just above the consumption of a tx that fails
at its first signer.
"""
import pytest

import gpuverify as gvm
import gvhost
import txkit as T
from ante_ref import AnteRef, account_value_len

CHAIN = "gv-gas"
SINK = b"\x07" * 20


class Key:
    def __init__(self, i):
        self.priv = T.privkey_from_secret(b"gas-key-" + bytes([i]))
        self.pub = T.amino_secp(T.secp_pubkey(self.priv))
        self.addr = T.address(self.pub)


KEYS = [Key(i) for i in range(6)]


def setup(ver=None, with_pub=True, height=3):
    app = gvhost.HostApp(ver, chain_id=CHAIN, height=height)
    ref = AnteRef(CHAIN, height=height)
    for i, k in enumerate(KEYS):
        pub = k.pub if with_pub else b""
        app.set_account(k.addr, 10 + i, 4 + i, pub)
        ref.set_account(k.addr, 10 + i, 4 + i, pub)
    return app, ref


def multisend(keys, gas, bad=(), memo="", supply_pub=False, ref=None):
    msgs = [T.MsgMultiSend([(k.addr, [(5, "stake")]) for k in keys], [(SINK, [(5 * len(keys), "stake")])])]
    fee = T.Fee([(0, "stake")], gas)
    sigs = []
    for j, k in enumerate(keys):
        acc = ref.accounts[k.addr]
        sb = T.std_sign_bytes(CHAIN, acc.number, acc.sequence, fee, msgs, memo)
        sig = T.secp_sign(k.priv, sb)
        if j in bad:
            sig = sig[:7] + bytes([sig[7] ^ 0x40]) + sig[8:]
        sigs.append((k.pub if supply_pub else b"", sig))
    return msgs, fee, memo, sigs


def run_both(app, ref, parts):
    msgs, fee, memo, sigs = parts
    tx = T.std_tx(msgs, fee, memo, sigs)
    rc, r = app.ante(tx)
    assert rc == 0
    want = ref.ante(msgs, fee, memo, sigs, len(tx))
    assert (r["code"], r["log"], r["gas_used"]) == want, (r, want)
    return want


def test_account_value_and_params_lengths():
    # proto std.Account{BaseAccount}: 22 B address field + optional pub / number / sequence fields
    assert account_value_len(b"", 0, 0) == 24
    assert account_value_len(b"\x00" * 38, 0, 0) == 64
    assert account_value_len(b"\x00" * 38, 127, 128) == 69


def test_failures_before_verification_cpu():
    """No secp256k1 leaf is verified on these paths (no verifier attached)."""
    app, ref = setup(None)
    for parts in (multisend(KEYS[:2], 200000, memo="m" * 257, ref=ref),       # ErrMemoTooLarge
                  multisend(KEYS[:2], 2000, ref=ref)):                         # out of gas in the params reads
        code, _, _ = run_both(app, ref, parts)
        assert code in (11, 12)
    # an unknown signer supplying its key: SetPubKey's read finds no account
    stranger = Key(99)
    ref.accounts.pop(stranger.addr, None)
    msgs = [T.MsgSend(stranger.addr, SINK, [(1, "stake")])]
    fee = T.Fee([(0, "stake")], 200000)
    code, _, _ = run_both(app, ref, (msgs, fee, "", [(stranger.pub, b"\x01" * 64)]))
    assert code == 9


def test_sign_bytes_panic_precedes_key_checks_in_restatement():
    """sigverify.go:194-207 computes signer i's sign bytes right after its
    (metered) account read and before the nil-key check: a Msg whose
    GetSignBytes panics ends the tx in ErrPanic at the first signer, charged
    for the chain's reads up to that account read.  The Go decorator keeps that
    order (batch_sigverify.go: sign bytes before the nil-key check, also under
    simulate); the restatement does too.  The mirror decodes only MsgSend /
    MsgMultiSend, whose sign bytes cannot panic, so this is a restatement-level
    check of the ordering the Go drop-in follows."""
    from ante_ref import Panic
    app, ref = setup(None, with_pub=True)
    parts = multisend(KEYS[:2], 200000, ref=ref)
    msgs, fee, memo, sigs = parts
    ok_code, _, ok_gas = ref.ante(msgs, fee, memo, sigs, 400)
    assert ok_code == 0

    calls = []

    def panicking(*a):
        calls.append(a)
        raise Panic("json: unsupported value")

    app, ref = setup(None, with_pub=True)
    ref.sign_bytes = panicking
    code, log, gas = ref.ante(msgs, fee, memo, sigs, 400)
    assert (code, log) == (111222, "json: unsupported value: panic")
    assert len(calls) == 1                      # the first signer's, right after its account read
    assert gas < ok_gas
    # nothing applied: sequences unchanged
    assert all(ref.accounts[k.addr].sequence == 4 + i for i, k in enumerate(KEYS))
    # the first signer's key missing from its account: the decorator chain
    # stops in SigGasConsume before any sign bytes are built
    calls.clear()
    app, ref = setup(None, with_pub=True)
    ref.sign_bytes = panicking
    ref.accounts[KEYS[0].addr].pub = b""
    # (in the full chain SigGasConsume rejects the nil key first: sigverify.go:342)
    code, _, _ = ref.ante(msgs, fee, memo, sigs, 400)
    assert code == 8 and not calls[1:]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_multi_signer_gas_follows_reference_order(n):
    with gvm.Verifier([0]) as ver:
        app, ref = setup(ver)
        keys = KEYS[:n]
        used = {}
        for bad in [()] + [(j,) for j in range(n)]:
            code, log, gas = run_both(app, ref, multisend(keys, 10 ** 6, bad=bad, ref=ref))
            assert code == (0 if not bad else 4)
            used[bad] = gas
        # failing at signer j skips the reads of signers j+1.. : strictly increasing in j
        fails = [used[(j,)] for j in range(n)]
        assert fails == sorted(fails) and len(set(fails)) == n
        # gas limits: exactly the reference's consumption passes, one less runs out of gas
        ok_gas = used[()]
        code, log, gas = run_both(app, ref, multisend(keys, ok_gas, ref=ref))
        assert code == 0 and gas == ok_gas
        code, log, gas = run_both(app, ref, multisend(keys, ok_gas - 1, ref=ref))
        assert code == 11
        # a limit just above a first-signer failure: the reference stops at
        # signer 0 (ErrUnauthorized); reading every signer first would run out
        code, log, gas = run_both(app, ref, multisend(keys, used[(0,)], bad=(0,), ref=ref))
        assert code == 4 and gas == used[(0,)]
        code, log, gas = run_both(app, ref, multisend(keys, used[(0,)] + 1, bad=(0,), ref=ref))
        assert code == 4
        app.close()


@pytest.mark.gpu
def test_set_pubkey_writes_and_sequence_writes_are_charged():
    """Accounts without a stored key: SetPubKey reads and writes each
    signer's account; a failing tx rolls the key back (runTx cache-wrap)."""
    with gvm.Verifier([0]) as ver:
        app, ref = setup(ver, with_pub=False)
        keys = KEYS[:3]
        code, _, gas_bad = run_both(app, ref, multisend(keys, 10 ** 6, bad=(1,), supply_pub=True, ref=ref))
        assert code == 4
        assert app.get_account(keys[0].addr)["pub"] == b""            # rolled back
        code, _, gas_ok = run_both(app, ref, multisend(keys, 10 ** 6, supply_pub=True, ref=ref))
        assert code == 0 and gas_ok > gas_bad
        assert app.get_account(keys[2].addr)["pub"] == keys[2].pub
        # next tx: keys stored, none supplied; sequences moved by one
        code, _, _ = run_both(app, ref, multisend(keys, 10 ** 6, ref=ref))
        assert code == 0 and app.get_account(keys[1].addr)["sequence"] == ref.accounts[keys[1].addr].sequence
        app.close()


@pytest.mark.gpu
def test_block_path_gas_matches_per_tx_reference():
    """DeliverBlock (PreVerifyTxs + the ante loop, memoised plans) charges the
    same gas as the per-tx restatement, failures at every signer position."""
    with gvm.Verifier([0]) as ver:
        app, ref = setup(ver)
        txs, want = [], []
        shapes = [(KEYS[:2], ()), (KEYS[2:5], (1,)), (KEYS[:3], (0,)), (KEYS[3:5], ()), (KEYS[:3], (2,)),
                  (KEYS[2:5], ())]
        for keys, bad in shapes:
            parts = multisend(keys, 10 ** 6, bad=bad, ref=ref)
            tx = T.std_tx(*parts)
            txs.append(tx)
            want.append(ref.ante(*parts, len(tx)))
        rc, res = app.deliver_block(txs)
        assert rc == 0
        assert [(r["code"], r["log"], r["gas_used"]) for r in res] == want
        app.close()
