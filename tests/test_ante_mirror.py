"""Tests of the C++ host mirror of the reference's signature ante path
(libgvhost over libgpuverify), modeled on the reference's own tests:

  x/auth/ante/sigverify_test.go   TestConsumeSignatureVerificationGas (:58-101),
                                  TestSigVerification (:103-160), TestSigIntegration (:162-176)
  x/auth/ante/ante_test.go        TestAnteHandlerSigErrors (:92-138), TestAnteHandlerMultiSigner (:416-464),
                                  TestAnteHandlerBadSignBytes (:466-541), TestAnteHandlerSetPubKey (:543-593),
                                  TestCountSubkeys (:627-659), TestAnteHandlerSigLimitExceeded (:661-698),
                                  TestAnteHandlerReCheck (:747-826)

Tests that never reach a secp256k1 verification run on the CPU (the host app
has no verifier attached and would fail loudly if one were needed); the rest
are marked gpu.
"""
import json
import os

import pytest

import gvhost
import gpuverify as gvm
import txkit as T
from ante_ref import AnteRef

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FEE = T.Fee([(150, "atom")], 200000)
UNAUTH = "signature verification failed; verify correct account sequence and chain-id: unauthorized"


class Key:
    def __init__(self, i):
        self.priv = T.privkey_from_secret(b"ante-key-" + bytes([i]))
        self.pub33 = T.secp_pubkey(self.priv)
        self.pub = T.amino_secp(self.pub33)
        self.addr = T.address(self.pub)

    def sign(self, msg: bytes) -> bytes:
        return T.secp_sign(self.priv, msg)


KEYS = [Key(i) for i in range(10)]


def make_parts(app_chain, signers, accnums, seqs, msgs=None, fee=FEE, memo="", with_pub=True, sign_keys=None):
    """(msgs, fee, memo, sigs) of a StdTx of MsgSends signed by `signers` (Key objects) over their sign bytes."""
    msgs = msgs or [T.MsgSend(s.addr, KEYS[9].addr, [(10, "atom")]) for s in signers]
    sign_keys = sign_keys or signers
    sigs = []
    for k, s, an, sq in zip(sign_keys, signers, accnums, seqs):
        sb = T.std_sign_bytes(app_chain, an, sq, fee, msgs, memo)
        sigs.append((s.pub if with_pub else b"", k.sign(sb)))
    return msgs, fee, memo, sigs


def make_tx(*a, **kw):
    """The amino StdTx bytes of make_parts(...)."""
    return T.std_tx(*make_parts(*a, **kw))


def new_app(verifier=None, chain="gv-test", height=1):
    app = gvhost.HostApp(verifier, chain_id=chain, height=height)
    for i, k in enumerate(KEYS):
        app.set_account(k.addr, i, 0)
    return app


def new_ref(chain="gv-test", height=1, recheck=False):
    """tests/ante_ref.py over new_app's accounts: the reference chain's (code, log, gas)."""
    ref = AnteRef(chain, height=height, recheck=recheck)
    for i, k in enumerate(KEYS):
        ref.set_account(k.addr, i, 0)
    return ref


# ---------------------------------------------------------------- CPU tests
def test_sign_bytes_and_address_goldens():
    sb = json.load(open(os.path.join(REPO, "tests", "golden", "sign_bytes.json")))
    addr = gvhost.bech32_address(KEYS[0].addr)
    got = gvhost.std_sign_bytes("1234", 3, 6, T.fee_json([(150, "atom")], 100000), [json.dumps([addr])], "memo")
    assert got.decode() == sb["std_sign_bytes"]["want_template"] % addr
    assert T.bech32("cosmos", b"input") == "cosmos1d9h8qat57ljhcm"              # msgs_test.go:61
    assert gvhost.bech32_address(KEYS[0].addr) == T.bech32("cosmos", KEYS[0].addr)
    kat = json.load(open(os.path.join(REPO, "tests", "golden", "fundraiser_kat.json")))["vectors"]
    for v in kat[:25]:
        pub = bytes.fromhex(v["pub"])
        assert gvhost.pubkey_address(T.amino_secp(pub)).hex() == v["addr"]


def test_go_json_escaping_in_sign_bytes():
    memo = 'a<b>&"\\\n é'
    got = gvhost.std_sign_bytes("c", 1, 2, FEE.json(), [], memo)
    assert got == T.std_sign_bytes("c", 1, 2, FEE, [], memo)
    assert b"\\u003c" in got and b"\\u2028" in got


def test_consume_signature_verification_gas():
    app = new_app()
    ed_seed, ed_pub = T.ed25519_keypair(b"\x07" * 32)
    r = app.consume_sig_gas(b"", T.amino_ed25519(ed_pub))
    assert r["gas_used"] == 590 and r["code"] == 8 and "ED25519 public keys are unsupported" in r["log"]
    r = app.consume_sig_gas(b"", KEYS[0].pub)
    assert r["gas_used"] == 1000 and r["code"] == 0
    # 5 keys mixing secp256k1 and ed25519, all five bits set (sigverify_test.go:62-69)
    pubs, sigs, expected = [], [], 0
    for i in range(5):
        if i % 2:
            pubs.append(T.amino_ed25519(T.ed25519_keypair(bytes([i]) * 32)[1]))
            expected += 590
        else:
            pubs.append(KEYS[i].pub)
            expected += 1000
        sigs.append(b"\x01" * 64)
    mk = T.amino_multisig(2, pubs)
    r = app.consume_sig_gas(T.multisignature([True] * 5, sigs), mk)
    assert r["code"] == 0 and r["gas_used"] == expected
    r = app.consume_sig_gas(b"", None)
    assert r["code"] == 8 and "unrecognized public key type" in r["log"]
    # malformed multisignature -> MustUnmarshalBinaryBare panics -> ErrPanic
    r = app.consume_sig_gas(b"\xff\xff", mk)
    assert r["code"] == 111222 and r["codespace"] == "undefined"


def test_count_subkeys_and_sig_limit():
    app = new_app()
    # 8 secp256k1 subkeys > TxSigLimit 7 (ante_test.go:661-698)
    mk = T.amino_multisig(2, [k.pub for k in KEYS[:8]])
    maddr = T.address(mk)
    app.set_account(maddr, 20, 0)
    tx = T.std_tx([T.MsgSend(maddr, KEYS[9].addr, [(1, "atom")])], FEE, "",
                  [(mk, T.multisignature([True, True] + [False] * 6, [b"\x00" * 64, b"\x00" * 64]))])
    rc, r = app.ante(tx)
    assert rc == 0 and r["code"] == 14 and r["log"] == "signatures: 8, limit: 7: maximum number of signatures exceeded"
    app.set_params(tx_sig_limit=8)
    rc, r = app.ante(tx)            # now passes the count, fails in verification (structure ok, bad sigs)
    assert rc in (0, gvhost.GVH_ENOVERIFIER)


def test_pubkey_mismatch_and_unknown_account():
    app = new_app()
    tx = make_tx(app_chain="gv-test", signers=[KEYS[0]], accnums=[0], seqs=[0])
    # wrong signer: tx claims KEYS[0]'s address but carries KEYS[1]'s pubkey (ante_test.go:535-540)
    bad = T.std_tx([T.MsgSend(KEYS[0].addr, KEYS[9].addr, [(10, "atom")])], FEE, "", [(KEYS[1].pub, b"\x00" * 64)])
    rc, r = app.ante(bad)
    assert r["code"] == 8 and r["log"].startswith("pubKey does not match signer address " +
                                                  gvhost.bech32_address(KEYS[0].addr) + " with signer index: 0")
    stranger = Key(200)
    tx = T.std_tx([T.MsgSend(stranger.addr, KEYS[9].addr, [(1, "atom")])], FEE, "", [(stranger.pub, b"\x00" * 64)])
    rc, r = app.ante(tx)
    assert r["code"] == 9 and r["log"] == f"account {gvhost.bech32_address(stranger.addr)} does not exist: unknown address"


def test_recheck_and_simulate_skip_verification():
    app = new_app()
    parts = make_parts("gv-test", [KEYS[0]], [0], [0])
    tx = T.std_tx(*parts)
    app.set_context("gv-test", 1, recheck=True)
    rc, r = app.ante(tx)                        # TestAnteHandlerReCheck: verification skipped
    want = new_ref(recheck=True).ante(*parts, len(tx))
    assert rc == 0 and r["code"] == 0 and r["gpu_leaves"] == 0 and r["gas_used"] == want[2]
    assert app.get_account(KEYS[0].addr)["sequence"] == 0          # no increment on ReCheck
    app.set_context("gv-test", 1)
    sim = T.std_tx([T.MsgSend(KEYS[1].addr, KEYS[9].addr, [(1, "atom")])], FEE, "", [(b"", b"")])
    app.set_gas_model(False)                    # signature gas alone: the sim pubkey's charge
    rc, r = app.ante(sim, simulate=True)        # Simulate: sim pubkey for gas, no verification
    assert rc == 0 and r["code"] == 0 and r["gas_used"] == 1000
    app.set_gas_model(True)
    assert app.get_account(KEYS[1].addr)["sequence"] == 1


def test_wrong_number_of_signatures():
    app = new_app()
    msgs = [T.MsgSend(KEYS[0].addr, KEYS[9].addr, [(1, "atom")]), T.MsgSend(KEYS[1].addr, KEYS[9].addr, [(1, "atom")])]
    app.set_account(KEYS[0].addr, 0, 0, KEYS[0].pub)
    tx = T.std_tx(msgs, FEE, "", [(KEYS[0].pub, b"\x00" * 64)])
    rc, r = app.ante(tx)
    assert r["code"] == 4 and r["log"] == "invalid number of signer;  expected: 2, got 1: unauthorized"


def test_multisig_structural_rejects_need_no_gpu():
    app = new_app()
    mk = T.amino_multisig(2, [k.pub for k in KEYS[:3]])
    maddr = T.address(mk)
    app.set_account(maddr, 30, 0)
    msg = [T.MsgSend(maddr, KEYS[9].addr, [(1, "atom")])]
    for bits, nsig in (([True, False, False], 1),          # fewer than K signatures
                       ([True, True, False, False], 2)):    # bit array size != number of keys
        tx = T.std_tx(msg, FEE, "", [(mk, T.multisignature(bits, [b"\x00" * 64] * nsig))])
        rc, r = app.ante(tx)
        assert rc == 0 and r["code"] == 4 and r["log"] == UNAUTH and r["gpu_leaves"] == 0


def test_no_verifier_fails_loudly():
    app = new_app()
    tx = make_tx("gv-test", [KEYS[2]], [2], [0])
    rc, r = app.ante(tx)
    assert rc == gvhost.GVH_ENOVERIFIER


# ---------------------------------------------------------------- GPU tests
@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


@pytest.mark.gpu
def test_sig_verification_cases(ver):
    """TestSigVerification / TestAnteHandlerSigErrors / BadSignBytes."""
    app = new_app(ver)
    parts = make_parts("gv-test", [KEYS[0]], [0], [0])
    ok_tx = T.std_tx(*parts)
    rc, r = app.ante(ok_tx)
    assert rc == 0 and r["code"] == 0 and r["gpu_leaves"] == 1
    assert (r["code"], r["log"], r["gas_used"]) == new_ref().ante(*parts, len(ok_tx))
    assert app.get_account(KEYS[0].addr)["sequence"] == 1
    # replay (sequence now 1) -> bad sign bytes
    rc, r = app.ante(ok_tx)
    assert r["code"] == 4 and r["log"] == UNAUTH
    for bad in (make_tx("other-chain", [KEYS[1]], [1], [0]),        # wrong chain-id
                make_tx("gv-test", [KEYS[2]], [7], [0]),            # wrong account number
                make_tx("gv-test", [KEYS[3]], [3], [5])):           # wrong sequence
        rc, r = app.ante(bad)
        assert r["code"] == 4 and r["log"] == UNAUTH
    # genesis: account number 0 in sign bytes (ante_test.go:200)
    gapp = new_app(ver, height=0)
    rc, r = gapp.ante(make_tx("gv-test", [KEYS[4]], [0], [0]))
    assert r["code"] == 0


@pytest.mark.gpu
def test_multi_signer_and_first_failure_order(ver):
    """TestAnteHandlerMultiSigner + the reference's first-failure reporting."""
    app = new_app(ver)
    parts = make_parts("gv-test", [KEYS[0], KEYS[1], KEYS[2]], [0, 1, 2], [0, 0, 0])
    tx = T.std_tx(*parts)
    rc, r = app.ante(tx)
    assert r["code"] == 0 and r["gpu_leaves"] == 3
    assert (r["code"], r["log"], r["gas_used"]) == new_ref().ante(*parts, len(tx))
    # signer 1 signs with the wrong key; signer 2 has no pubkey anywhere
    app2 = new_app(ver)
    msgs = [T.MsgSend(k.addr, KEYS[9].addr, [(10, "atom")]) for k in KEYS[:3]]
    sb = [T.std_sign_bytes("gv-test", i, 0, FEE, msgs, "") for i in range(3)]
    tx = T.std_tx(msgs, FEE, "", [(KEYS[0].pub, KEYS[0].sign(sb[0])), (KEYS[1].pub, KEYS[5].sign(sb[1])),
                                  (b"", b"\x00" * 64)])
    rc, r = app2.ante(tx)
    assert r["code"] == 8 and "unrecognized public key type" in r["log"]   # gas stage sees the nil pubkey first
    app3 = new_app(ver)
    app3.set_account(KEYS[2].addr, 2, 0, KEYS[2].pub)
    tx = T.std_tx(msgs, FEE, "", [(KEYS[0].pub, KEYS[0].sign(sb[0])), (KEYS[1].pub, KEYS[5].sign(sb[1])),
                                  (KEYS[2].pub, KEYS[2].sign(sb[2]))])
    rc, r = app3.ante(tx)
    assert r["code"] == 4 and r["log"] == UNAUTH and r["gpu_leaves"] == 3
    assert app3.get_account(KEYS[0].addr)["sequence"] == 0        # failed tx: no increment


@pytest.mark.gpu
def test_multisig_k_of_n(ver):
    """tendermint multisig threshold verification, fanned out into GPU leaves
    (secp256k1 and ed25519 sub-keys)."""
    app = new_app(ver)
    subs = [KEYS[0], KEYS[1], KEYS[2], KEYS[3], KEYS[4]]
    ed_seed, ed_pub = T.ed25519_keypair(b"\x11" * 32)
    pubs = [k.pub for k in subs] + [T.amino_ed25519(ed_pub)]
    mk = T.amino_multisig(3, pubs)
    maddr = T.address(mk)
    app.set_account(maddr, 40, 0)
    ref = new_ref()
    ref.set_account(maddr, 40, 0)
    msgs = [T.MsgSend(maddr, KEYS[9].addr, [(5, "atom")])]
    sb = T.std_sign_bytes("gv-test", 40, 0, FEE, msgs, "")
    bits = [True, False, True, False, True, True]
    sigs = [subs[0].sign(sb), subs[2].sign(sb), subs[4].sign(sb), T.ed25519_sign(ed_seed, sb)]
    tx_sigs = [(mk, T.multisignature(bits, sigs))]
    tx = T.std_tx(msgs, FEE, "", tx_sigs)
    rc, r = app.ante(tx)
    # 3 secp256k1 leaves + 1 ed25519 leaf, all on the GPU (gv_verify_ed25519_msgs for the ed25519 one);
    # gas: 3 x 1000 + 590 of signature gas besides the KV reads / writes
    assert rc == 0 and r["code"] == 0 and r["gpu_leaves"] == 4
    assert (r["code"], r["log"], r["gas_used"]) == ref.ante(msgs, FEE, "", tx_sigs, len(tx))
    # one bad secp256k1 leaf -> whole multisig false
    sb1 = T.std_sign_bytes("gv-test", 40, 1, FEE, msgs, "")
    bad = [subs[0].sign(sb1), subs[1].sign(sb1), subs[4].sign(sb1), T.ed25519_sign(ed_seed, sb1)]
    tx = T.std_tx(msgs, FEE, "", [(b"", T.multisignature(bits, bad))])
    rc, r = app.ante(tx)
    assert r["code"] == 4 and r["log"] == UNAUTH
    # bad ed25519 leaf
    ok = [subs[0].sign(sb1), subs[2].sign(sb1), subs[4].sign(sb1), T.ed25519_sign(ed_seed, sb1 + b"x")]
    tx = T.std_tx(msgs, FEE, "", [(b"", T.multisignature(bits, ok))])
    rc, r = app.ante(tx)
    assert r["code"] == 4
    ok[3] = T.ed25519_sign(ed_seed, sb1)
    tx = T.std_tx(msgs, FEE, "", [(b"", T.multisignature(bits, ok))])
    rc, r = app.ante(tx)
    assert r["code"] == 0


@pytest.mark.gpu
def test_preverify_block_fills_cache(ver):
    """PreVerifyTxs: one GPU batch for the block, sequences predicted per signer;
    the per-tx decorator then answers every leaf from the cache."""
    app = new_app(ver)
    block = []
    seqs = {k.addr: 0 for k in KEYS[:6]}
    for t in range(18):
        k = KEYS[t % 6]
        block.append(make_tx("gv-test", [k], [KEYS.index(k)], [seqs[k.addr]]))
        seqs[k.addr] += 1
    rc, n = app.preverify(block)
    assert rc == 0 and n == 18 and app.cache_size() == 18
    for tx in block:
        rc, r = app.ante(tx)
        assert rc == 0 and r["code"] == 0 and r["gpu_leaves"] == 0 and r["cache_hits"] == 1
    # a wrong prediction is only a cache miss, never a different verdict:
    # the tx is signed for sequence 3; preverify predicts 0 (state) and caches
    # "false" for the seq-0 sign bytes; the state then moves to 3 before ante.
    app2 = new_app(ver)
    tx = make_tx("gv-test", [KEYS[7]], [7], [3])
    app2.preverify([tx])
    app2.set_account(KEYS[7].addr, 7, 3)
    rc, r = app2.ante(tx)
    assert r["code"] == 0 and r["cache_hits"] == 0 and r["gpu_leaves"] == 1


@pytest.mark.gpu
def test_parallel_preverify_matches_serial_and_plain_ante(ver):
    """PreVerifyTxs' parallel decode / sign-bytes / SHA stages (threads=8) fill
    the same cache as one thread, and the ante verdicts with the cache equal
    the verdicts without it -- over a block with repeat signers (predicted
    sequences), a wrong-sequence tx, a bad signature and a malformed tx."""
    def block():
        txs, seqs = [], {k.addr: 0 for k in KEYS[:8]}
        for t in range(400):
            k = KEYS[t % 8]
            s = seqs[k.addr] + (5 if t == 101 else 0)          # t=101: signed for a wrong sequence
            tx = make_tx("gv-test", [k], [KEYS.index(k)], [s])
            if t == 202:                                       # bad signature
                tx = make_tx("gv-test", [k], [KEYS.index(k)], [s], sign_keys=[KEYS[9]])
            txs.append(tx)
            if t not in (101, 202):                            # a rejected tx leaves the sequence
                seqs[k.addr] += 1
        txs.insert(150, b"\x01\x02")                           # undecodable bytes
        return txs

    txs = block()
    results = []
    for threads, pre in ((1, True), (8, True), (8, False)):
        app = new_app(ver)
        app.set_threads(threads)
        if pre:
            rc, n = app.preverify(txs)
            assert rc == 0 and n == 400
        out = []
        for tx in txs:
            rc, r = app.ante(tx)
            out.append((rc, r["code"], r["log"]) if rc == 0 else (rc,))
        results.append((out, app.cache_size()))
        app.close()
    assert results[0] == results[1]
    assert results[0][0] == results[2][0]
    codes = [o[1] for o in results[0][0] if len(o) > 1]
    assert codes.count(0) == 398 and codes.count(4) == 2 and codes.count(2) == 1   # 2: ErrTxDecode
