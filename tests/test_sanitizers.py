"""Sanitizer builds of the host mirror (reference Makefile:123-124
`test-race`): host/gvhost.cpp built with ASan + UBSan and with TSan, driven
from several threads by tests/sanitize/harness.cpp over a CPU fake of the
verifier (tests/sanitize/fake_gpuverify.cpp: the oracle for secp256k1,
OpenSSL for ed25519 -- test infrastructure, not the product library).

The harness replays blocks through gvh_deliver_blocks (block b+1's
pre-verification batch on the helper thread while block b's DeliverTx loop
runs on the 8-thread pool, sharing pinned pack buffers and the key-slot map)
and compares codes and final accounts with block-by-block delivery and with
the per-tx ante; then 8 threads call gvh_checktx at once (the accumulation
window) and the codes must equal serial ante runs.  A sanitizer report makes
the binary exit nonzero.  The codes are also checked against the Python
restatement of the chain (tests/ante_ref.py).
"""
import os
import random
import struct
import subprocess
import json

import pytest

import txkit as T
from ante_ref import AnteRef

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "sanitize")
CHAIN = "gv-san"
HEIGHT = 5
FEE = T.Fee([(0, "stake")], 1000000)


def _build():
    r = subprocess.run(["make", "-s", "-j2", "-C", SAN], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


class Key:
    def __init__(self, tag: bytes):
        self.priv = T.privkey_from_secret(b"san-" + tag)
        self.amino = T.amino_secp(T.secp_pubkey(self.priv))
        self.addr = T.address(self.amino)

    def sign(self, msg):
        return T.secp_sign(self.priv, msg)


def _workload():
    rng = random.Random(0x5A4)
    singles = [Key(b"s%d" % i) for i in range(48)]
    subs = [[Key(b"m%d-%d" % (i, j)) for j in range(3)] for i in range(6)]
    multis = [(T.amino_multisig(2, [k.amino for k in ss]), ss) for ss in subs]
    sink = Key(b"sink").addr
    accts = []                                   # (addr, number, seq, stored pub)
    for i, k in enumerate(singles):
        accts.append((k.addr, 10 + i, 0, k.amino if i % 4 == 0 else b""))
    for i, (am, _) in enumerate(multis):
        accts.append((T.address(am), 200 + i, 0, am))
    seq = {a[0]: 0 for a in accts}
    stored = {a[0]: bool(a[3]) for a in accts}
    blocks, parts = [], []
    for b in range(3):
        txs = []
        for t in range(1100 if b % 2 else 250):           # block 1 takes the parallel ante loop (>= 1024 txs)
            if t % 10 == 9:
                mi = rng.randrange(len(multis))
                am, ss = multis[mi]
                addr = T.address(am)
                msgs = [T.MsgSend(addr, sink, [(1, "m")])]
                sb = T.std_sign_bytes(CHAIN, 200 + mi, seq[addr], FEE, msgs, "")
                chosen = sorted(rng.sample(range(3), 2))
                sigs = [ss[j].sign(sb) for j in chosen]
                if rng.random() < 0.1:
                    sigs[0] = sigs[0][:5] + bytes([sigs[0][5] ^ 1]) + sigs[0][6:]
                else:
                    seq[addr] += 1
                sg = [(b"", T.multisignature([j in chosen for j in range(3)], sigs))]
                txs.append(T.std_tx(msgs, FEE, "", sg))
                parts.append((msgs, sg))
                continue
            i = rng.randrange(len(singles))
            k = singles[i]
            msgs = [T.MsgSend(k.addr, sink, [(1 + t % 5, "s")])]
            wrong = rng.random() < 0.03
            sb = T.std_sign_bytes(CHAIN, 10 + i, seq[k.addr] + (2 if wrong else 0), FEE, msgs, "")
            bad = rng.random() < 0.03
            sig = singles[(i + 1) % len(singles)].sign(sb) if bad else k.sign(sb)
            supply = not stored[k.addr] and rng.random() < 0.7
            sg = [(k.amino if supply else b"", sig)]
            txs.append(T.std_tx(msgs, FEE, "", sg))
            parts.append((msgs, sg))
            if not (wrong or bad) and (stored[k.addr] or supply):
                seq[k.addr] += 1
                stored[k.addr] = True
        blocks.append(txs)
    # CheckTx: 8 threads, each with its own 4 signers (order-independent across threads)
    check = []
    ckeys = [[Key(b"c%d-%d" % (th, j)) for j in range(4)] for th in range(8)]
    for th, ks in enumerate(ckeys):
        cseq = [0] * 4
        txs = []
        for t in range(40):
            j = t % 4
            k = ks[j]
            num = 500 + 4 * th + j
            msgs = [T.MsgSend(k.addr, sink, [(1, "c")])]
            sb = T.std_sign_bytes(CHAIN, num, cseq[j], FEE, msgs, "")
            bad = t % 13 == 7
            txs.append(T.std_tx(msgs, FEE, "", [(k.amino, ks[(j + 1) % 4].sign(sb) if bad else k.sign(sb))]))
            cseq[j] += 0 if bad else 1
        check.append(txs)
        for j, k in enumerate(ks):
            accts.append((k.addr, 500 + 4 * th + j, 0, b""))
    return accts, blocks, check, parts


def _fixture(path, accts, blocks, check):
    out = bytearray(b"GVSAN1")
    out += struct.pack("<I", len(CHAIN)) + CHAIN.encode() + struct.pack("<q", HEIGHT)
    out += struct.pack("<I", len(accts))
    for addr, num, seq, pub in accts:
        out += addr + struct.pack("<QQI", num, seq, len(pub)) + pub
    for group in (blocks, check):
        out += struct.pack("<I", len(group))
        for txs in group:
            out += struct.pack("<I", len(txs))
            for tx in txs:
                out += struct.pack("<I", len(tx)) + tx
    with open(path, "wb") as f:
        f.write(out)


@pytest.fixture(scope="module")
def fixture(tmp_path_factory):
    _build()
    accts, blocks, check, parts = _workload()
    path = str(tmp_path_factory.mktemp("san") / "fixture.bin")
    _fixture(path, accts, blocks, check)
    return path, accts, blocks, parts


def _run(binary, path, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([os.path.join(SAN, "build", binary), path], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-6000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    return json.loads(r.stdout)


def _reference_codes(accts, blocks, parts):
    ref = AnteRef(CHAIN, height=HEIGHT)
    for addr, num, seq, pub in accts:
        ref.set_account(addr, num, seq, pub)
    txs = [tx for b in blocks for tx in b]
    return [ref.ante(msgs, FEE, "", sigs, len(tx))[0] for tx, (msgs, sigs) in zip(txs, parts)]


def test_asan_ubsan_host_mirror(fixture):
    path, accts, blocks, parts = fixture
    got = _run("harness_asan", path, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1"})
    assert len(got["blocks"]) == sum(len(b) for b in blocks)
    assert 0 < got["blocks"].count(0) < len(got["blocks"])
    assert 4 in got["check"] and 0 in got["check"]
    assert got["blocks"] == _reference_codes(accts, blocks, parts)


def test_tsan_host_mirror(fixture):
    path, _, blocks, _ = fixture
    # detect_deadlocks=0: the verdict cache's resize() holds every lock stripe
    # at once, past the deadlock detector's 64-held-locks table (its own CHECK
    # fails); data-race detection is unaffected
    got = _run("harness_tsan", path, {"TSAN_OPTIONS": "halt_on_error=1:detect_deadlocks=0"})
    assert len(got["blocks"]) == sum(len(b) for b in blocks)
    assert got["windows"] >= 1
