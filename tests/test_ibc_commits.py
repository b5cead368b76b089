"""IBC 07-tendermint commit checks through the batched hook
(gvh_verify_commits): tendermint v0.33.4 VerifyCommit /
VerifyCommitTrusting semantics -- first wrong signature, +2/3 (or trust
level) tallies over commit-flagged votes only, nil and absent votes, unknown
validators, double votes, the trusting loop's early return (a bad signature
after the tally passed is never read), signatures of the wrong length, size
and basic-check failures -- with every signature of every commit in one GPU
batch, compared field for field (code, index, tallies) with the sequential
restatement tests/commit_ref.py over the ed25519 oracle."""
import ctypes
import hashlib

import numpy as np
import pytest

import bench
import commit_ref as R

ABSENT, COMMIT, NIL = R.ABSENT, R.COMMIT, R.NIL


def _signer():
    wl = bench.workload_lib()
    vp = ctypes.c_void_p
    wl.gvw_ed25519_sign.argtypes = [ctypes.c_size_t, ctypes.c_size_t, vp, vp, vp, vp, vp, vp, ctypes.c_int]
    return wl


def sign_many(wl, seeds, msgs):
    """OpenSSL Ed25519 signatures: item i = seeds[i] over msgs[i]; returns (pubs, sigs)."""
    n = len(msgs)
    sd = np.frombuffer(b"".join(seeds), np.uint8).copy()
    ln = np.array([len(m) for m in msgs], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(msgs), np.uint8).copy()
    pub = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    assert wl.gvw_ed25519_sign(n, n, sd.ctypes.data, blob.ctypes.data, off.ctypes.data, ln.ctypes.data,
                               pub.ctypes.data, sig.ctypes.data, 4) == 0
    return [bytes(p) for p in pub], [bytes(s) for s in sig]


class Chain:
    """A validator set (seeds, keys, addresses, powers) and commits signed by it."""

    def __init__(self, wl, rng, n_vals, chain_id="ibc-chain"):
        self.wl, self.rng, self.chain_id = wl, rng, chain_id
        self.seeds = [hashlib.sha256(b"val%d-%d" % (n_vals, int(rng.integers(1 << 62)))).digest()
                      for _ in range(n_vals)]
        pubs, _ = sign_many(wl, self.seeds, [b"x"] * n_vals)
        self.pubs = pubs
        self.vals = [(p, R.address(p), int(rng.integers(1, 1000))) for p in pubs]

    def commit(self, height, flags, signers=None):
        """Signature i by validator signers[i] (default i) with flag flags[i]."""
        signers = list(range(len(flags))) if signers is None else signers
        msgs = [R.vote_sign_bytes(self.chain_id, height, 0, b"\x11" * 32, 1, b"\x22" * 32, 1_600_000_000 + i,
                                  i * 7, f == COMMIT) for i, f in enumerate(flags)]
        _, sigs = sign_many(self.wl, [self.seeds[v] for v in signers], msgs)
        out = []
        for i, f in enumerate(flags):
            s = sigs[i] if f != ABSENT else b""
            out.append((f, self.vals[signers[i]][1], s, msgs[i]))
        return out


def flip(sigs, idx, how="bit"):
    f, a, s, m = sigs[idx]
    if how == "bit":
        s = s[:7] + bytes([s[7] ^ 1]) + s[8:]
    elif how == "short":
        s = s[:63]
    elif how == "msg":
        m = m + b"!"
    sigs[idx] = (f, a, s, m)
    return sigs


def ref(d):
    if d.get("trusting"):
        num, den = d.get("trust", (1, 3))
        return R.verify_commit_trusting(d["vals"], d["sigs"], num, den, d.get("basic_ok", True))
    return R.verify_commit(d["vals"], d["sigs"], d.get("basic_ok", True))


def test_restatement_cases_cpu():
    """The restatement alone (no GPU): the loop rules on a small set."""
    wl = _signer()
    ch = Chain(wl, np.random.default_rng(1), 4)
    s = ch.commit(5, [COMMIT] * 4)
    assert R.verify_commit(ch.vals, s)[0] == "ok"
    assert R.verify_commit(ch.vals, flip(list(s), 2))[:2] == ("wrong_sig", 2)
    assert R.verify_commit(ch.vals, s[:3])[0] == "size"
    assert R.verify_commit_trusting(ch.vals, s, 1, 4)[0] == "bad_trust"
    dv = list(s)
    dv[3] = (COMMIT, ch.vals[0][1], s[0][2], s[0][3])
    got = R.verify_commit_trusting(ch.vals, dv, 1, 1)
    assert got[:3] == ("double_vote", 0, 3)


@pytest.fixture(scope="module")
def app():
    import gpuverify as gvm
    import gvhost
    v = gvm.Verifier([0])
    a = gvhost.HostApp(v, chain_id="ibc-chain", height=1)
    yield a
    a.close()
    v.close()


def cases(wl, rng):
    out = []
    ch = Chain(wl, rng, 10)
    good = ch.commit(10, [COMMIT] * 10)
    out.append({"vals": ch.vals, "sigs": good})                                         # all good
    out.append({"vals": ch.vals, "sigs": flip(list(good), 3)})                          # wrong sig early
    out.append({"vals": ch.vals, "sigs": flip(list(good), 9)})                          # ... at the end (checked)
    out.append({"vals": ch.vals, "sigs": flip(list(good), 4, "short")})                 # 63-byte signature
    out.append({"vals": ch.vals, "sigs": flip(list(good), 5, "msg")})                   # wrong sign bytes
    mixed = ch.commit(11, [COMMIT, NIL, ABSENT, COMMIT, NIL, NIL, ABSENT, COMMIT, NIL, NIL])
    out.append({"vals": ch.vals, "sigs": mixed})                                        # not enough power
    out.append({"vals": ch.vals, "sigs": good[:9]})                                     # size mismatch
    out.append({"vals": ch.vals, "sigs": good, "basic_ok": False})                      # basic check failed
    # trusting: the trusted set overlaps the signers; early return
    big = Chain(wl, rng, 40)
    sigs = big.commit(20, [COMMIT] * 40)
    trusted = big.vals[:25] + ch.vals[:5]                                              # 15 signers unknown
    t = {"vals": trusted, "sigs": sigs, "trusting": True, "trust": (1, 3)}
    out.append(t)
    late = flip(list(sigs), 38)                                                        # after the tally passed
    out.append(dict(t, sigs=late))
    early = flip(list(sigs), 1)                                                        # before it passed
    out.append(dict(t, sigs=early))
    out.append(dict(t, trust=(1, 1)))                                                  # 1/1: never passes
    out.append(dict(t, trust=(1, 4)))                                                  # panics in the reference
    out.append(dict(t, basic_ok=False))
    dv = list(sigs)
    dv[6] = (COMMIT, sigs[2][1], sigs[2][2], sigs[2][3])                               # validator 2 twice
    out.append(dict(t, sigs=dv, trust=(2, 3)))
    nil_only = big.commit(21, [NIL] * 40)
    out.append(dict(t, sigs=nil_only))                                                 # verified, never tallied
    # random commits
    for k in range(12):
        n = int(rng.integers(1, 60))
        c = Chain(wl, rng, n)
        flags = [int(x) for x in rng.choice([ABSENT, COMMIT, COMMIT, COMMIT, NIL], size=n)]
        s = c.commit(30 + k, flags)
        for j in rng.choice(n, size=int(rng.integers(0, 3)), replace=True):
            if s[j][0] != ABSENT:
                s = flip(s, int(j), str(rng.choice(["bit", "short", "msg"])))
        if k % 2:
            out.append({"vals": c.vals, "sigs": s})
        else:
            perm = [int(i) for i in rng.permutation(n)]
            out.append({"vals": [c.vals[i] for i in perm], "sigs": s, "trusting": True,
                        "trust": [(1, 3), (2, 3), (1, 2)][k % 3]})
    return out


@pytest.mark.gpu
def test_commits_batched_match_the_sequential_loops(app):
    wl = _signer()
    cs = cases(wl, np.random.default_rng(7))
    got = app.verify_commits(cs)
    exp = [ref(d) for d in cs]
    assert got == exp
    kinds = {g[0] for g in got}
    assert {"ok", "wrong_sig", "not_enough", "size", "basic", "double_vote", "bad_trust"} <= kinds
    # the trusting loop's early return: a bad signature after the tally passed is never read
    assert got[9][0] == "ok" and got[10][0] == "wrong_sig"
    st = app.stats()
    assert st["gpu_calls"] >= 1


@pytest.mark.gpu
def test_one_gpu_batch_for_many_commits(app):
    """A relayer-sized call: 64 headers of a 100-validator chain (VerifyAdjacent
    shape), one bad signature in some -- one GPU batch for all 6,400 votes."""
    wl = _signer()
    rng = np.random.default_rng(9)
    ch = Chain(wl, rng, 100)
    cs = []
    for h in range(64):
        s = ch.commit(100 + h, [COMMIT] * 100)
        if h % 5 == 0:
            s = flip(s, int(rng.integers(100)))
        cs.append({"vals": ch.vals, "sigs": s, "keys_trusted": True})   # adjacent: the trusted next set
    c0 = app.stats()["gpu_calls"]
    got = app.verify_commits(cs)
    assert app.stats()["gpu_calls"] - c0 == 1
    for h, g in enumerate(got):
        if h % 5 == 0:
            assert g[0] == "wrong_sig"
        else:
            assert g[0] == "ok" and g[3] == sum(v[2] for v in ch.vals)
    # spot-check against the restatement (pure-Python ed25519 is slow)
    for h in (0, 1, 5, 63):
        assert got[h] == ref(cs[h])


@pytest.mark.gpu
def test_untrusted_sets_do_not_load_keys(app):
    """a relayer-supplied validator set (VerifyNonAdjacent's new set)
    is verified without loading its keys into the ed25519 key arena, so fresh
    keys in every update cannot churn the arena; the trusted set's keys are
    loaded (they sign block after block).  Same verdicts either way."""
    wl = _signer()
    rng = np.random.default_rng(11)
    v = app._v
    v.ed_keys_reset()
    fresh = Chain(wl, rng, 30)
    s = fresh.commit(500, [COMMIT] * 30)
    s = flip(s, 7)
    untrusted = {"vals": fresh.vals, "sigs": s}                  # keys_trusted defaults to trusting (False)
    got = app.verify_commits([untrusted])
    assert got == [ref(untrusted)] and got[0][0] == "wrong_sig"
    assert v.ed_keys_count == 0
    trusted = {"vals": fresh.vals, "sigs": fresh.commit(501, [COMMIT] * 30), "keys_trusted": True}
    got = app.verify_commits([trusted])
    assert got == [ref(trusted)] and got[0][0] == "ok"
    assert v.ed_keys_count == 30
    v.ed_keys_reset()
