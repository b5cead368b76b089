"""ed25519 against cached keys on the GPU (csrc/ed_lat.hip
through gv_ed_keys_load / gv_verify_ed25519_msgs_keyed): the verdict of
gv_verify_ed25519_msgs -- go1.14 crypto/ed25519 Verify -- for every golden
vector (oracle/ed25519_ref.py verdicts: non-canonical and small-order keys,
keys off the curve, S >= L, sig[63] & 224, non-canonical R, R' = identity),
the RFC 8032 vectors and OpenSSL on random batches, on both schedules (the
sliced small-batch kernel k_ed_lat_sl and, past "ed_lat_max", the throughput
kernels), at message lengths around the kernel's 2,048-byte LDS staging."""
import json
import os
import random
import time

import numpy as np
import pytest

import ed_openssl as OSSL
import gpuverify as gvm

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


def golden():
    g = json.load(open(os.path.join(GOLD, "ed25519_vectors.json")))
    return [(cat, bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), v["ok"])
            for cat, vs in g["categories"].items() for v in vs]


def load_keys(ver, pubs):
    """distinct keys loaded once; returns the slot of every item"""
    uniq = list(dict.fromkeys(pubs))
    slots = ver.ed_keys_load(np.array([np.frombuffer(p, np.uint8) for p in uniq]).reshape(-1, 32))
    where = {p: int(s) for p, s in zip(uniq, slots)}
    return np.array([where[p] for p in pubs], np.uint32)


def sigs(items):
    return np.array([np.frombuffer(s, np.uint8) for s in items]).reshape(-1, 64)


@pytest.mark.parametrize("lat_max", [2048, 0])
def test_golden_vectors_keyed(ver, lat_max):
    gv = golden()
    ver.set_option("ed_lat_max", lat_max)
    try:
        slots = load_keys(ver, [p for _, p, _, _, _ in gv])
        got = ver.verify_batch_ed25519_keyed(slots, sigs([s for *_, s, _ in gv]), [m for _, _, m, _, _ in gv])
    finally:
        ver.set_option("ed_lat_max", 2048)
    bad = [(c, ok) for (c, _, _, _, ok), g in zip(gv, got) if bool(g) != ok]
    assert not bad, bad[:10]
    # the same items through the unkeyed entry point
    pub = np.array([np.frombuffer(p, np.uint8) for _, p, _, _, _ in gv]).reshape(-1, 32)
    ref = ver.verify_batch_ed25519(pub, sigs([s for *_, s, _ in gv]), [m for _, _, m, _, _ in gv])
    assert np.array_equal(got, ref)


def test_rfc8032_keyed(ver):
    vs = json.load(open(os.path.join(GOLD, "ed25519_rfc8032.json")))["vectors"]
    pubs = [bytes.fromhex(v["pub"]) for v in vs]
    msgs = [bytes.fromhex(v["msg"]) for v in vs]
    sg = sigs([bytes.fromhex(v["sig"]) for v in vs])
    slots = load_keys(ver, pubs)
    assert ver.verify_batch_ed25519_keyed(slots, sg, msgs).all()
    assert not ver.verify_batch_ed25519_keyed(slots, sg, [m + b"." for m in msgs]).any()


def random_items(rng, seeds, pubs, n, maxlen=420):
    items, want = [], []
    for i in range(n):
        k = rng.randrange(len(seeds))
        msg = rng.randbytes(rng.randrange(0, maxlen))
        sig = OSSL.sign(seeds[k], msg)
        r = rng.random()
        if r < 0.1:
            sig = bytearray(sig)
            sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(sig)
        elif r < 0.2:
            msg = msg + b"\x01"
        elif r < 0.25:                                       # S + L: rejected by ScMinimal
            s = int.from_bytes(sig[32:], "little") + 2**252 + 27742317777372353535851937790883648493
            if s < 2**253:
                sig = sig[:32] + s.to_bytes(32, "little")
        items.append((k, msg, sig))
        want.append(OSSL.verify(pubs[k], msg, sig))
    return items, np.array(want)


def test_random_batches_vs_openssl_both_schedules(ver):
    rng = random.Random(0xED)
    seeds = [rng.randbytes(32) for _ in range(100)]           # a validator set
    pubs = [OSSL.public_key(s) for s in seeds]
    slots = ver.ed_keys_load(np.array([np.frombuffer(p, np.uint8) for p in pubs]))
    for n in (1, 7, 64, 150, 2048, 2049, 5000):
        items, want = random_items(rng, seeds, pubs, n)
        got = ver.verify_batch_ed25519_keyed(slots[[k for k, _, _ in items]], sigs([s for *_, s in items]),
                                             [m for _, m, _ in items])
        assert np.array_equal(got.astype(bool), want), (n, np.nonzero(got.astype(bool) != want)[0][:10])


def test_long_messages_across_the_lds_staging(ver):
    rng = random.Random(7)
    seed = rng.randbytes(32)
    pub = OSSL.public_key(seed)
    slot = ver.ed_keys_load(np.frombuffer(pub, np.uint8).reshape(1, 32))[0]
    lens = [0, 1, 63, 64, 127, 128, 2046, 2047, 2048, 2049, 2050, 2111, 2112, 4095, 4096, 9000]
    msgs = [rng.randbytes(n) for n in lens]
    sg = [OSSL.sign(seed, m) for m in msgs]
    bad = [m[:-1] + bytes([m[-1] ^ 0x80]) if m else b"x" for m in msgs]   # last byte flipped (past the LDS part too)
    got = ver.verify_batch_ed25519_keyed(np.full(2 * len(lens), slot, np.uint32), sigs(sg + sg), msgs + bad)
    assert got[:len(lens)].all() and not got[len(lens):].any()


def test_slots_without_a_key_and_reset(ver):
    rng = random.Random(3)
    seed = rng.randbytes(32)
    pub = OSSL.public_key(seed)
    slot = int(ver.ed_keys_load(np.frombuffer(pub, np.uint8).reshape(1, 32))[0])
    msg = b"commit"
    sg = sigs([OSSL.sign(seed, msg)] * 2)
    count = ver.ed_keys_count
    got = ver.verify_batch_ed25519_keyed(np.array([slot, count + 5], np.uint32), sg, [msg, msg])
    assert list(got) == [1, 0]
    gen = ver.ed_keys_generation
    ver.ed_keys_reset()
    assert ver.ed_keys_count == 0 and ver.ed_keys_generation == gen + 1
    assert not ver.verify_batch_ed25519_keyed(np.array([slot], np.uint32), sg[:1], [msg]).any()
    assert int(ver.ed_keys_load(np.frombuffer(pub, np.uint8).reshape(1, 32))[0]) == 0


def test_small_batch_latency(ver):
    """64 signatures of a 100-key validator set against cached keys: the
    sliced kernel answers in well under the throughput kernels' time."""
    rng = random.Random(64)
    seeds = [rng.randbytes(32) for _ in range(100)]
    pubs = [OSSL.public_key(s) for s in seeds]
    slots = ver.ed_keys_load(np.array([np.frombuffer(p, np.uint8) for p in pubs]))
    msgs = [rng.randbytes(120) for _ in range(64)]
    sg = sigs([OSSL.sign(seeds[i], m) for i, m in enumerate(msgs)])
    sl = slots[:64]
    pub = np.array([np.frombuffer(pubs[i], np.uint8) for i in range(64)])
    for _ in range(5):
        assert ver.verify_batch_ed25519_keyed(sl, sg, msgs).all()
        assert ver.verify_batch_ed25519(pub, sg, msgs).all()
    tk, tu = [], []
    for _ in range(50):
        t = time.perf_counter()
        ver.verify_batch_ed25519_keyed(sl, sg, msgs)
        tk.append(time.perf_counter() - t)
        t = time.perf_counter()
        ver.verify_batch_ed25519(pub, sg, msgs)
        tu.append(time.perf_counter() - t)
    pk, pu = float(np.median(tk)) * 1e3, float(np.median(tu)) * 1e3
    print(f"ed25519 @64: keyed sliced p50 {pk:.3f} ms, throughput kernels p50 {pu:.3f} ms")
    assert pk < pu


def test_large_keyed_batches_schedules_agree(ver):
    """Past ed_lat_max the cached-key throughput kernel (k_ed_keyed, lanes in
    slot order, [s]B from either comb table) must give the throughput kernels'
    verdicts: goldens tiled and
    shuffled (every rejection class, keys that FromBytes rejects included),
    never-loaded slots interleaved, both lane orders."""
    gv = golden()
    reps = max(1, 6000 // len(gv))
    order = np.random.default_rng(21).permutation(reps * len(gv))
    items = [gv[i % len(gv)] for i in order]
    slots = load_keys(ver, [p for _, p, _, _, _ in items])
    slots[::7] = ver.ed_keys_count + np.arange(len(slots[::7]), dtype=np.uint32)   # no key: false
    exp = np.array([ok for *_, ok in items])
    exp[::7] = False
    sg, msgs = sigs([s for *_, s, _ in items]), [m for _, _, m, _, _ in items]
    runs = {}
    try:
        # (ed_keyed, sort_keys, ed_btab16): [s]B from the radix-2^16 table
        # (16 additions, the default) and from the radix-256 one (32)
        for keyed, srt, b16 in ((1, 1, 1), (1, 0, 1), (1, 1, 0), (0, 1, 1)):
            ver.set_option("ed_keyed", keyed)
            ver.set_option("sort_keys", srt)
            ver.set_option("ed_btab16", b16)
            runs[(keyed, srt, b16)] = ver.verify_batch_ed25519_keyed(slots, sg, msgs)
    finally:
        ver.set_option("ed_keyed", 1)
        ver.set_option("sort_keys", 1)
        ver.set_option("ed_btab16", 1)
    for k, got in runs.items():
        bad = np.nonzero(got.astype(bool) != exp)[0]
        assert bad.size == 0, (k, [(items[i][0], bool(exp[i])) for i in bad[:10]])


def test_split_key_build_same_verdicts(ver):
    """gv_ed_keys_load with the key chain and the table additions in two
    launches (ed_keys_split, default) and in one serial lane per key: the
    golden vectors (keys FromBytes rejects included) and random validator-set
    items verify identically, on the sliced and the per-lane keyed kernels."""
    gv = golden()
    rng = random.Random(0x5B)
    seeds = [rng.randbytes(32) for _ in range(40)]
    pubs = [OSSL.public_key(s) for s in seeds]
    items, want = random_items(rng, seeds, pubs, 3000)
    res = {}
    try:
        for split in (1, 0):
            ver.set_option("ed_keys_split", split)
            ver.ed_keys_reset()
            slots = load_keys(ver, [p for _, p, _, _, _ in gv] + pubs)
            gs, rs = slots[:len(gv)], slots[len(gv):]
            g = ver.verify_batch_ed25519_keyed(gs, sigs([s for *_, s, _ in gv]), [m for _, _, m, _, _ in gv])
            r = ver.verify_batch_ed25519_keyed(rs[[k for k, _, _ in items]], sigs([s for *_, s in items]),
                                               [m for _, m, _ in items])
            res[split] = (g.astype(bool), r.astype(bool))
    finally:
        ver.set_option("ed_keys_split", 1)
    exp = np.array([ok for *_, ok in gv])
    for split, (g, r) in res.items():
        assert np.array_equal(g, exp), (split, np.nonzero(g != exp)[0][:10])
        assert np.array_equal(r, want), (split, np.nonzero(r != want)[0][:10])
