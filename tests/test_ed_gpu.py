"""ed25519 VerifyBytes on the GPU (csrc/ed_verify.hip through the C ABI
gv_verify_ed25519_msgs / gv_dev_verify_ed25519_msgs) against the committed
golden vectors (verdicts of oracle/ed25519_ref.py, go1.14 crypto/ed25519
semantics: non-canonical and small-order keys, S >= L, sig[63] & 224,
non-canonical R), the RFC 8032 vectors, and OpenSSL on random batches --
on both host-batch schedules: the throughput kernels and the small-batch
kernel k_ed_lat_unc (csrc/ed_lat.hip, one signature per block, FromBytes(A)
in the kernel; "ed_unc_lat_max" picks one per call)."""
import json
import os
import random

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


SCHEDULES = {"throughput": 0, "small": 1 << 30}      # ed_unc_lat_max


@pytest.fixture(params=sorted(SCHEDULES))
def sched(request, ver):
    ver.set_option("ed_unc_lat_max", SCHEDULES[request.param])
    yield request.param
    ver.set_option("ed_unc_lat_max", 2048)


def arrays(items):
    pub = np.array([np.frombuffer(p, np.uint8) for p, _, _ in items]).reshape(-1, 32)
    sig = np.array([np.frombuffer(s, np.uint8) for _, _, s in items]).reshape(-1, 64)
    return pub, sig, [m for _, m, _ in items]


def golden():
    g = json.load(open(os.path.join(GOLD, "ed25519_vectors.json")))
    out = []
    for cat, vs in g["categories"].items():
        for v in vs:
            out.append((cat, bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]), v["ok"]))
    return out


def test_golden_vectors(ver, sched):
    gv = golden()
    pub, sig, msgs = arrays([(p, m, s) for _, p, m, s, _ in gv])
    got = ver.verify_batch_ed25519(pub, sig, msgs)
    bad = [(c, ok) for (c, _, _, _, ok), g in zip(gv, got) if bool(g) != ok]
    assert not bad, bad[:10]
    assert int(got.sum()) == sum(ok for *_, ok in gv)


def test_rfc8032(ver, sched):
    vs = json.load(open(os.path.join(GOLD, "ed25519_rfc8032.json")))["vectors"]
    items = [(bytes.fromhex(v["pub"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]
    pub, sig, msgs = arrays(items)
    assert ver.verify_batch_ed25519(pub, sig, msgs).all()
    assert not ver.verify_batch_ed25519(pub, sig, [m + b"." for m in msgs]).any()


def test_random_batch_vs_openssl(ver, sched):
    rng = random.Random(11)
    seeds = [rng.randbytes(32) for _ in range(64)]
    pubs = [OSSL.public_key(s) for s in seeds]
    items, want = [], []
    for i in range(6000):
        k = i % 64
        msg = rng.randbytes(rng.randrange(0, 420))
        sig = OSSL.sign(seeds[k], msg)
        r = rng.random()
        if r < 0.1:
            sig = bytearray(sig)
            sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(sig)
        elif r < 0.2:
            msg = msg + b"\x01"
        elif r < 0.25:                                       # S + L: malleated, rejected by ScMinimal
            s = int.from_bytes(sig[32:], "little") + 2**252 + 27742317777372353535851937790883648493
            if s < 2**253:
                sig = sig[:32] + s.to_bytes(32, "little")
        items.append((pubs[k], msg, sig))
        want.append(OSSL.verify(pubs[k], msg, sig))
    pub, sig, msgs = arrays(items)
    r0 = ver.route_stats()["ed_lat"]
    got = ver.verify_batch_ed25519(pub, sig, msgs)
    assert np.array_equal(got.astype(bool), np.array(want)), np.nonzero(got.astype(bool) != np.array(want))[0][:10]
    assert 0.6 < got.mean() < 0.9
    assert (ver.route_stats()["ed_lat"] > r0) == (sched == "small")


@pytest.mark.parametrize("n", [1, 63, 64, 65, 257])
def test_ragged_sizes_and_empty_messages(ver, sched, n):
    rng = random.Random(n)
    seed = rng.randbytes(32)
    pub = OSSL.public_key(seed)
    items = [(pub, b"", OSSL.sign(seed, b"")) for _ in range(n)]
    p, s, _ = arrays(items)
    z = np.zeros(n, np.uint64)
    got = ver.verify_batch_ed25519(p, s, (np.zeros(1, np.uint8), z, z.astype(np.uint32)))
    assert got.all()
    assert ver.verify_batch_ed25519(p[:0], s[:0], []).shape == (0,)


def test_chunked_batch_and_device_resident(ver):
    """> 262,144 items: several chunks of the host path; the same batch
    device-resident (gv_dev_verify_ed25519_msgs) gives the same bitmap."""
    base = 2048
    rng = random.Random(5)
    seeds = [rng.randbytes(32) for _ in range(16)]
    pubs = [OSSL.public_key(s) for s in seeds]
    items, want = [], []
    for i in range(base):
        msg = rng.randbytes(rng.randrange(0, 200))
        sig = OSSL.sign(seeds[i % 16], msg)
        if i % 5 == 0:
            msg += b"!"
        items.append((pubs[i % 16], msg, sig))
        want.append(i % 5 != 0)
    reps = 150                                               # 307,200 items
    pub, sig, msgs = arrays(items)
    blob, off, ln = gvm.pack_msgs(msgs)
    total = base * reps
    P = np.tile(pub, (reps, 1))
    S = np.tile(sig, (reps, 1))
    O = (np.tile(off, reps) + np.repeat(np.arange(reps, dtype=np.uint64) * np.uint64(len(blob)), base)).astype(np.uint64)
    Lh = np.tile(ln, reps)
    Bl = np.tile(blob, reps)
    W = np.tile(np.array(want), reps)
    got = ver.verify_batch_ed25519(P, S, (Bl, O, Lh))
    assert np.array_equal(got.astype(bool), W)
    d = [ver.dev_alloc(a.nbytes) for a in (P, S, Bl, O, Lh)]
    for ptr, a in zip(d, (P, S, Bl, O, Lh)):
        ver.dev_upload(ptr, np.ascontiguousarray(a))
    nw = (total + 63) // 64
    d_bits = ver.dev_alloc(nw * 8)
    ver.dev_verify_ed25519(0, total, d[0], d[1], d[2], d[3], d[4], d_bits)
    ver.dev_sync()
    bits = np.zeros(nw, np.uint64)
    ver.dev_download(bits, d_bits)
    dev = np.unpackbits(bits.view(np.uint8), bitorder="little")[:total].astype(bool)
    assert np.array_equal(dev, W)
    for ptr in d + [d_bits]:
        ver.dev_free(ptr)


def test_two_device_slots_split_ed25519():
    """gv_open with device slots [0, 0]: the ed25519 host path splits a batch
    across the two slots (persistent worker for slot 1) and concatenates."""
    v = gvm.Verifier([0, 0])
    try:
        rng = random.Random(21)
        seeds = [rng.randbytes(32) for _ in range(8)]
        pubs = [OSSL.public_key(s) for s in seeds]
        items, want = [], []
        for i in range(1500):
            msg = rng.randbytes(rng.randrange(0, 120))
            sig = OSSL.sign(seeds[i % 8], msg)
            if i % 3 == 0:
                msg += b"?"
            items.append((pubs[i % 8], msg, sig))
            want.append(i % 3 != 0)
        pub, sig, msgs = arrays(items)
        assert np.array_equal(v.verify_batch_ed25519(pub, sig, msgs).astype(bool), np.array(want))
    finally:
        v.close()


def test_in_batch_key_grouping_matches_throughput_kernels(ver):
    """ed_group: a batch repeating few keys builds each key's comb table once
    (k_ed_keys) and verifies on k_ed_keyed; every golden vector (keys that
    FromBytes rejects, small-order keys, S >= L, non-canonical R ...) tiled
    and shuffled with random OpenSSL items must give the throughput kernels'
    verdicts, host and device-resident, both lane orders, radix-64 and
    radix-16 key combs."""
    gv = golden()
    rng = random.Random(0x6E)
    seeds = [rng.randbytes(32) for _ in range(24)]
    pubs = [OSSL.public_key(s) for s in seeds]
    items, want = [], []
    for i in range(1200):
        msg = rng.randbytes(rng.randrange(0, 300))
        sig = OSSL.sign(seeds[i % 24], msg)
        if i % 7 == 0:
            sig = sig[:5] + bytes([sig[5] ^ 4]) + sig[6:]
        items.append((pubs[i % 24], msg, sig))
        want.append(i % 7 != 0)
    items += [(p, m, s) for _, p, m, s, _ in gv]
    want += [ok for *_, ok in gv]
    reps = 20
    order = np.random.default_rng(9).permutation(reps * len(items))
    items = [items[i % len(items)] for i in order]
    want = np.array([want[i % len(want)] for i in order])
    pub, sig, msgs = arrays(items)
    blob, off, ln = gvm.pack_msgs(msgs)
    n = len(items)
    ver.set_option("ed_group_min", 4096)
    try:
        runs = {}
        # (ed_group, sort_keys, ed_group_r64): radix-64 grouped key tables (the
        # default) and radix-16 ones
        for grp, srt, r64 in ((1, 1, 1), (1, 0, 1), (1, 1, 0), (0, 1, 1)):
            ver.set_option("ed_group", grp)
            ver.set_option("sort_keys", srt)
            ver.set_option("ed_group_r64", r64)
            b0, _ = ver.group_stats()
            host = ver.verify_batch_ed25519(pub, sig, (blob, off, ln))
            d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, blob, off, ln)]
            for ptr, a in zip(d, (pub, sig, blob, off, ln)):
                ver.dev_upload(ptr, np.ascontiguousarray(a))
            d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
            ver.dev_verify_ed25519(0, n, d[0], d[1], d[2], d[3], d[4], d_bits)
            ver.dev_sync()
            bits = np.zeros((n + 63) // 64, np.uint64)
            ver.dev_download(bits, d_bits)
            for ptr in d + [d_bits]:
                ver.dev_free(ptr)
            dev = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n].astype(bool)
            runs[(grp, srt, r64)] = (host.astype(bool), dev, ver.group_stats()[0] - b0)
    finally:
        ver.set_option("ed_group", 1)
        ver.set_option("sort_keys", 1)
        ver.set_option("ed_group_r64", 1)
        ver.set_option("ed_group_min", 196608)
    for k, (host, dev, grouped) in runs.items():
        assert grouped == (2 if k[0] else 0), (k, grouped)
        assert np.array_equal(host, want), (k, np.nonzero(host != want)[0][:10])
        assert np.array_equal(dev, want), (k, np.nonzero(dev != want)[0][:10])
