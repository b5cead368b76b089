"""GPU parity tests: libgpuverify (HIP, gfx950) vs the oracle, through the C-ABI.

Bit-exact bar: every accept/reject verdict must equal the oracle's
(oracle/secp256k1_oracle.c, pinned in tests/test_oracle.py), which restates
tendermint VerifyBytes / btcec / crypto/ecdsa (x/auth/ante/sigverify.go:210).
"""
import random

import numpy as np
import pytest

import gpuverify as gvm
from golden_io import load_digest_vectors, load_msg_vectors
from oracle import oracle as O
from oracle import secp_ref as R

pytestmark = pytest.mark.gpu

P, N = R.P, R.N
BETA = R.BETA


@pytest.fixture(scope="module")
def ver():
    v = gvm.Verifier([0])
    yield v
    v.close()


def to_words(a: int, b: int):
    return [(a >> (32 * i)) & 0xFFFFFFFF for i in range(8)] + [(b >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def from_words(ws, lo=0, n=8):
    return sum(int(ws[lo + i]) << (32 * i) for i in range(n))


EDGE = [0, 1, 2, 977, 2**32, 2**32 + 977, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2**32 - 978,
        2**255, 2**224 - 1, N, N - 1, BETA, (1 << 128) - 1]


def operand_pairs(rng, count):
    vals = EDGE + [rng.randrange(2**256) for _ in range(count)]
    pairs = [(a, b) for a in EDGE for b in EDGE]
    pairs += [(rng.choice(vals), rng.choice(vals)) for _ in range(count)]
    return pairs


def run_op(ver, op, pairs):
    w = np.array([to_words(a, b) for a, b in pairs], dtype=np.uint32)
    return ver.debug_op(op, w)


@pytest.mark.parametrize("op,fn", [
    (0, lambda a, b: a * b % P),
    (1, lambda a, b: a * a % P),
    (2, lambda a, b: (a + b) % P),
    (3, lambda a, b: (a - b) % P),
    (6, lambda a, b: a % P),
    (12, lambda a, b: 2 * a % P),
    (13, lambda a, b: 4 * a % P),
    (14, lambda a, b: 8 * a % P),
    (15, lambda a, b: 3 * a % P),
    (16, lambda a, b: (a - 2 * b) % P),
    (17, lambda a, b: (a - 4 * b) % P),
    (18, lambda a, b: (a - 8 * b) % P),
])
def test_field_ops(ver, op, fn):
    rng = random.Random(op)
    pairs = operand_pairs(rng, 3000)
    out = run_op(ver, op, pairs)
    for (a, b), o in zip(pairs, out):
        assert from_words(o) == fn(a, b), (op, hex(a), hex(b))


@pytest.mark.parametrize("op,fn", [
    (19, lambda a, b: a * b % P),
    (20, lambda a, b: a * a % P),
    (21, lambda a, b: (a - b) % P),
    (25, lambda a, b: int((a - b) % P == 0)),
])
def test_field29_ops(ver, op, fn):
    """The 9 x 29 reduced-radix layer (csrc/secp_fe29.cuh) on the device: words
    in (any value < 2^256), canonical words out, incl. the fast zero test."""
    rng = random.Random(100 + op)
    pairs = operand_pairs(rng, 3000)
    if op == 25:
        pairs += [(b + k * P, b) for b in (0, 1, 5, 2**200, P - 1) for k in (0, 1) if b + k * P < 2**256]
        pairs += [(a, a) for a in EDGE]
    out = run_op(ver, op, pairs)
    for (a, b), o in zip(pairs, out):
        assert from_words(o) == fn(a, b), (op, hex(a), hex(b))


def test_field29_inv_sqrt_double(ver):
    rng = random.Random(23)
    xs = [1, 2, P - 1, 7, BETA] + [rng.randrange(1, P) for _ in range(500)]
    out = run_op(ver, 22, [(x, 0) for x in xs])
    for x, o in zip(xs, out):
        assert from_words(o) == pow(x, P - 2, P)
    out = run_op(ver, 23, [(x, 0) for x in xs])
    for x, o in zip(xs, out):
        assert from_words(o) == pow(x, (P + 1) // 4, P)
    pts = [R.point_mul(k, R.G) for k in (1, 2, 3, 12345, N - 1, R.LAMBDA)]
    pts += [R.point_mul(rng.randrange(1, N), R.G) for _ in range(64)]
    out = run_op(ver, 24, [(p[0], p[1]) for p in pts])
    for p, o in zip(pts, out):
        q = R.point_add(p, p)
        assert from_words(o, 0) == q[0] and from_words(o, 8) == q[1]


def test_mul512(ver):
    rng = random.Random(7)
    pairs = operand_pairs(rng, 3000)
    out = run_op(ver, 7, pairs)
    for (a, b), o in zip(pairs, out):
        assert from_words(o, 0, 16) == a * b, (hex(a), hex(b))


def test_field_inv_and_sqrt(ver):
    rng = random.Random(11)
    xs = [1, 2, P - 1, 7, BETA] + [rng.randrange(1, P) for _ in range(500)]
    out = run_op(ver, 4, [(x, 0) for x in xs])
    for x, o in zip(xs, out):
        assert from_words(o) == pow(x, P - 2, P)
    out = run_op(ver, 5, [(x, 0) for x in xs])
    for x, o in zip(xs, out):
        assert from_words(o) == pow(x, (P + 1) // 4, P)


def test_scalar_montmul(ver):
    rng = random.Random(13)
    Rinv = pow(2**256, -1, N)
    pairs = [(a, b) for a in (0, 1, N - 1, 2) for b in (0, 1, N - 1, 3)]
    pairs += [(rng.randrange(N), rng.randrange(N)) for _ in range(3000)]
    out = run_op(ver, 8, pairs)
    for (a, b), o in zip(pairs, out):
        assert from_words(o) == a * b * Rinv % N


def test_scalar29_montmul(ver):
    """Radix-2^29 Montgomery product mod n (csrc/secp_sc29.cuh), R = 2^261."""
    rng = random.Random(29)
    Rinv = pow(2**261, -1, N)
    pairs = [(a, b) for a in (0, 1, N - 1, 2, 2**256 - 1) for b in (0, 1, N - 1, 3, 2**256 - 1)]
    pairs += [(rng.randrange(2**256), rng.randrange(2**256)) for _ in range(3000)]
    out = run_op(ver, 26, pairs)
    for (a, b), o in zip(pairs, out):
        assert from_words(o) == a * b * Rinv % N


def test_scalar_inverse_divsteps(ver):
    """op 27: s^-1 mod n by divsteps (the latency kernel's inverse) == pow(s, -1, n)."""
    rng = random.Random(27)
    xs = [1, 2, N - 1, N - 2, (N - 1) // 2, 2**255, 2**128 + 1] + [rng.randrange(1, N) for _ in range(4000)]
    ws = np.array([to_words(x, 0) for x in xs], dtype=np.uint32)
    out = ver.debug_op(27, ws)
    for i, x in enumerate(xs):
        assert from_words(out[i]) == pow(x, -1, N), hex(x)


def test_glv_split(ver):
    rng = random.Random(17)
    ks = [0, 1, 2, N - 1, N - 2, N // 2, R.LAMBDA, 2**128, 2**128 - 1] + [rng.randrange(N) for _ in range(4000)]
    out = run_op(ver, 9, [(k, 0) for k in ks])
    for k, o in zip(ks, out):
        k1 = from_words(o, 0, 4) * (-1 if o[8] else 1)
        k2 = from_words(o, 4, 4) * (-1 if o[9] else 1)
        assert (k1 + k2 * R.LAMBDA - k) % N == 0, hex(k)
        assert abs(k1) < 2**128 and abs(k2) < 2**128


def test_batch_inversion_across_wave(ver):
    rng = random.Random(19)
    xs = [rng.randrange(1, N) for _ in range(1000)] + [1, N - 1]
    out = run_op(ver, 10, [(x, 0) for x in xs])
    for x, o in zip(xs, out):
        assert from_words(o) == pow(x, N - 2, N)


def test_point_double(ver):
    pts = [R.point_mul(k, R.G) for k in (1, 2, 3, 12345, N - 1, R.LAMBDA)]
    out = run_op(ver, 11, [(p[0], p[1]) for p in pts])
    for p, o in zip(pts, out):
        q = R.point_add(p, p)
        assert from_words(o, 0) == q[0] and from_words(o, 8) == q[1]


# ------------------------------------------------------------ full verification
# Four schedules compute every verdict: the throughput pipeline
# (gv_kernels.hip, one lane per signature), the small-batch kernels on the
# limb-sliced field layer (one signature per block, one field element per
# 16-lane row: k_verify_lat_sl, and k_verify_lat_sl4 whose ladder waves keep
# one accumulator in four rows, G from the 24-bit tables -- the default up to
# "lat_rows_max") and the one-lane-field small-batch kernel (k_verify_lat:
# four lanes per signature); "lat_max", "lat_sliced" and "lat_rows_max" pick
# one per call.
PATHS = {"throughput": (0, 1, 0), "latency": (1 << 30, 1, 0), "latency_rows": (1 << 30, 1, 1 << 30),
         "latency_onelane": (1 << 30, 0, 0)}  # (lat_max, sliced, rows)


@pytest.fixture(params=sorted(PATHS))
def path(request, ver):
    lat_max, sliced, rows = PATHS[request.param]
    ver.set_option("lat_max", lat_max)
    ver.set_option("lat_sliced", sliced)
    ver.set_option("lat_sl_max", 1 << 30)
    ver.set_option("lat_rows_max", rows)
    yield request.param
    ver.reset_schedule()
    ver.set_option("lat_sliced", 1)


def test_golden_digest_vectors(ver, path):
    pub, sig, dig, ok, cats = load_digest_vectors()
    got = ver.verify_batch_digests(pub, sig, dig)
    bad = [(i, cats[i], int(ok[i])) for i in range(len(ok)) if got[i] != ok[i]]
    assert not bad, bad[:20]


def test_golden_message_vectors(ver, path):
    pub, sig, msgs, ok, cats = load_msg_vectors()
    got = ver.verify_batch_msgs(pub, sig, msgs)
    bad = [(i, cats[i], int(ok[i])) for i in range(len(ok)) if got[i] != ok[i]]
    assert not bad, bad[:20]


def make_random_batch(n, seed, adversarial=0.25, nkeys=257):
    rng = np.random.default_rng(seed)
    privs = rng.integers(0, 256, size=(nkeys, 32), dtype=np.uint8)
    privs[:, 0] &= 0x7F
    privs[:, 31] |= 1
    pubs = O.pubkey_batch(privs, threads=8)
    kidx = np.arange(n) % nkeys
    dig = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sig = O.sign_batch(np.ascontiguousarray(privs[kidx]), dig, threads=8)
    pub = np.ascontiguousarray(pubs[kidx])
    m = rng.random(n) < adversarial
    kinds = rng.integers(0, 6, size=n)
    for i in np.nonzero(m)[0]:
        k = kinds[i]
        if k == 0:        # high-S
            s = int.from_bytes(bytes(sig[i, 32:]), "big")
            sig[i, 32:] = np.frombuffer((N - s).to_bytes(32, "big"), np.uint8)
        elif k == 1:      # r out of range
            sig[i, :32] = np.frombuffer((N + int(rng.integers(0, 1000))).to_bytes(32, "big"), np.uint8)
        elif k == 2:      # s zero / huge
            sig[i, 32:] = 0 if rng.random() < 0.5 else 0xFF
        elif k == 3:      # off-curve / random x
            pub[i, 1:] = rng.integers(0, 256, size=32, dtype=np.uint8)
        elif k == 4:      # malformed prefix
            pub[i, 0] = rng.choice([0, 1, 4, 5, 6, 7, 0xFF])
        else:             # wrong message
            dig[i, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return pub, sig, dig


def test_random_adversarial_batch_vs_oracle(ver, path):
    pub, sig, dig = make_random_batch(20000, seed=0xC3)
    want = O.verify_digests(pub, sig, dig, threads=16)
    got = ver.verify_batch_digests(pub, sig, dig)
    assert 0.6 < want.mean() < 0.9
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:20]


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1000])
def test_ragged_sizes_and_bitmap(ver, n, path):
    pub, sig, dig = make_random_batch(n, seed=n, adversarial=0.3, nkeys=7)
    want = O.verify_digests(pub, sig, dig, threads=8)
    assert np.array_equal(ver.verify_batch_digests(pub, sig, dig), want)
    bits = ver.verify_batch_digests_bits(pub, sig, dig)
    unpacked = np.array([(int(bits[i // 64]) >> (i % 64)) & 1 for i in range(n)], dtype=np.uint8)
    assert np.array_equal(unpacked, want)
    tail = int(bits[-1]) >> (n % 64) if n % 64 else 0
    assert tail == 0


def test_empty_batch(ver):
    z = np.zeros((0, 33), np.uint8)
    assert ver.verify_batch_digests(z, np.zeros((0, 64), np.uint8), np.zeros((0, 32), np.uint8)).size == 0


def test_chunked_batches(ver):
    pub, sig, dig = make_random_batch(3000, seed=5, adversarial=0.2, nkeys=11)
    want = O.verify_digests(pub, sig, dig, threads=8)
    ver.set_option("max_batch", 512)
    try:
        assert np.array_equal(ver.verify_batch_digests(pub, sig, dig), want)
    finally:
        ver.set_option("max_batch", 1 << 20)


def test_message_path_random(ver):
    rng = random.Random(23)
    msgs, pubs, sigs, want = [], [], [], []
    for i in range(600):
        d = rng.randrange(1, N)
        msg = rng.randbytes(rng.randrange(0, 700))
        sig = bytearray(R.sign(d, msg)) if i < 40 else None
        if sig is None:
            priv = d.to_bytes(32, "big")
            sig = bytearray(O.sign(priv, O.sha256(msg)))
        if i % 5 == 0:
            msg = msg + b"!"
        pub = O.pubkey(d.to_bytes(32, "big"))
        msgs.append(msg)
        pubs.append(np.frombuffer(pub, np.uint8))
        sigs.append(np.frombuffer(bytes(sig), np.uint8))
        want.append(O.verify_bytes(pub, msg, bytes(sig)))
    got = ver.verify_batch_msgs(np.array(pubs), np.array(sigs), msgs)
    assert np.array_equal(got, np.array(want, dtype=np.uint8))


def test_fault_injection_fails_closed(ver):
    pub, sig, dig = make_random_batch(8, seed=1, nkeys=2)
    ver.set_option("fault_inject", 1)
    try:
        with pytest.raises(gvm.GpuVerifyError) as ei:
            ver.verify_batch_digests(pub, sig, dig)
        assert ei.value.code == gvm.GV_EFAULT
    finally:
        ver.set_option("fault_inject", 0)


def test_device_resident_path(ver):
    pub, sig, dig = make_random_batch(5000, seed=9, adversarial=0.25, nkeys=31)
    want = O.verify_digests(pub, sig, dig, threads=16)
    n = 5000
    bufs = {k: ver.dev_alloc(a.nbytes) for k, a in (("pub", pub), ("sig", sig), ("dig", dig))}
    d_bits = ver.dev_alloc(((n + 63) // 64) * 8)
    try:
        ver.dev_upload(bufs["pub"], pub)
        ver.dev_upload(bufs["sig"], sig)
        ver.dev_upload(bufs["dig"], dig)
        ver.set_option("time_kernels", 1)
        for _ in range(3):
            ver.dev_verify_digests(0, n, bufs["pub"], bufs["sig"], bufs["dig"], d_bits)
        cnt, a, b, c = ver.stage_stats()
        assert cnt == 3 and c > 0 and b > 0
        bits = np.zeros((n + 63) // 64, dtype=np.uint64)
        ver.dev_download(bits, d_bits)
    finally:
        ver.set_option("time_kernels", 0)
        for p in list(bufs.values()) + [d_bits]:
            ver.dev_free(p)
    got = np.array([(int(bits[i // 64]) >> (i % 64)) & 1 for i in range(n)], dtype=np.uint8)
    assert np.array_equal(got, want)


def test_pubkey_class_mirror():
    d = 0xC0FFEE
    msg = b'{"account_number":"1"}'
    sig = R.sign(d, msg)
    pk = gvm.PubKeySecp256k1(R.pubkey(d))
    assert pk.verify_bytes(msg, sig) is True
    assert pk.verify_bytes(msg + b" ", sig) is False
    assert pk.verify_bytes(msg, sig[:63]) is False


def test_multi_device_split_and_gather():
    """gv_open with two device slots (here: the same GPU twice) exercises the
    host-side slicing, per-device worker threads and bitmap gather."""
    pub, sig, dig = make_random_batch(3001, seed=77, adversarial=0.25, nkeys=13)
    want = O.verify_digests(pub, sig, dig, threads=16)
    with gvm.Verifier([0, 0]) as v2:
        assert v2.num_devices == 2
        assert np.array_equal(v2.verify_batch_digests(pub, sig, dig), want)
        bits = v2.verify_batch_digests_bits(pub, sig, dig)
        assert np.array_equal(np.unpackbits(bits.view(np.uint8), bitorder="little")[:3001], want)


def test_overlapping_device_calls_on_separate_streams(ver):
    """gv_dev_* calls on two caller streams, then a host-buffer call, issued
    back to back with no host sync: every use of the device scratch is ordered
    after the previous one (gv_runtime.cpp set_acquire/set_release), so no call
    overwrites the inputs of kernels still in flight."""
    s1, s2 = ver.stream_create(), ver.stream_create()
    batches = [make_random_batch(60000, seed=300 + k, adversarial=0.3, nkeys=97) for k in range(2)]
    wants = [O.verify_digests(*b, threads=16) for b in batches]
    bufs = []
    for pub, sig, dig in batches:
        d = [ver.dev_alloc(a.nbytes) for a in (pub, sig, dig)]
        for p, a in zip(d, (pub, sig, dig)):
            ver.dev_upload(p, a)
        bufs.append(d + [ver.dev_alloc(((len(pub) + 63) // 64) * 8)])
    try:
        for (pub, _, _), d, st in zip(batches, bufs, (s1, s2)):
            ver.dev_verify_digests(0, len(pub), d[0], d[1], d[2], d[3], stream=st)
        pub3, sig3, dig3 = make_random_batch(3000, seed=399, adversarial=0.3, nkeys=5)
        got3 = ver.verify_batch_digests(pub3, sig3, dig3)
        ver.stream_sync(s1)
        ver.stream_sync(s2)
        assert np.array_equal(got3, O.verify_digests(pub3, sig3, dig3, threads=8))
        for (pub, _, _), d, want in zip(batches, bufs, wants):
            bits = np.zeros((len(pub) + 63) // 64, dtype=np.uint64)
            ver.dev_download(bits, d[3])
            assert np.array_equal(np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(pub)], want)
    finally:
        for d in bufs:
            for p in d:
                ver.dev_free(p)
        ver.stream_destroy(s1)
        ver.stream_destroy(s2)


@pytest.mark.parametrize("chunk,growth,stage", [(256, 1, 8), (256, 3, 3), (4096, 4, 8), (0, 4, 1)])
def test_host_pipeline_chunking(ver, chunk, growth, stage):
    """The two-stream host pipeline (pinned staging, chunks alternating between
    two scratch sets, ramped chunk sizes) over ragged chunk boundaries, digests
    and messages, with several staging-thread counts."""
    pub, sig, dig = make_random_batch(10007, seed=chunk + 1, adversarial=0.25, nkeys=29)
    want = O.verify_digests(pub, sig, dig, threads=16)
    ver.set_option("pipe_chunk", chunk)
    ver.set_option("pipe_growth", growth)
    ver.set_option("stage_threads", stage)
    try:
        assert np.array_equal(ver.verify_batch_digests(pub, sig, dig), want)
        bits = ver.verify_batch_digests_bits(pub, sig, dig)
        assert np.array_equal(np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(want)], want)
        rng = random.Random(chunk)
        msgs = [rng.randbytes(rng.randrange(0, 300)) for _ in range(5000)]
        mdig = np.array([np.frombuffer(O.sha256(m), np.uint8) for m in msgs])
        privs = np.array([np.frombuffer(rng.randrange(1, N).to_bytes(32, "big"), np.uint8) for _ in range(5000)])
        mpub = O.pubkey_batch(privs, threads=8)
        msig = O.sign_batch(privs, mdig, threads=8)
        msgs = [m + b"x" if i % 7 == 0 else m for i, m in enumerate(msgs)]
        mwant = np.array([i % 7 != 0 for i in range(5000)], np.uint8)
        assert np.array_equal(ver.verify_batch_msgs(mpub, msig, msgs), mwant)
    finally:
        ver.set_option("pipe_chunk", 131072)
        ver.set_option("pipe_growth", 4)
        ver.set_option("stage_threads", 8)


def test_option_bounds(ver):
    for key, val in (("max_batch", 1 << 32), ("max_batch", 255), ("lat_max", -1), ("lat_max", 1 << 33),
                     ("pipe_chunk", 100), ("pipe_growth", 0), ("stage_threads", 0), ("no_such_option", 1)):
        with pytest.raises(gvm.GpuVerifyError):
            ver.set_option(key, val)


def test_sliced_latency_kernels_at_scale(ver):
    """k_verify_lat_sl and k_verify_lat_sl4 (pub33) and k_verify_lat16_sl (keyed) far past their
    production batch size: 262,144 mixed signatures (25 % invalid over the
    generator's six classes, 4,096 keys) forced through the small-batch
    schedule, against the verdicts the generator constructed, and a sample
    against the C oracle."""
    import bench
    pub, sig, dig, exp = bench.make_digest_workload(262144, 0x5A, 4096, 0.25, 16)
    assert 0.70 < exp.mean() < 0.80
    want = O.verify_digests(pub[:4000], sig[:4000], dig[:4000], threads=16)
    assert np.array_equal(want, exp[:4000])
    uniq, inv = np.unique(pub, axis=0, return_inverse=True)
    ver.set_option("lat_max", 1 << 30)
    ver.set_option("lat_sl_max", 1 << 30)
    try:
        for rows in (0, 1 << 30):                            # k_verify_lat_sl, k_verify_lat_sl4
            ver.set_option("lat_rows_max", rows)
            got = ver.verify_batch_digests(pub, sig, dig)
            bad = np.nonzero(got != exp)[0]
            assert bad.size == 0, (rows, bad[:20])
        slots = ver.keys_load(uniq)[inv.reshape(-1)]
        got = ver.verify_batch_digests_keyed(slots, sig, dig)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, bad[:20]
    finally:
        ver.reset_schedule()
        ver.keys_reset()


@pytest.mark.parametrize("zc", [0, 1])
def test_small_batches_zero_copy_and_staged(ver, zc):
    """Host-buffer small batches on the sliced kernels, zero-copy (the kernel
    reads the pinned staging buffer, verdict bytes in pinned memory) and staged
    (H2D + bitmap + D2H): same verdicts, byte and bitmap entry points, pub33
    and keyed."""
    pub, sig, dig = make_random_batch(700, seed=0x2C + zc, adversarial=0.3, nkeys=9)
    want = O.verify_digests(pub, sig, dig, threads=8)
    ver.set_option("lat_zero_copy", zc)
    try:
        assert np.array_equal(ver.verify_batch_digests(pub, sig, dig), want)
        bits = ver.verify_batch_digests_bits(pub, sig, dig)
        assert np.array_equal(np.unpackbits(bits.view(np.uint8), bitorder="little")[:700], want)
        assert (int(bits[-1]) >> (700 % 64)) == 0
        uniq, inv = np.unique(pub, axis=0, return_inverse=True)
        slots = ver.keys_load(uniq)[inv.reshape(-1)]
        assert np.array_equal(ver.verify_batch_digests_keyed(slots, sig, dig), want)
    finally:
        ver.set_option("lat_zero_copy", 1)
        ver.keys_reset()


@pytest.mark.parametrize("zc", [0, 1])
def test_message_lengths_at_block_and_chunk_edges(ver, zc):
    """The sliced kernels hash the sign bytes themselves (sha256_msg_wave:
    256-byte chunks, one word per lane, the next chunk prefetched): every
    padding edge (55/56/63/64 mod 64) and chunk edge (multiples of 256, and
    the 4-block boundary the padding can spill over), empty and long
    messages, pub33 and keyed, zero-copy and staged, against the oracle."""
    rng = random.Random(0x5A + zc)
    lens = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 183, 184, 191, 192, 247, 248, 255, 256, 257,
            311, 312, 319, 320, 503, 504, 511, 512, 513, 1015, 1016, 1023, 1024, 1025, 2048, 4000]
    msgs, pubs, sigs, want = [], [], [], []
    for i, L in enumerate(lens * 2):
        d = rng.randrange(1, N)
        msg = rng.randbytes(L)
        priv = d.to_bytes(32, "big")
        sig = bytearray(O.sign(priv, O.sha256(msg)))
        if i >= len(lens):                      # second copy: one flipped message bit
            msg = bytes(msg[:-1]) + bytes([msg[-1] ^ 1]) if L else b"\x00"
        pub = O.pubkey(priv)
        msgs.append(msg)
        pubs.append(np.frombuffer(pub, np.uint8))
        sigs.append(np.frombuffer(bytes(sig), np.uint8))
        want.append(O.verify_bytes(pub, msg, bytes(sig)))
    pubs, sigs, want = np.array(pubs), np.array(sigs), np.array(want, dtype=np.uint8)
    assert want[:len(lens)].all() and not want[len(lens):].any()
    ver.set_option("lat_zero_copy", zc)
    try:
        assert np.array_equal(ver.verify_batch_msgs(pubs, sigs, msgs), want)
        slots = ver.keys_load(pubs)
        assert np.array_equal(ver.verify_batch_msgs_keyed(slots, sigs, msgs), want)
    finally:
        ver.set_option("lat_zero_copy", 1)
        ver.keys_reset()
